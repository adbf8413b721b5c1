"""Multi-GPU plan on CPU: world_size 2 over gloo (no GPU).

Utterances shard contiguously over ranks with no data-path collective; each
rank's inputs are generated per utterance so shards reproduce the full batch;
the host gathers the hypotheses to rank 0.  The ranks here run bench.py's own
shard plan (shard_range, uneven splits included), record packing, gather
(gather_hypotheses over gloo), merge/count check and digest, with the CPU
oracle standing in for each rank's decoder; plus bench.py's max-over-ranks
timing reduce.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, oracle

T, V, BEAM = 30, 12, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _decode_arrays(emis):
    """(labels [B][T], lengths [B], logp [B]) of the best hypotheses, in the
    array form CTCDecoder.best_arrays() hands bench.py."""
    Tn, B, _ = emis.shape
    best = oracle.decode(emis, BEAM, 0, max_hyps=1)
    lab = np.zeros((B, Tn), np.int32)
    ln = np.zeros(B, np.int32)
    lp = np.zeros(B, np.float64)
    for b, ((l, p),) in enumerate(best):
        lab[b, :len(l)] = l
        ln[b] = len(l)
        lp[b] = p
    return lab, ln, lp


def _worker(rank, world, port, global_batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench   # the product's shard plan, gather, merge and digest
    first, count = bench.shard_range(rank, world, global_batch)
    emis = oracle.synthetic_emissions(T, count, V, first=first)
    lab, ln, lp = _decode_arrays(emis)
    records = bench.gather_hypotheses(bench.pack_hypotheses(first, lab, ln, lp), world, rank)
    slowest = bench.reduce_max_over_ranks(float(rank + 1), world)
    dist.barrier()
    if rank == 0:
        hyps, lps = bench.merge_records(records)
        q.put((hyps, lps.tolist(), bench.hyp_digest(hyps, lps), slowest))
    else:
        assert records is None
    dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [6, 7])   # even and uneven splits
def test_two_rank_shard_gather_equals_single_process(global_batch):
    sys.path.insert(0, str(ROOT))
    import bench
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, global_batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    hyps, lps, digest, slowest = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(hyps) == global_batch
    lab, ln, lp = _decode_arrays(oracle.synthetic_emissions(T, global_batch, V))
    rec = bench.pack_hypotheses(0, lab, ln, lp)
    assert hyps == rec[1]
    assert lps == rec[2]
    assert digest == bench.hyp_digest(rec[1], np.asarray(rec[2]))
    assert slowest == float(world)


def test_shard_range_covers_batch():
    sys.path.insert(0, str(ROOT))
    import bench
    for gb in (1, 7, 64, 2048, 2049):
        for world in (1, 2, 3, 8):
            spans = [bench.shard_range(r, world, gb) for r in range(world)]
            nxt = 0
            for first, count in spans:
                assert first == nxt and count >= 0
                nxt += count
            assert nxt == gb
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_merge_records_rejects_gaps():
    sys.path.insert(0, str(ROOT))
    import bench
    with pytest.raises(AssertionError):
        bench.merge_records([(0, [[1]], [0.0]), (2, [[2]], [0.0])])


def _run_bench(args, env_extra=None, timeout=300):
    """bench.py as the driver starts it (`python bench.py --gpus N ...`), in a
    fresh process without rank variables in its environment."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, cwd="/tmp",
                       capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("n,extra,gb", [(2, ["--config", "C2", "--T", "40"], 128),    # weak: 64 per rank
                                        (2, ["--global-batch", "7", "--T", "30"], 7),   # strong, uneven
                                        (8, ["--T", "60"], 2048)])                      # C4 default, 8 ranks
def test_bench_self_launches_ranks(n, extra, gb):
    """`bench.py --gpus N` with no WORLD_SIZE starts N rank processes itself
    (gloo rendezvous on 127.0.0.1), shards, gathers to rank 0 and checks the
    gathered batch against one process (--dry-run-cpu: no GPU, a host greedy
    decode stands in for the GPU path)."""
    rc, line, err = _run_bench(["--gpus", str(n), "--dry-run-cpu"] + extra)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == n
    assert line["gather"]["utterances"] == gb
    assert line["gather"]["verified_vs_1process"] is True


def test_bench_rejects_world_size_mismatch():
    rc, line, err = _run_bench(["--gpus", "3", "--dry-run-cpu"], env_extra={"WORLD_SIZE": "2"})
    assert rc != 0 and line is None
    assert "does not match --gpus 3" in err

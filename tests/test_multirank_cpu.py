"""Multi-GPU plan on CPU: world_size 2 over gloo (no GPU).

Utterances shard contiguously over ranks with no data-path collective; each
rank's inputs are generated per utterance so shards reproduce the full batch;
the host gathers the hypotheses.  Checked here with the CPU oracle standing
in for each rank's decoder, plus bench.py's max-over-ranks timing reduce.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, oracle

T, B_PER, V, BEAM = 30, 3, 12, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench   # bench.py: shard plan + timing reduce
    first = bench.shard_first(rank, B_PER)
    emis = oracle.synthetic_emissions(T, B_PER, V, first=first)
    mine = oracle.decode(emis, BEAM, 0, max_hyps=1)
    best = [(lab, lp) for ((lab, lp),) in mine]
    gathered = [None] * world
    dist.all_gather_object(gathered, best)          # host-side gather of hypotheses
    slowest = bench.reduce_max_over_ranks(float(rank + 1), world)
    dist.barrier()
    if rank == 0:
        q.put(([h for part in gathered for h in part], slowest))
    dist.destroy_process_group()


def test_two_rank_shard_gather_equals_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    import sys
    sys.path.insert(0, str(ROOT))
    for p in procs:
        p.start()
    hyps, slowest = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = oracle.decode(oracle.synthetic_emissions(T, B_PER * world, V), BEAM, 0, max_hyps=1)
    assert hyps == [(lab, lp) for ((lab, lp),) in full]
    assert slowest == float(world)

"""Benchmark: frames/sec decoded (RNN + CTC beam) on 1..8 MI355X.

One step = one pass of the hot path over one batch of synthetic input that is
already resident in HBM:
    RNN forward (hoisted x.W_ih GEMM + recurrence, H=256)
    -> Linear H->V with fused bias + log_softmax (emissions, time-major)
    -> CTC prefix beam search (beam=50, V=29) -> best-path traceback
    -> best label sequences and log-probs copied to the host.
Steps are pipelined by default (--no-pipeline: strictly sequential): the RNN
and emission projection of batch i+1 run on one HIP stream while batch i is
decoded on another (double-buffered emissions, event-ordered), so the 64
recurrence workgroups and the 64 decoder workgroups share the 256 CUs; the
results of batch i come back in one copy of a packed buffer behind its decode
(an event wait).
Every step still does all of its work inside the timed region.
Default workload = BASELINE.json configs[1] (C2): B=64 utterances per GPU,
T=500 frames, hidden 256, vocab 29, beam 50.  Multi-GPU: one process per GPU
(torch.distributed.run); each rank decodes its own 64 utterances (weak
scaling, no collective on the data path: utterances are independent); the
gloo group only carries the timing barrier and the max-over-ranks reduce.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--decode-only]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")

METRIC = "frames/sec decoded (RNN+CTC beam) at beam=50, vocab=29; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def shard_first(rank: int, per_rank: int) -> int:
    """Global index of rank's first utterance (contiguous shards)."""
    return rank * per_rank


def reduce_max_over_ranks(x: float, world: int) -> float:
    """Max of x over ranks (the job ends when the slowest rank ends)."""
    if world <= 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def algorithmic_bytes_per_frame(V: int, beam: int) -> int:
    """4V (emission row, fp32, read once) + 32K (16-B beam
    record read + written) + 8K (8-B traceback record), K = beam + 1."""
    K = beam + 1
    return 4 * V + 40 * K


def make_inputs(T, B, In, H, V, first, seed=20261015):
    """Synthetic features and random-init weights (no datasets/checkpoints)."""
    rng_w = np.random.default_rng(seed)
    s = 1.0 / np.sqrt(H)
    w_ih = rng_w.uniform(-s, s, (In, H)).astype(np.float32)
    w_hh = rng_w.uniform(-s, s, (H, H)).astype(np.float32)
    b_ih = rng_w.uniform(-0.1, 0.1, H).astype(np.float32)
    b_hh = rng_w.uniform(-0.1, 0.1, H).astype(np.float32)
    w_out = rng_w.uniform(-4 * s, 4 * s, (H, V)).astype(np.float32)
    b_out = rng_w.uniform(-0.5, 0.5, V).astype(np.float32)
    x = np.empty((T, B, In), np.float32)
    for b in range(B):   # per-utterance stream: shard-invariant inputs
        x[:, b, :] = np.random.default_rng(seed + 1 + first + b).uniform(-1, 1, (T, In))
    return x.reshape(T * B, In), (w_ih, w_hh, b_ih, b_hh), (w_out, b_out)


def load_traffic(kernel: str):
    """Measured HBM bytes per launch of `kernel` (rocprofv3 FETCH_SIZE +
    WRITE_SIZE passes, summarised by tools/traffic_from_pmc.py into the
    committed profiles/traffic.json); None when not profiled."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())[kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="utterances per GPU")
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=29)
    ap.add_argument("--beam", type=int, default=50)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--decode-only", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run RNN and decode of each step back to back on one stream")
    ap.add_argument("--overlap-results", action="store_true",
                    help="queue batch i+1's decode before reading batch i's results "
                         "(measured slower on MI355X: see DESIGN.md §9)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; more ranks than GPUs (a rehearsal on a smaller box)
    # wrap around.  device_count() does not initialise the GPU.
    ndev = torch.cuda.device_count() if torch is not None else 1
    local = local % max(1, ndev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    asr.set_device(local)

    T, B, H, V, beam = args.T, args.batch, args.hidden, args.vocab, args.beam
    cname = {(500, 64, 256, 29, 50): "C2", (2000, 32, 1024, 1000, 200): "C5 (32 utterances/GPU)"}.get(
        (T, B, H, V, beam), "custom")
    In = H
    first = shard_first(rank, B)
    x, (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = make_inputs(T, B, In, H, V, first)
    DM = asr.DeviceMatrix.from_numpy
    d_x, d_wih, d_whh = DM(x), DM(w_ih), DM(w_hh)
    d_bih, d_bhh = DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1))
    d_wout, d_bout = DM(w_out), DM(b_out.reshape(V, 1))
    pipeline = not args.no_pipeline and not args.decode_only
    nbuf = 2 if pipeline else 1
    d_hid = [asr.DeviceMatrix(T * B, H) for _ in range(nbuf)]
    d_emis = [asr.DeviceMatrix(T * B, V) for _ in range(nbuf)]
    # one decoder handle per buffer (with --overlap-results the results of batch
    # i are read after batch i+1's decode is already queued behind it)
    decs = [asr.CTCDecoder(V, beam, 0, waves=args.waves) for _ in range(nbuf)]
    dec = decs[0]
    if pipeline:   # HIP streams/events via torch (same HIP runtime as libasr_amd)
        torch.cuda.set_device(local)
        s_prod, s_dec = torch.cuda.Stream(), torch.cuda.Stream()
        ev_ready = [torch.cuda.Event() for _ in range(nbuf)]
        ev_free = [torch.cuda.Event() for _ in range(nbuf)]
        prod_stream, dec_stream = s_prod.cuda_stream, s_dec.cuda_stream
    else:
        prod_stream = dec_stream = 0

    def produce(k):
        """RNN forward + emission projection of a batch into buffer k."""
        asr.rnn_fwd(d_x, d_wih, d_whh, d_bih, d_bhh, d_hid[k], T, B, stream=prod_stream)
        asr.linear_fwd(d_hid[k], d_wout, d_bout, d_emis[k], asr.EPI_BIAS_LOGSOFTMAX, prod_stream)

    if args.decode_only:   # emissions computed once, outside the timed region
        produce(0)
        asr.synchronize()

    kernel_ms = []

    def enqueue(k):
        """Decode buffer k and its traceback; the results follow to pinned host memory."""
        decs[k].decode_device(d_emis[k].ptr, T, B, is_log=True, stream=dec_stream)

    def collect(k):
        """Wait for buffer k's results (an event, not the stream) and read them."""
        labels, lens, lp = decs[k].best_arrays()
        kernel_ms.append(decs[k].last_kernel_ms())
        return labels, lp

    def consume(k):
        enqueue(k)
        return collect(k)

    def run(n):
        """n steps; every step's RNN, projection, decode and result copy."""
        out = None
        if not pipeline:
            for _ in range(n):
                if not args.decode_only:
                    produce(0)
                out = consume(0)
            return out
        with torch.cuda.stream(s_prod):
            produce(0)
            ev_ready[0].record(s_prod)
        prev = None
        for i in range(n):
            k = i % 2
            if i + 1 < n:   # batch i+1 is produced while batch i is decoded
                kn = (i + 1) % 2
                s_prod.wait_event(ev_free[kn])
                produce(kn)
                ev_ready[kn].record(s_prod)
            s_dec.wait_event(ev_ready[k])
            enqueue(k)
            ev_free[k].record(s_dec)
            if not args.overlap_results:
                out = collect(k)
                continue
            if prev is not None:   # batch i-1's results, while batch i decodes
                out = collect(prev)
            prev = k
        return out if prev is None else collect(prev)

    run(args.warmup)
    kernel_ms.clear()
    if world > 1:
        dist.barrier()
    asr.synchronize()
    t0 = time.perf_counter()
    labels, lp = run(args.steps)
    asr.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = reduce_max_over_ranks(elapsed, world)
    if world > 1:
        dist.barrier()

    frames = world * B * T * args.steps
    value = frames / elapsed
    avg_kernel_ms = float(np.mean(kernel_ms)) if kernel_ms else None
    bpf = algorithmic_bytes_per_frame(V, beam)
    roof = None
    if avg_kernel_ms:
        achieved = bpf * B * T / (avg_kernel_ms * 1e-3) / 1e9
        roof = {"kernel": "ctc_beam_kernel", "bound": "hbm", "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "avg_launch_ms": round(avg_kernel_ms, 4), "bytes_per_frame": bpf,
                "frames_per_launch": B * T, "traffic": load_traffic("ctc_beam_kernel")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        oracle = _load("ctc_oracle", ROOT / "oracle" / "ctc_oracle.py")
        threads = max(1, min(16, os.cpu_count() or 1))
        S = min(B, 2 * threads)
        # bounded sample: ~4e7 candidate expansions (all T at C2; a prefix of
        # the same frames when K*V is large, e.g. C5)
        Ts = min(T, max(4, int(4.0e7 / (S * (beam + 1) * (V + 1)))))
        emis = d_emis[0].toCpu().reshape(T, B, V)[:Ts, :S, :].copy()
        secs = oracle.time_decode(emis, beam, 0, is_log=True, nthreads=threads)
        cpu = {"value": round(S * Ts / secs, 1), "unit": "frames/s", "cores": threads,
               "kind": "port",
               "sample": f"oracle/ctc_oracle.cpp decode of the first {S} utterances x {Ts} frames of this "
                         f"run's emissions (beam={beam}, V={V}), {threads} std::threads, {secs:.2f} s wall; "
                         "decoder only (the reference has no CPU RNN)"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (RNN/Linear MFMA) + f64 (beam scores)",
            "data": "synthetic (U(-1,1) features, random-init weights)",
            "config": {"workload": (cname + (" decode-only" if args.decode_only else " RNN+Linear+CTC")) +
                       f": B={B}/GPU, T={T}, hidden={H}, vocab={V}, beam={beam}",
                       "batch_per_gpu": B, "global_batch": B * world, "T": T, "hidden": H,
                       "vocab": V, "beam": beam, "parallelism": f"utterance-shard x{world}",
                       "pipeline": ("RNN+projection of batch i+1 on one HIP stream || decode of batch i "
                                    "on another" if pipeline else "none (sequential)")},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    for d in decs:
        d.close()


if __name__ == "__main__":
    main()

"""Benchmark: frames/sec decoded (RNN + CTC beam) on 1..8 MI355X.

One step = one pass of the hot path over one batch of synthetic input that is
already resident in HBM:
    RNN forward (hoisted x.W_ih GEMM + recurrence, H=256)
    -> Linear H->V with fused bias + log_softmax (emissions, time-major)
    -> CTC prefix beam search (beam=50, V=29) -> best-path traceback
    -> best label sequences and log-probs copied to the host.
Steps are pipelined by default (--no-pipeline: strictly sequential): the RNN
and emission projection of batch i+1 run on one HIP stream while batch i is
decoded on another (event-ordered emission buffers), and up to D batches
decode at once when one batch leaves most CUs idle (--inflight D; auto: D = 3
when a batch needs at most a quarter of the CUs at one decode workgroup per
utterance and H <= 256, as at C2; D = 2 at C5), batch i on decode stream
i % D, each stream restricted to its own group of CUs and the production
stream to the rest (hipExtStreamCreateWithCUMask).  One utterance is still
decoded by one workgroup frame after frame.  The results of batch i come back
in one copy of a packed buffer behind its decode (an event wait), read on the
host once the D-1 younger batches are queued.  Every step does all of its work
inside the timed region.

Default workload = BASELINE.json configs[3] (C4), the configuration the
metric's 1/2/4/8-GPU line is quoted on: 2048 utterances in all, split over the
GPUs (strong scaling), T=1000 frames, hidden 256, vocab 29, beam 50 (also
north_star's >= 10x target shape).  --config C2/C3/C5/BL select the other
configurations (parity-test cases and extra lines, not the headline).

Multi-GPU: one process per GPU.  `python bench.py --gpus N` with no
WORLD_SIZE in the environment starts N fresh rank processes itself (this
parent never touches the GPU and never execs; it exits with the first
failing rank's status); under torch.distributed.run the ranks come from the
environment and WORLD_SIZE must equal --gpus.  Rank r decodes the contiguous
utterance range shard_range(r) with no collective on the data path
(utterances are independent).  After the timed region every
rank's hypotheses (labels, fp64 log-prob) are gathered to rank 0 over gloo
(the host-side gather of north_star), counted against the global batch, and
checked bit for bit against a 1-GPU decode of the same utterance ids on rank
0's device.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C4]
                    [--global-batch G | --batch B] [--decode-only] [--no-pipeline]
"""
import argparse
import collections
import ctypes
import gc
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

# Hardware queues: HIP maps the UNMASKED streams of a process round-robin
# onto GPU_MAX_HW_QUEUES queues (default 4, read when the runtime starts);
# the pipeline's CU-masked decode and production streams get queues of
# their own, so the bench runs at whatever the environment sets — HIP's
# default unless exported (round 6: the same frames/s at 4 and 24 queues,
# DESIGN.md §11).  --hw-queues N (read here, before the HIP runtime starts)
# measures another count.
_hwq = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--hw-queues=")), None)
if _hwq is None and "--hw-queues" in sys.argv[:-1]:
    _hwq = sys.argv[sys.argv.index("--hw-queues") + 1]
if _hwq is not None:
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(_hwq))

# c10's INFO lines (gloo's "[Gloo] Rank r is connected to n peer ranks") can
# land on stdout before rank 0's JSON line: keep stdout to that one line.
# Read when torch is imported, so set here, before the import.
os.environ.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402

METRIC = "frames/sec decoded (RNN+CTC beam) at beam=50, vocab=29; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3  # dense fp32 MFMA = fp32 vector peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TF = 2516.6  # dense bf16 MFMA: 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz (~2.5 PF)
SPLIT_PRODUCTS = 6          # bf16 MFMA products per fp32 product on the split arithmetic (dense_x3.hip)

# BASELINE.json configs: T, utterances per GPU, hidden, vocab, beam.
CONFIGS = {
    "C2": dict(T=500, batch=64, hidden=256, vocab=29, beam=50),
    "C3": dict(T=1000, batch=256, hidden=256, vocab=29, beam=100),
    "C4": dict(T=1000, batch=256, hidden=256, vocab=29, beam=50, global_batch=2048),
    "C5": dict(T=2000, batch=32, hidden=1024, vocab=1000, beam=200),
    # the reference's own Python-harness workload, baseline/config.json:1-28
    # (seg_len 200, batch 256, rnn_hidden_size 2048, vocab 46 + blank, beam 100)
    "BL": dict(T=200, batch=256, hidden=2048, vocab=47, beam=100),
}


# ------------------------------------------------------------------ sharding
def shard_range(rank: int, world: int, global_batch: int):
    """Contiguous utterance range [first, first + count) of `rank` when
    `global_batch` utterances are split over `world` ranks (the first
    global_batch % world ranks take one more)."""
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def shard_first(rank: int, per_rank: int) -> int:
    """Global index of rank's first utterance under weak scaling."""
    return rank * per_rank


def reduce_max_over_ranks(x: float, world: int) -> float:
    """Max of x over ranks (the job ends when the slowest rank ends)."""
    if world <= 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pack_hypotheses(first: int, labels, lengths, logp):
    """One rank's best hypotheses as a picklable record: (first utterance,
    [label list per utterance], fp64 log-probs)."""
    labels = np.asarray(labels)
    lengths = np.asarray(lengths)
    hyps = [labels[b, :int(lengths[b])].astype(np.int32).tolist() for b in range(len(lengths))]
    return (int(first), hyps, np.asarray(logp, np.float64).tolist())


def gather_hypotheses(record, world: int, rank: int):
    """Host-side gather of every rank's hypotheses to rank 0 (gloo, KB-scale;
    no collective on the data path).  Returns, on rank 0, the records of all
    ranks in utterance order; None elsewhere."""
    if world <= 1:
        return [record]
    out = [None] * world if rank == 0 else None
    dist.gather_object(record, out, dst=0)
    if rank != 0:
        return None
    return sorted(out, key=lambda r: r[0])


def merge_records(records):
    """Concatenate gathered records into (labels list, logp array) in global
    utterance order; checks that the shards are contiguous and disjoint."""
    hyps, lps, nxt = [], [], 0
    for first, h, lp in records:
        if first != nxt:
            raise AssertionError(f"gathered shards not contiguous: expected utterance {nxt}, got {first}")
        hyps += h
        lps += lp
        nxt = first + len(h)
    return hyps, np.asarray(lps, np.float64)


def hyp_digest(hyps, logp) -> str:
    """sha256 over every utterance's label ids and fp64 log-prob bits."""
    m = hashlib.sha256()
    for h, lp in zip(hyps, np.asarray(logp, np.float64)):
        m.update(np.asarray(h, np.int32).tobytes())
        m.update(b"|")
        m.update(np.float64(lp).tobytes())
    return m.hexdigest()


# ---------------------------------------------------------------- workload
def algorithmic_bytes_per_frame(V: int, beam: int) -> int:
    """4V (emission row, fp32, read once) + 32K (16-B beam
    record read + written) + 8K (8-B traceback record), K = beam + 1."""
    K = beam + 1
    return 4 * V + 40 * K


def make_weights(In, H, V, seed=20261015):
    """Random-init weights of the model's shapes (no checkpoints)."""
    rng_w = np.random.default_rng(seed)
    s = 1.0 / np.sqrt(H)
    w_ih = rng_w.uniform(-s, s, (In, H)).astype(np.float32)
    w_hh = rng_w.uniform(-s, s, (H, H)).astype(np.float32)
    b_ih = rng_w.uniform(-0.1, 0.1, H).astype(np.float32)
    b_hh = rng_w.uniform(-0.1, 0.1, H).astype(np.float32)
    w_out = rng_w.uniform(-4 * s, 4 * s, (H, V)).astype(np.float32)
    b_out = rng_w.uniform(-0.5, 0.5, V).astype(np.float32)
    return (w_ih, w_hh, b_ih, b_hh), (w_out, b_out)


def make_features(T, B, In, first, seed=20261015):
    """Features [T*B, In], time-major; utterance u's rows come from its own
    generator (seed + 1 + u), so every shard reproduces the full batch."""
    x = np.empty((T, B, In), np.float32)
    for b in range(B):
        x[:, b, :] = np.random.default_rng(seed + 1 + first + b).uniform(-1, 1, (T, In))
    return x.reshape(T * B, In)


def load_profile_json(name: str):
    p = ROOT / "profiles" / name
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())
    except Exception:
        return None


# profiles/<round>/ hold the counter summaries this line embeds: the newest
# round that profiled the workload and kernel variant (every record names its
# source run and commit)
PROFILE_ROUNDS = ("r06", "r05", "r04", "r03")


def decoder_variant(V: int, waves: int, max_states: int) -> str:
    """Template instance of the beam-search kernel a decode ran, as rocprofv3
    names it without spaces (ctc_beam_v*.hip / ctc_beam_wide.hip tables)."""
    rpt = 1 if max_states <= 64 else (2 if max_states <= 128 else 4)
    R = V + 1
    if R > 64:
        return f"ctc_wide_kernel<{rpt},false>"
    if waves < 0:   # the one-wave kernel (ASR_CTC_WAVES_LIST)
        return f"ctc_wave_kernel<{rpt},{'true' if V > 32 else 'false'}>"
    cls = 8 if R <= 8 else (32 if R <= 32 else 64)
    return f"ctc_beam_kernel<{waves},{cls // waves},{rpt},false>"


def load_counters(name: str, workload: str, variant: str):
    """A counter summary (profiles/<round>/<name>.json, written by
    tools/traffic_from_pmc.py / tools/issue_from_pmc.py from rocprofv3 --pmc
    passes over this bench) for exactly this workload and kernel variant, with
    the run it came from; None when that pair was not profiled (a changed
    kernel or schedule never picks up stale counters)."""
    for rnd in PROFILE_ROUNDS:
        d = load_profile_json(f"{rnd}/{name}.json")
        try:
            rec = d[workload][variant]
        except Exception:
            continue
        if name == "issue" and "issue" not in rec and "valu_mix" not in rec:
            continue
        return dict(rec, workload=workload, variant=variant, round=rnd)
    return None


def load_kernel_stats(workload: str, variant: str):
    """rocprofv3 --kernel-trace --stats average dispatch duration of this
    kernel variant in the committed trace of this bench workload
    (profiles/<round>/<workload>_final_kernel_stats.csv), or None."""
    import csv as _csv
    for rnd in PROFILE_ROUNDS:
        p = ROOT / "profiles" / rnd / f"{workload.lower()}_final_kernel_stats.csv"
        if not p.exists():
            continue
        try:
            for r in _csv.DictReader(open(p)):
                name = r["Name"].split("(")[0].replace("void ", "").replace("asr::", "").replace(" ", "")
                if name == variant:
                    return {"avg_ms": round(float(r["AverageNs"]) * 1e-6, 4), "calls": int(r["Calls"]),
                            "source": f"profiles/{rnd}/{p.name}"}
        except Exception:
            continue
    return None


def load_mfma_counters(workload: str):
    """Counter evidence of the dense kernels (profiles/<round>/mfma.json, from
    tools/mfma_from_pmc.py over a rocprofv3 --pmc pass of this bench):
    per kernel, MFMA busy cycles against the CUs' matrix-pipe cycles."""
    for rnd in PROFILE_ROUNDS:
        d = load_profile_json(f"{rnd}/mfma.json")
        if d and workload in d:
            return dict(d[workload], round=rnd)
    return None


def init_gloo(rank: int, world: int) -> None:
    """dist.init_process_group("gloo") with the native stdout (fd 1) pointed
    at stderr meanwhile: gloo prints "[Gloo] Rank r is connected to n peer
    ranks" to stdout from C++ while it connects, and rank 0's stdout must be
    the one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def cpu_share():
    """Host cores this process may use: the affinity mask, capped by a cgroup
    CPU quota (a GPU box may show many more CPUs than its share), else
    OMP_NUM_THREADS when the affinity shows the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    if quota is not None:
        n = min(n, quota)
    elif n == (os.cpu_count() or n) and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    return max(1, n), quota


class ClockSampler:
    """The GPU's shader (gfx) clock, socket power and hotspot temperature,
    sampled every ~10 ms from the driver's gpu_metrics (amdsmi) in a
    background thread over the timed region, so that a line measured on a
    slower-clocked box says so.  None fields when amdsmi is unavailable."""

    def __init__(self, local: int):
        self.samples, self.err, self.h = [], None, None
        self._stop = None
        try:
            import amdsmi
            self.amdsmi = amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            want = None
            try:   # match torch's device by PCI bus id
                pr = torch.cuda.get_device_properties(local)
                want = (int(pr.pci_domain_id), int(pr.pci_bus_id), int(pr.pci_device_id))
            except Exception:
                pass
            for h in handles:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)   # "dddd:bb:dd.f"
                dom, bus, rest = bdf.split(":")
                dev = rest.split(".")[0]
                if want is None or (int(dom, 16), int(bus, 16), int(dev, 16)) == want:
                    self.h = h
                    break
            if self.h is None and len(handles) == 1:
                self.h = handles[0]
            if self.h is None:
                self.err = f"no amdsmi device matches the torch device ({len(handles)} visible)"
        except Exception as e:  # pragma: no cover - depends on the box
            self.err = f"amdsmi unavailable: {type(e).__name__}: {e}"

    def _one(self):
        m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        def num(v):
            try:
                v = float(v)
                return v if v < 65535 else None   # 0xFFFF: field not supported
            except Exception:
                return None
        clk = m.get("current_gfxclk")
        if num(clk) is None:   # per-XCD clocks (gpu_metrics v1.4+)
            xs = [num(v) for v in (m.get("current_gfxclks") or [])]
            xs = [v for v in xs if v]
            clk = sum(xs) / len(xs) if xs else None
        return (time.perf_counter(), num(clk), num(m.get("current_socket_power") or m.get("average_socket_power")),
                num(m.get("temperature_hotspot")))

    def start(self):
        import threading
        if self.h is None:
            return
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                try:
                    self.samples.append(self._one())
                except Exception as e:  # pragma: no cover
                    self.err = f"{type(e).__name__}: {e}"
                    return
                self._stop.wait(0.01)
        self._t = threading.Thread(target=loop, daemon=True)
        self._t.start()

    def stop(self):
        if self._stop is not None:
            self._stop.set()
            self._t.join()
        try:
            if self.h is not None:
                self.amdsmi.amdsmi_shut_down()
        except Exception:
            pass
        clk = [c for _, c, _, _ in self.samples if c]
        pw = [w for _, _, w, _ in self.samples if w]
        tp = [t for _, _, _, t in self.samples if t]
        if not clk:
            return {"source": "amdsmi gpu_metrics", "samples": len(self.samples), "gfxclk_mhz": None,
                    "error": self.err}
        return {"source": "amdsmi gpu_metrics (current_gfxclk), every ~10 ms over the timed region",
                "samples": len(self.samples), "gfxclk_mhz": {"mean": round(float(np.mean(clk)), 1),
                                                             "min": round(float(min(clk)), 1),
                                                             "max": round(float(max(clk)), 1)},
                "socket_power_w": round(float(np.mean(pw)), 1) if pw else None,
                "hotspot_c_max": round(float(max(tp)), 1) if tp else None}


def serialized_decode(asr, em_host, T, Bp, V, beam, dcus, conc, queued=2, rounds=3):
    """The decoder alone, live, after the timed region, at the pipeline's load:
    the last batch's emissions decoded on conc + queued streams over the
    pipeline's decode CUs [0, dcus) (conc decodes are what those CUs hold at
    16 utterances per CU; the pipeline keeps `queued` more waiting so that
    their workgroups fill the CUs the oldest decodes' last utterances free),
    `rounds` decodes back to back on every stream, with the pipeline's decoder
    schedule; HIP events on those streams.  Returns ms per decode launch: the
    wall time of all rounds / (rounds x streams), i.e. the kernel's throughput
    with its dispatch tails filled as in the pipeline and nothing else
    running."""
    d_em = asr.DeviceMatrix.from_numpy(np.ascontiguousarray(em_host).reshape(T * Bp, V))
    ns = conc + queued
    sts = [cu_range_stream(0, dcus) for _ in range(ns)]
    # one handle per stream: its decodes run one after another there
    decs = [asr.CTCDecoder(V, beam, 0, waves=asr.ASR_CTC_WAVES_LIST) for _ in range(ns)]
    for d in decs:
        d.set_concurrency(conc)
    best = None
    for _ in range(2):   # the first pass sizes the workspaces
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(sts[0])
        ends = []
        for st, d in zip(sts, decs):
            st.wait_event(e0)
            for _ in range(rounds):
                d.decode_device(d_em.ptr, T, Bp, is_log=True, stream=st.cuda_stream)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(st)
            ends.append(e1)
        for e in ends:
            e.synchronize()
        ms = max(e0.elapsed_time(e) for e in ends)
        best = ms if best is None else min(best, ms)
    for d in decs:
        d.close()
    return best / (rounds * ns)


def union_ms(iv):
    """Total length of the union of intervals [(a, b)]."""
    tot, end = 0.0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def stage_figures(stamps, elapsed_ms, host_wait_ms, steps, nsub, inflight):
    """Per-stage figures of the timed region from the pipeline's timeline
    (asr_pipeline_get_timeline: per batch, ms after the region's start, of
    its production start / end and decode start / end) and the host's time
    blocked in collect: what the step is made of."""
    if stamps is None or len(stamps) == 0:
        return None
    t = np.asarray(stamps, np.float64)
    prod, dec = t[:, 1] - t[:, 0], t[:, 3] - t[:, 2]
    # steady state: the mean spacing of decode ends (in time order) over the
    # middle half of the batches, i.e. without the fill and the drain; with
    # fewer than 3 x inflight batches there is no such middle (every batch is
    # in the fill or the drain: the 256-per-GPU shard's 20 batches at 10 in
    # flight), and the figure is null
    n = len(t)
    steady = None
    if n >= 3 * max(1, inflight) and n >= 4:
        ends = np.sort(t[:, 3])
        lo, hi = n // 4, (3 * n) // 4
        steady = round(float((ends[hi] - ends[lo]) / (hi - lo) * nsub), 4)
    return {
        "source": "HIP timing events recorded by the pipeline in the timed run (asr_pipeline_set_timing)",
        "batches": int(n),
        "production_ms_per_batch": round(float(prod.mean()), 4),
        "decode_span_ms_per_batch": round(float(dec.mean()), 4),
        "production_busy_frac": round(union_ms(list(zip(t[:, 0], t[:, 1]))) / elapsed_ms, 4),
        "decode_busy_frac": round(union_ms(list(zip(t[:, 2], t[:, 3]))) / elapsed_ms, 4),
        "first_decode_start_ms": round(float(t[:, 2].min()), 4),
        "last_production_end_ms": round(float(t[:, 1].max()), 4),
        "last_decode_end_ms": round(float(t[:, 3].max()), 4),
        "steady_ms_per_step": steady,
        "host_wait_ms_per_step": round(host_wait_ms / steps, 4),
        "note": "a decode's start is when its stream reached it (it may then wait for CUs); steady_ms_per_step "
                "= mean spacing of the decode ends over the middle half of the batches x batches per step "
                "(null below 3 x inflight batches)"}


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


# ------------------------------------------------------------------- main
def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE and a
    127.0.0.1 rendezvous in their environment) and wait for them.  The parent
    makes no GPU call and does not exec: each rank is a fresh child process.
    Returns 0 when every rank succeeded, else the first failing status (the
    other ranks are then stopped: they would wait forever at a barrier)."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:],
                                      env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in live:   # the exact children started here, nothing else
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this run (default: the environment's, HIP's 4 if unset; the library fits its unmasked streams to it)")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); started by this script when WORLD_SIZE is unset")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="total utterances split over the GPUs (strong scaling)")
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--hidden", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--beam", type=int, default=None)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--decode-only", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-serialized", action="store_true",
                    help="skip the live stand-alone decoder timing after the timed region (profiling runs: "
                         "keeps the trace's decoder dispatches to the pipeline's own)")
    ap.add_argument("--prime-s", type=float, default=0.0,
                    help="native pipeline: seconds of untimed steps before the W warmup steps (for the clocks "
                         "to settle under the load; measured no effect at C4 / 256 per GPU, run ss)")
    ap.add_argument("--no-timeline", action="store_true",
                    help="native pipeline: no per-batch timing events in the timed run (the line's "
                         "config.stages is then null)")
    ap.add_argument("--cpu-full-T", action="store_true",
                    help="CPU baseline / parity sample over all T frames at any shape (default: all of "
                         "them when that is ~20 s of CPU work, as at C4; a prefix otherwise)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the rank-0 1-GPU re-decode of the gathered shards")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run RNN and decode of each step back to back on one stream")
    ap.add_argument("--cu-split", default="auto", choices=["auto", "none", "half", "fit", "interleave"],
                    help="production and decode streams on disjoint CU masks (auto: halves when the "
                         "batch's decode workgroups fit in half of the CUs; fit: one CU per workgroup)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches decoded concurrently, each on its own HIP stream and CU group "
                         "(0 = auto: as many one-CU-per-utterance groups as fit beside production, "
                         "at most 3; 1 = one decode at a time)")
    ap.add_argument("--segments", type=int, default=0,
                    help="T-segments per batch handed from production to decode (native pipeline, "
                         "fused production; 0 = the library's choice)")
    ap.add_argument("--decode-cus", type=int, default=0,
                    help="CUs per decode group (0: one per utterance, B rounded up to 8); fewer "
                         "CUs than utterances puts several decode workgroups on a CU when their "
                         "registers allow (--waves 4: 188 VGPRs, one wave per SIMD each)")
    ap.add_argument("--decode-partition", type=int, default=0,
                    help="batches that fill the chip: decode streams on CUs [0, N), production on the rest "
                         "(0: every stream on every CU)")
    ap.add_argument("--pipeline-batch", type=int, default=0,
                    help="utterances per pipeline batch (the rank's B go through as B / N batches; "
                         "0 = auto: 1024 when B is a larger multiple of it on the split-bf16 arithmetic)")
    ap.add_argument("--coalesce", type=int, default=0,
                    help="dynamic batching in the native pipeline (asr_pipeline_create_coalesced): this many "
                         "consecutive submits run as one batch (1 = off; 0 = auto: submits under 512 utterances "
                         "in launches of 512-640 (C2: 10, 256 per GPU: 2), else 1)")
    ap.add_argument("--py-pipeline", action="store_true",
                    help="the round-2 Python orchestration over torch streams instead of the library's "
                         "native pipeline (asr_pipeline_*); implied by its Python-only knobs")
    ap.add_argument("--no-partition", action="store_true",
                    help="batches that fill the chip: decode and production share every CU")
    ap.add_argument("--packed", action="store_true",
                    help="4-wave decode workgroups two to a CU, 5 batches in flight (C2-like shapes)")
    ap.add_argument("--prod-split", default="auto", choices=["auto", "off", "prod", "all", "norec"],
                    help="production on two streams: the recurrence on the production CUs, the "
                         "input/emission GEMMs on a second stream (prod: the same CUs, all: every CU, "
                         "norec: every CU but the recurrence's, which then get exactly one per utterance) "
                         "issued one batch ahead, so batch i+2's input projection overlaps batch "
                         "i+1's recurrence (auto: all when D > 1 and H <= 256)")
    ap.add_argument("--prod-streams", type=int, default=0,
                    help="production streams (unsplit production): batch i is produced on stream "
                         "i %% P, P batches ahead of its decode, so the recurrences of P batches run "
                         "at once (0 = auto: 2 when D > 1 and H > 256, i.e. C5's latency-bound "
                         "per-frame recurrence launches; else 1)")
    ap.add_argument("--graph-production", default="auto", choices=["auto", "on", "off"],
                    help="capture each buffer's whole production (RNN + projection) in a torch CUDA graph "
                         "and replay it per batch (auto: off; the library already replays C5's ~2000 "
                         "per-frame recurrence launches from its own HIP graph)")
    ap.add_argument("--result-stream", action="store_true",
                    help="run each batch's traceback on a third stream (measured slower at C2)")
    ap.add_argument("--dry-run-cpu", action="store_true",
                    help="no GPU: run the rank launcher, rendezvous, shard plan, gather and "
                         "1-process check with a host greedy decode standing in for the GPU "
                         "path (a plumbing rehearsal for CPU tests; prints no throughput)")
    ap.add_argument("--overlap-results", action="store_true",
                    help="queue batch i+1's decode before reading batch i's results "
                         "(measured slower on MI355X: see DESIGN.md §9)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    for k in ("T", "hidden", "vocab", "beam"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)
    if args.batch is not None:
        cfg["batch"] = args.batch
        cfg.pop("global_batch", None)
    if args.global_batch is not None:
        cfg["global_batch"] = args.global_batch

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"world size {world} (WORLD_SIZE) does not match --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run_cpu:
        return dry_run_cpu(cfg, rank, world)
    asr = _load("asr_amd", PKG / "asr_amd.py")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; more ranks than GPUs (a rehearsal on a smaller box)
    # wrap around.  device_count() does not initialise the GPU.
    ndev = torch.cuda.device_count() if torch is not None else 1
    local = local % max(1, ndev)
    if world > 1:
        init_gloo(rank, world)
    asr.set_device(local)

    T, H, V, beam = cfg["T"], cfg["hidden"], cfg["vocab"], cfg["beam"]
    strong = "global_batch" in cfg
    if strong:
        GB = cfg["global_batch"]
        first, B = shard_range(rank, world, GB)
    else:
        B = cfg["batch"]
        GB = B * world
        first = shard_first(rank, B)
    In = H
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = make_weights(In, H, V)
    DM = asr.DeviceMatrix.from_numpy
    d_wih, d_whh = DM(w_ih), DM(w_hh)
    d_bih, d_bhh = DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1))
    d_wout, d_bout = DM(w_out), DM(b_out.reshape(V, 1))
    d_x = DM(make_features(T, B, In, first))
    pipeline = not args.no_pipeline and not args.decode_only
    ncu = torch.cuda.get_device_properties(local).multi_processor_count if torch is not None else 256
    # the library's native pipeline unless a knob of the Python orchestration is asked for
    native = (pipeline and not args.py_pipeline and not (args.packed or args.decode_cus or args.waves or
              args.result_stream or args.overlap_results) and args.prod_split == "auto" and
              args.graph_production != "on" and args.cu_split == "auto")
    if native:
        return main_native(args, asr, rank, world, first, GB, B, T, In, H, V, beam, strong,
                           [d_x, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout])
    bcu = -(-B // 8) * 8   # CUs of one workgroup per utterance
    # --packed (C2-like shapes: H <= 256, V <= 63, a batch on at most a
    # quarter of the CUs): 4-wave decode workgroups (188 VGPRs, one wave per
    # SIMD) two to a CU, so a batch's decode group is half as many CUs; 1.72 ->
    # 1.89 ms per decode, 5 groups in flight: 64.5 M vs 58.8 M frames/s at 100
    # steps (r2g49), but its first timed run after a short warmup pays ~10 ms
    # once (20 steps / warmup 5: 27-28 M; gone at warmup 20, worse after an
    # idle 0.1 s: a clock ramp, r2g50/51/58), so it is not the default.
    packed = (args.packed and pipeline and not args.waves and not args.decode_cus and not args.inflight
              and H <= 256 and V + 1 <= 64 and 4 * bcu <= ncu)
    waves = 4 if packed else args.waves
    gcu = min(ncu, args.decode_cus or (-(-B // 16) * 8 if packed else bcu))
    Kb = beam + 1   # the library's automatic beam capacity (runtime.hip asr_ctc_create)
    kcap = -(-(Kb + max(8, Kb // 8)) // 32) * 32   # > 64 (C3's beam 100): no 3-per-CU 4-wave kernel
    D = 1
    plain = False   # batches that fill the chip: D decodes sharing the decode CUs
    dpart = args.decode_partition   # decode CUs [0, dpart), production on the rest (0: all shared)
    if pipeline:
        # auto: up to 3 decode groups for H <= 256 (C2: 38.7 M vs 21.1 M frames/s at
        # D = 1), 2 for the H = 1024 recurrence (C5: D = 2 3.48 M, D = 3 2.99 M,
        # gpurun_out/r2g31); packed: 5 (one recurrence group of bcu CUs beside them)
        if packed:
            D = max(1, min(5, (ncu - bcu) // gcu))
        elif 2 * bcu > ncu and H <= 256 and V + 1 <= 64 and kcap <= 64 and not args.decode_cus:
            # A batch fills the chip (C4: 2048 / N utterances per GPU).
            # Consecutive batches then decode concurrently until ~3 utterances
            # share each CU — the library packs them three 4-wave workgroups
            # to a CU (asr_ctc_set_concurrency); C4 on one GPU (2048 = 8 per
            # CU) needs no second batch.  Up to 4 per CU the production gets
            # its own CUs (the decodes would otherwise starve it: its GEMM and
            # recurrence workgroups cannot share a CU with three decode
            # workgroups), half of them, with 3 production streams and the
            # MFMA recurrence (16 utterances per CU; its 4.6 ms latency is
            # hidden by the streams), and at least two batches decode at once
            # (the next batch's workgroups fill the CUs the last round of the
            # previous one leaves idle).  Measured (profiles/r03/bench_scan.md):
            # 256 per GPU: every CU shared 73.2 M frames/s, decode on 192 /
            # 160 / 144 / 128 / 112 CUs 63.4 / 82.3 / 86.0 / 89.3 / 69.2 M;
            # 1024 per GPU: one decode at a time 79.3 M, two 94.4 M.
            u = -(-B // ncu)
            plain = True
            if u <= 4 and not args.no_partition:
                dpart = args.decode_partition or (ncu // 2) // 8 * 8
                D = args.inflight or max(2, -(-3 // u))
            else:
                D = args.inflight or max(1, -(-3 // u))
        else:
            D = args.inflight or max(1, min(3 if H <= 256 else 2, ncu // gcu - 1))
        if D > 1 and not plain and (D + 1) * gcu > ncu:
            raise SystemExit(f"--inflight {D}: {D} decode groups of {gcu} CUs + production exceed {ncu} CUs")
    # Buffer i % nbuf holds batch i.  D batches are decoding while batch i+1 is
    # produced, and a buffer is only produced into after its batch's results
    # were read (asr_amd.h lifetime rule: an overflow retry re-reads it), so
    # D + 1 buffers (--overlap-results, D = 1: a third one).
    split_prod_auto = D > 1 and H <= 256 and not plain   # --prod-split auto (below)
    Pn = 1
    if pipeline and not (args.prod_split in ("prod", "all", "norec") or
                         (args.prod_split == "auto" and split_prod_auto)):
        Pn = args.prod_streams or (3 if plain and dpart else (2 if D > 1 and H > 256 else 1))
    if plain and H <= 256:
        # 16 utterances per CU (the production partition's, or beside the
        # decodes), and the same recurrence kernel at every shard size, so
        # that an utterance's emissions are the same bits at N = 1 / 2 / 4 / 8
        asr.rnn_set_recurrence(asr.RNN_RECUR_MFMA)
    # P production streams produce P batches ahead: D + P buffers
    nbuf = (D + Pn if D > 1 or Pn > 1 else (3 if args.overlap_results else 2)) if pipeline else 1
    d_hid = [asr.DeviceMatrix(T * B, H) for _ in range(nbuf)]
    d_emis = [asr.DeviceMatrix(T * B, V) for _ in range(nbuf)]
    decs = [asr.CTCDecoder(V, beam, 0, waves=waves) for _ in range(nbuf)]
    if plain:   # D decodes of B utterances share the CUs: schedule for D x B
        for d in decs:
            d.set_concurrency(D)
    if pipeline:   # HIP streams/events via torch (same HIP runtime as libasr_amd)
        torch.cuda.set_device(local)
        s_prod, s_dec = torch.cuda.Stream(), torch.cuda.Stream()
        s_decs = [s_dec]
        split = args.cu_split
        if plain:
            split = "plain"
            if dpart:   # decodes on CUs [0, dpart), production on [dpart, ncu)
                s_decs = [cu_range_stream(0, dpart) for _ in range(D)]
                s_prod = cu_range_stream(dpart, ncu)
            else:
                s_decs = [torch.cuda.Stream() for _ in range(D)]
            s_dec = s_decs[0]
        elif D > 1:
            split = "groups"
            s_prod, s_decs = cu_group_streams(D, gcu, ncu)
            s_dec = s_decs[0]
        elif split == "auto":   # one decode workgroup per utterance, one per CU
            split = "half" if B <= ncu // 2 else "none"   # fit: equal at C2, slower at C5 (r2g28)
        if split not in ("none", "groups", "plain"):   # the RNN's workgroups then never share a CU with the decoder's
            s_prod, s_dec = cu_masked_streams(split, B)
            s_decs = [s_dec]
        split_note = {"none": "", "plain": f"; {D} batches decoding at once (batch i on stream i % {D}) "
                                           + (f"on CUs [0, {dpart}), production on the rest"
                                              if dpart else "on every CU") +
                                           f", decoders scheduled for {D} x {B} utterances "
                                           f"(asr_ctc_set_concurrency)",
                      "half": "; decode on CUs [0, n/2), production on [n/2, n)",
                      "fit": f"; decode on CUs [0, {gcu}) (one per utterance), production on the rest",
                      "interleave": "; decode on even CUs, production on odd",
                      "groups": f"; {D} batches decoding at once, batch i on stream i % {D} restricted to "
                                f"CUs [{gcu}*(i % {D}), {gcu}*(i % {D} + 1)) (one per utterance), "
                                f"production on CUs [{D * gcu}, {ncu})"}[split]
        psplit = args.prod_split
        if psplit == "auto":   # C2 (r2g34): off 46.4, prod 49.4, all 58.6 M frames/s;
            # C5 (H = 1024, 2000 recurrence launches): a split is slower
            psplit = ("norec" if packed else "all") if split_prod_auto else "off"
        if psplit == "off":
            s_gemm = s_prod
        elif psplit == "all":
            s_gemm = cu_range_stream(dpart, ncu) if split == "plain" and dpart else torch.cuda.Stream()
        elif psplit == "norec" and split == "groups":
            # recurrence on the B CUs after the decode groups (one workgroup per
            # utterance); the GEMMs on every other CU, decode groups included
            r0, r1 = D * gcu, min(ncu, D * gcu + -(-B // 8) * 8)
            s_prod = cu_range_stream(r0, r1)
            s_gemm = cu_ranges_stream([(0, r0), (r1, ncu)])
            split_note = split_note.replace(f"production on CUs [{D * gcu}, {ncu})",
                                            f"recurrence on CUs [{r0}, {r1})")
        else:   # a second stream on the production CUs
            s_gemm = cu_range_stream(D * gcu if D > 1 else 0, ncu) if split == "groups" else torch.cuda.Stream()
        if psplit != "off":
            where = {"prod": "production CUs", "all": "all CUs", "norec": "all CUs but the recurrence's"}[psplit]
            split_note += (f"; production split: recurrence on its stream, input/emission GEMMs on a "
                           f"second stream ({where}) one batch ahead")
        s_prods = [s_prod]
        for _ in range(Pn - 1):   # more production streams on the production CUs
            s_prods.append(cu_range_stream(D * gcu, ncu) if split == "groups" else
                           cu_range_stream(dpart, ncu) if split == "plain" and dpart else torch.cuda.Stream())
        if Pn > 1:
            split_note += f"; {Pn} production streams, batch i produced on stream i % {Pn}"
        if args.result_stream:   # tracebacks off the decode stream
            s_res = torch.cuda.Stream()
            for d in decs:
                d.set_result_stream(s_res.cuda_stream)
        ev_ready = [torch.cuda.Event() for _ in range(nbuf)]
        ev_free = [torch.cuda.Event() for _ in range(nbuf)]
        ev_proj = [torch.cuda.Event() for _ in range(nbuf)]
        ev_rec = [torch.cuda.Event() for _ in range(nbuf)]
        prod_stream = s_prod.cuda_stream
    else:
        prod_stream = 0
        split_note = ""
        psplit = "off"

    def produce(k, x=d_x, nb=B, stream=None):
        """RNN forward + emission projection of a batch into buffer k."""
        st = prod_stream if stream is None else stream
        asr.rnn_fwd(x, d_wih, d_whh, d_bih, d_bhh, d_hid[k], T, nb, stream=st)
        asr.linear_fwd(d_hid[k], d_wout, d_bout, d_emis[k], asr.EPI_BIAS_LOGSOFTMAX, st)

    def produce_head(k):
        """Split production, part 1: input projection of buffer k's batch on the
        GEMM stream, then its recurrence on the recurrence stream."""
        asr.linear_fwd(d_x, d_wih, None, d_hid[k], asr.EPI_NONE, s_gemm.cuda_stream)
        ev_proj[k].record(s_gemm)
        s_prod.wait_event(ev_proj[k])
        asr.rnn_recur_fwd(d_whh, d_bih, d_bhh, d_hid[k], T, B, stream=prod_stream)
        ev_rec[k].record(s_prod)

    def produce_tail(k):
        """Split production, part 2: emission projection of buffer k once its
        recurrence is done and its previous batch's decode has finished."""
        s_gemm.wait_event(ev_rec[k])
        s_gemm.wait_event(ev_free[k])
        asr.linear_fwd(d_hid[k], d_wout, d_bout, d_emis[k], asr.EPI_BIAS_LOGSOFTMAX, s_gemm.cuda_stream)
        ev_ready[k].record(s_gemm)

    if args.decode_only:   # emissions computed once, outside the timed region
        produce(0)
        asr.synchronize()

    kernel_ms = []
    last = {}

    def enqueue(k, stream=0):
        """Decode buffer k and its traceback; the results follow to pinned host memory."""
        decs[k].decode_device(d_emis[k].ptr, T, B, is_log=True, stream=stream)

    def collect(k):
        """Wait for buffer k's results (an event, not the stream) and read them."""
        labels, lens, lp = decs[k].best_arrays()
        kernel_ms.append(decs[k].last_kernel_ms())
        last["k"] = k
        return labels, lens, lp

    def run(n):
        """n steps; every step's RNN, projection, decode and result copy."""
        if not pipeline:
            for _ in range(n):
                if not args.decode_only:
                    produce(0)
                enqueue(0)
                collect(0)
            return
        lag = D - 1 if D > 1 else (1 if args.overlap_results else 0)
        split_prod = psplit != "off"
        if split_prod:
            produce_head(0)
            produce_tail(0)
            if n > 1:
                produce_head(1 % nbuf)
        else:   # the first P batches, one per production stream
            for j in range(min(Pn, n)):
                produce(j % nbuf, stream=s_prods[j % Pn].cuda_stream)
                ev_ready[j % nbuf].record(s_prods[j % Pn])
        pending = []   # buffers decoded, results not read yet (oldest first)
        for i in range(n):
            k = i % nbuf
            sd = s_decs[i % D]
            # batch i's decode is queued first: the host time spent queueing
            # the production (C5: one recurrence launch per frame) then
            # overlaps the decode instead of delaying it
            sd.wait_event(ev_ready[k])
            enqueue(k, sd.cuda_stream)
            ev_free[k].record(sd)
            pending.append(k)
            if split_prod:
                # GEMM stream order: batch i+2's input projection, then batch
                # i+1's emission projection (which waits for i+1's recurrence),
                # so the projection overlaps the recurrence of batch i+1
                if i + 2 < n:
                    produce_head((i + 2) % nbuf)
                if i + 1 < n:
                    produce_tail((i + 1) % nbuf)
            elif i + Pn < n:   # batch i+P is produced while batch i is decoded
                kn = (i + Pn) % nbuf
                sp = s_prods[(i + Pn) % Pn]
                sp.wait_event(ev_free[kn])
                produce(kn, stream=sp.cuda_stream)
                ev_ready[kn].record(sp)
            # read the oldest batch once `lag` newer ones are decoding behind it
            while len(pending) > lag:
                collect(pending.pop(0))
        while pending:
            collect(pending.pop(0))

    graphs = None
    # auto = off: the library replays the per-frame recurrence launches of
    # H > 256 from its own HIP graph (runtime.hip rnn_recurrence_frames)
    if pipeline and psplit == "off" and args.graph_production == "on":
        # one HIP graph per buffer (fixed pointers), captured after a first
        # eager production sized every workspace; replayed on the production
        # streams by produce_graph()
        produce(0)
        asr.synchronize()
        s_cap = torch.cuda.Stream()
        graphs = []
        for k in range(nbuf):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s_cap):
                produce(k, stream=s_cap.cuda_stream)
            graphs.append(g)
        asr.synchronize()
        split_note += "; each batch's production replayed from a HIP graph"

    if graphs is not None:
        eager_produce = produce

        def produce(k, x=d_x, nb=B, stream=None):   # noqa: F811
            """Replay buffer k's captured production on `stream`."""
            if x is not d_x or nb != B:
                return eager_produce(k, x, nb, stream)
            sp = next((t for t in s_prods if t.cuda_stream == stream), s_prod) if stream is not None else s_prod
            with torch.cuda.stream(sp):
                graphs[k].replay()

    if pipeline:
        # every buffer's decoder handle sizes its workspace (hipMalloc, which
        # synchronises the device) before the warmup: with D batches in flight
        # the warmup alone may not reach every buffer
        for k in range(nbuf):
            produce(k)
            asr.synchronize()
            enqueue(k, s_decs[k % D].cuda_stream)
            collect(k)
        # and one pipelined pass over every buffer, stream and event (torch
        # creates an event's HIP event at its first record)
        run(nbuf + Pn)
        kernel_ms.clear()
    run(args.warmup)
    kernel_ms.clear()
    if world > 1:
        dist.barrier()
    # no Python garbage collection inside the timed region (the host loop
    # only queues work and reads results; a collection pause stalls the queue)
    gc.collect()
    gc.disable()
    asr.synchronize()
    if os.environ.get("ASR_BENCH_SLEEP"):   # diagnostics: idle before the timed region
        time.sleep(float(os.environ["ASR_BENCH_SLEEP"]))
    t0 = time.perf_counter()
    run(args.steps)
    asr.synchronize()
    elapsed = time.perf_counter() - t0
    gc.enable()
    if os.environ.get("ASR_BENCH_REPEAT"):   # diagnostics: the same timed run again, to stderr
        for _ in range(int(os.environ["ASR_BENCH_REPEAT"])):
            asr.synchronize()
            t1 = time.perf_counter()
            run(args.steps)
            asr.synchronize()
            print(f"repeat: {1e3 * (time.perf_counter() - t1) / args.steps:.4f} ms/step", file=sys.stderr)
    elapsed = reduce_max_over_ranks(elapsed, world)
    if world > 1:
        dist.barrier()

    finish(args, asr, rank, world, first, GB, B, T, In, H, V, beam, strong, elapsed, kernel_ms,
           decs[last["k"]].best_arrays(), decs[last["k"]].config(),
           [d_x, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout], d_hid[0], d_emis[0], d_emis[last["k"]],
           {"inflight_decodes": D, "production_streams": Pn, "decode_partition_cus": dpart or None,
            "decode_cus_per_batch": gcu if pipeline and D > 1 and not plain else None,
            "pipeline": ("python orchestration over torch streams (--py-pipeline): RNN+projection of "
                         "batch i+1 on one HIP stream || decode of batch i on another" + split_note +
                         ("; tracebacks on a third stream" if args.result_stream else "")
                         if pipeline else "none (sequential)")})
    for d in decs:
        d.close()
    asr.synchronize()
    destroy_raw_streams()


def finish(args, asr, rank, world, first, GB, B, T, In, H, V, beam, strong, elapsed, kernel_ms, best,
           dec_config, weights, d_hid0, d_emis0, d_emis_last, sched, parity_src=None):
    """Everything after the timed region: host gather of the hypotheses,
    roofline, GEMM MFMA utilisation, CPU baseline and the JSON line (rank 0)."""
    d_x, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout = weights
    # per-stage spans, clock and CU placement of the timed run: top-level fields of the line
    sched = dict(sched or {})
    measured = {k: sched.pop(k) for k in ("stages", "clock", "cu_placement", "host") if k in sched}
    ser = sched.pop("serialized", None)
    DM = asr.DeviceMatrix.from_numpy
    # ---- host-side gather of the hypotheses (outside the timed region)
    labels, lens, lp = best
    records = gather_hypotheses(pack_hypotheses(first, labels, lens, lp), world, rank)
    gather = None
    if rank == 0:
        hyps, lps = merge_records(records)
        if len(hyps) != GB:
            raise AssertionError(f"gathered {len(hyps)} hypotheses, expected {GB}")
        gather = {"utterances": len(hyps), "digest": hyp_digest(hyps, lps)[:16]}
        if world > 1 and not args.no_verify:
            # the same utterance ids decoded shard by shard on this one GPU
            ok = True
            for (f, h, l) in records:
                nb = len(h)
                xg = DM(make_features(T, nb, In, f))
                em_g = asr.DeviceMatrix(T * nb, V)
                asr.model_emissions(xg, [d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout], T, nb, em_g,
                                    bool((sched or {}).get("fused_emission")),
                                    recurrence=(sched or {}).get("recurrence"))
                dg = asr.CTCDecoder(V, beam, 0, waves=args.waves)
                dg.decode_device(em_g.ptr, T, nb, is_log=True)
                lab1, lp1 = dg.best()
                dg.close()
                ok = ok and lab1 == h and np.array_equal(np.asarray(lp1), np.asarray(l))
            gather["verified_vs_1gpu"] = bool(ok)
            if not ok:
                raise AssertionError("gathered hypotheses differ from the 1-GPU decode")
    if world > 1:
        dist.barrier()

    frames = GB * T * args.steps
    value = frames / elapsed
    avg_kernel_ms = float(np.mean(kernel_ms)) if kernel_ms else None
    bpf = algorithmic_bytes_per_frame(V, beam)
    roof = None
    # one decode launch covers a pipeline batch (Bl utterances); the parity
    # witness is the last collected batch
    Bl, best_p = parity_src if parity_src else (B, best)
    if avg_kernel_ms:
        achieved = bpf * Bl * T / (avg_kernel_ms * 1e-3) / 1e9
        ms_, waves_run, _ = dec_config
        variant = decoder_variant(V, waves_run, ms_)
        wl = args.config + (" decode-only" if args.decode_only else "")
        traffic = load_counters("traffic", wl, variant)
        issue = load_counters("issue", wl, variant)
        # a T-segmented decode (asr_pipeline segments) is S kernel dispatches
        # of T / S frames each; a "launch" here is the whole decode of a
        # batch (the HIP-event spans of its dispatches, summed), so the
        # per-dispatch counter and trace figures are scaled by S
        nseg = int((sched or {}).get("segments") or 1)
        kstats = load_kernel_stats(wl, variant)
        if kstats:
            kstats = dict(kstats, dispatches_per_launch=nseg, per_launch_ms=round(kstats["avg_ms"] * nseg, 4))
        # The decoder moves ~4V + 8 bytes per live node per frame: the beam
        # never leaves the CU, so HBM is not what bounds it.  Its limiter is
        # the per-frame dependency chain on chip (LDS round trips, barriers,
        # the selection passes), so `bound` names that and `frac` stays the
        # HBM fraction of SURVEY §8(d)'s algorithmic bytes, for information.
        roof = {"kernel": variant, "bound": "latency", "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "frac_of": "HBM roofline (SURVEY §8(d) algorithmic bytes: 4V + 40K per frame)",
                "avg_launch_ms": round(avg_kernel_ms, 4), "bytes_per_frame": bpf,
                "frames_per_launch": Bl * T, "us_per_frame_step": round(1e3 * avg_kernel_ms / T, 4),
                "decode_dispatches_per_launch": nseg,
                "traffic": traffic["hbm_bytes_per_launch"] * nseg if traffic else None,
                "traffic_source": traffic, "issue": issue,
                # avg_launch_ms is the HIP-event span on the decode stream: with
                # one decode queued beyond those the decode CUs hold it includes
                # that decode's wait for CUs; rocprofv3's dispatch duration of
                # the same kernel in the committed trace of this workload:
                "rocprof_kernel": kstats,
                # the same kernel alone at the pipeline's load (live), and the
                # chip-level rate: algorithmic bytes of a whole step / ms_per_step
                "serialized": (dict(ser, achieved=round(bpf * Bl * T / (ser["ms_per_launch"] * 1e-3) / 1e9, 3),
                                    frac=round(bpf * Bl * T / (ser["ms_per_launch"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5))
                               if ser else None),
                "chip_level": {"achieved": round(bpf * GB * T * args.steps / elapsed / world / 1e9, 3),
                               "frac": round(bpf * GB * T * args.steps / elapsed / world / 1e9 / HBM_PEAK_GBS, 5),
                               "how": "algorithmic bytes of every frame decoded in the timed region / its "
                                      "wall time, per GPU"},
                "limiter": "on-chip dependency latency per frame (beam resident in LDS): "
                           "see roofline.issue for the measured issue/wait fractions"}

    mfma = None
    if rank == 0 and world == 1 and not args.decode_only:
        mfma = measure_gemms(asr, d_x, d_wih, d_hid0, d_wout, d_bout, d_emis0, T, B, In, H, V,
                             fused=(d_whh, d_bih, d_bhh) if (sched or {}).get("fused_emission") else None)
        pmc = load_mfma_counters(args.config)
        if pmc:   # the rocprofv3 counters of the same stages (MFMA busy cycles, clock)
            ks = pmc.get("kernels", {})

            def pick(prefix, biggest=True):
                lst = [r for k, v in ks.items() if k.startswith(prefix) for r in v]
                return max(lst, key=lambda r: r["gflop"]) if lst else None
            split = mfma.get("arith") == "split_bf16"
            for stage, kern in (("input_gemm", "gemm_x3_kernel<" if split else "gemm_wide_kernel"),
                                ("emission_gemm", "gemm_narrow_kernel"),
                                ("recurrence_emission",
                                 "rnn_recur_x3_kernel<8,true" if split else "rnn_recur_mfma_kernel<true")):
                r = pick(kern)
                if stage in mfma and r:
                    mfma[stage]["counters"] = {k: r[k] for k in ("mfma_busy", "cus", "gflop", "clock_ghz",
                                                                 "duration_ms", "dispatches")}
            mfma["counters_source"] = {"source": pmc.get("source"), "round": pmc.get("round"),
                                       "note": pmc.get("note")}

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if isinstance(d_emis_last, tuple):   # (host emissions, how they were obtained)
            emis_host, note = d_emis_last
        else:
            emis_host, note = d_emis_last.toCpu(), "the decoded buffer of the timed region's last batch"
        cpu = cpu_baseline(asr, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout, T, Bl, In, H, V, beam, emis_host,
                           best_p, full_T=args.cpu_full_T, emis_note=note)
        parity = cpu.pop("parity")

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": ("f32 (RNN/Linear: fp32-accurate split-bf16 MFMA, x = h + m + l, 6 products) + f64 "
                      "(beam scores)" if asr.get_dense_arith() == asr.DENSE_SPLIT_BF16
                      else "f32 (RNN/Linear fp32 MFMA) + f64 (beam scores)"),
            "data": "synthetic: U(-1,1) features from numpy PCG64 seeded per utterance "
                    "(20261016+u), random-init weights (PCG64 20261015); emissions = "
                    "log_softmax of the RNN->Linear output (not SURVEY §8(d)'s mt19937_64 "
                    "softmax(N(0,3^2)) emissions, which the parity tests use)",
            "config": {"workload": (args.config + (" decode-only" if args.decode_only else " RNN+Linear+CTC")) +
                       f": B={B}/GPU (global {GB}), T={T}, hidden={H}, vocab={V}, beam={beam}",
                       "batch_per_gpu": B, "global_batch": GB, "T": T, "hidden": H,
                       "vocab": V, "beam": beam, "parallelism": f"utterance-shard x{world}",
                       "decode_waves": dec_config[1],   # the schedule the decodes ran
                       "dense_arith": "split_bf16" if asr.get_dense_arith() == asr.DENSE_SPLIT_BF16 else "f32",
                       **sched},
            "roofline": roof, "mfma": mfma, "cpu_baseline": cpu, "parity": parity, "gather": gather,
            **measured,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and parity.get("checked") and not parity.get("match"):
        raise SystemExit(f"parity: the measured path's results differ from the oracle on utterances "
                         f"{parity.get('mismatched_ids')}")


def main_native(args, asr, rank, world, first, GB, B, T, In, H, V, beam, strong, weights):
    """The default pipelined bench: the library's own throughput pipeline
    (asr_pipeline_*: streams, buffers, CU placement and decoder schedule chosen
    natively from the shapes), the host loop only submitting batches and
    reading each batch's results once `inflight` newer ones are queued."""
    d_x, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout = weights
    dcus = -1 if args.no_partition else args.decode_partition
    # The rank's B utterances go through the pipeline as B / Bp batches of Bp
    # (--pipeline-batch; auto: 1024 when B is a multiple of 1024 above it on
    # the split-bf16 arithmetic — measured at 2048 per GPU: 269 M frames/s as
    # two 1024-utterance batches against 240 M as one, the two decodes and
    # two productions in flight overlapping where one 2048 batch serialises
    # them; profiles/r04/bench_scan.md).  Every step still produces and
    # decodes all B utterances x T frames.
    split = asr.get_dense_arith() == asr.DENSE_SPLIT_BF16
    Bp = args.pipeline_batch or (1024 if split and B > 1024 and B % 1024 == 0 else B)
    if B % Bp:
        raise SystemExit(f"--pipeline-batch {Bp} does not divide the {B} utterances per GPU")
    nsub = B // Bp
    if nsub > 1:
        xh = d_x.toCpu().reshape(T, B, In)
        xs = [asr.DeviceMatrix.from_numpy(np.ascontiguousarray(xh[:, k * Bp:(k + 1) * Bp, :]).reshape(T * Bp, In))
              for k in range(nsub)]
        del xh
    else:
        xs = [d_x]
    # dynamic batching: submits under 512 utterances as launches of 512-640
    # (runs r6cc / r6dd, 20 / 5, frames/s: C2's 64 per submit at 1 / 4 / 5 /
    # 10 / 20 per launch 66.0 / 104.7 / 107.7 / 113.0-115.1 / 82.6 M; 128 per
    # GPU 1 / 4: 133.8 / 204.6 M; 256 per GPU 1 / 2 / 4: 218.8-224.2 /
    # 232.4-236.4 / 213.8 M; 512 per GPU 1 / 2: 303.5 / 266.6 M — fewer,
    # larger batches lengthen the fill and the drain once a batch fills the chip)
    # (measured for the fused H <= 256, V <= 32, beam <= 56 shapes only: C5,
    # BL and C3's beam 100 keep one submit per launch)
    small = H <= 256 and V <= 32 and beam <= 56 and Bp < 512
    cg = args.coalesce if args.coalesce > 0 else (min(10, max(1, (640 if Bp < 128 else 512) // Bp)) if small else 1)
    pw = [d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout]
    try:
        pl = asr.Pipeline(T, Bp, In, H, V, beam, pw, inflight=args.inflight, prod_streams=args.prod_streams,
                          decode_cus=dcus, segments=args.segments, coalesce=cg)
    except asr.AsrError:
        if cg == 1 or args.coalesce > 0:
            raise
        cg = 1   # a schedule the library does not coalesce
        pl = asr.Pipeline(T, Bp, In, H, V, beam, pw, inflight=args.inflight, prod_streams=args.prod_streams,
                          decode_cus=dcus, segments=args.segments)
    desc = pl.describe()
    if desc["mode"] == asr.PIPELINE_MODES[1] and H <= 256:
        # the pipeline's MFMA recurrence for chip-filling batches, also for
        # the 1-GPU re-decode that checks the gathered shards
        asr.rnn_set_recurrence(asr.RNN_RECUR_MFMA)
    # results of batch i are read once the pipeline's buffers hold newer work:
    # D decoding and P producing
    lag = (desc["inflight"] + desc["prod_streams"]) * cg   # submits: cg per pipeline batch
    kernel_ms = []
    best = {}

    hostlog = [] if os.environ.get("ASR_BENCH_HOSTLOG") else None   # diagnostic: host call times

    # one result slot per sub-batch (collects come in submission order, so
    # the last step's B utterances end up in slots 0 .. nsub-1, in order)
    _l, _n, _p = pl._lab, pl._len, pl._lp
    slots = [(np.empty_like(_l), np.empty_like(_n), np.empty_like(_p)) for _ in range(nsub)]

    def take():
        tw = time.perf_counter()
        lab, ln, lp, ms = pl.collect(out=slots[take.j % nsub])
        take.wait += time.perf_counter() - tw
        take.j += 1
        kernel_ms.append(ms)
        if hostlog is not None:
            hostlog.append(("collect", time.perf_counter()))

    def run(n):
        for _ in range(n * nsub):
            pl.submit(xs[run.k % nsub])
            run.k += 1
            if hostlog is not None:
                hostlog.append(("submit", time.perf_counter()))
            while pl.pending() > lag:
                take()
        while pl.pending():
            take()
    run.k = 0
    take.j = 0
    take.wait = 0.0

    run(-(-(2 * (desc["inflight"] + desc["prod_streams"]) + 1) * cg // nsub))   # every buffer, stream and workspace once
    # priming: the GPU's clocks settle under this load before the W warmup
    # steps (untimed, like the line above; --prime-s 0 skips it)
    tp = time.perf_counter()
    while time.perf_counter() - tp < args.prime_s:
        run(1)
    run(args.warmup)
    kernel_ms.clear()
    timeline = not args.no_timeline
    clock = ClockSampler(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    if world > 1:
        dist.barrier()
    gc.collect()
    gc.disable()
    asr.synchronize()
    if timeline:   # per-batch stage stamps of the timed run (4 timing events per batch), from now
        pl.set_timing(True)
    clock.start()
    take.wait = 0.0
    c0 = time.process_time()
    t0 = time.perf_counter()
    run(args.steps)
    asr.synchronize()
    elapsed = time.perf_counter() - t0
    host_cpu_ms = 1e3 * (time.process_time() - c0) / args.steps
    clock_fig = clock.stop()
    gc.enable()
    stages = None
    if timeline:
        _, stamps = pl.timeline()
        stages = stage_figures(stamps, 1e3 * elapsed, 1e3 * take.wait, args.steps, nsub / cg, desc["inflight"])
        if os.environ.get("ASR_BENCH_TIMELINE"):   # diagnostics: the raw per-batch stamps
            np.savetxt(os.environ["ASR_BENCH_TIMELINE"], stamps, fmt="%.4f",
                       header="production start, production end, decode start, decode end (ms)")
        pl.set_timing(False)
    placement = {"streams": [list(r) for r in pl.placement()]}
    try:   # physical CUs per XCD that each role's CU mask reaches (HW_REG_XCC_ID / HW_ID probe)
        for role in ("decode", "production"):
            if any(r[0] == role for r in placement["streams"]):
                placement[role + "_cus_per_xcd"] = pl.probe_placement(role)
    except Exception as e:  # pragma: no cover
        placement["probe_error"] = str(e)
    if hostlog is not None:
        with open(os.environ["ASR_BENCH_HOSTLOG"], "w") as f:
            for what, tt in hostlog:
                f.write(f"{what} {1e3 * (tt - t0):.3f}\n")
    elapsed = reduce_max_over_ranks(elapsed, world)
    host = {"cpu_ms_per_step": round(host_cpu_ms, 4),
            "cpu_ms_per_step_max_over_ranks": round(reduce_max_over_ranks(host_cpu_ms, world), 4),
            "how": "time.process_time() of the rank's process (all its threads) over the timed region / steps: "
                   "the host CPU one rank spends per step (an 8-rank node shares its host cores)"}
    if world > 1:
        dist.barrier()
    desc = pl.describe()
    assert take.j % nsub == 0 and run.k % nsub == 0
    last = [tuple(a.copy() for a in r) for r in slots]
    lab_p, ln_p, lp_p = last[-1]   # the last collected batch: the parity witness's
    lab = np.concatenate([r[0] for r in last])
    ln = np.concatenate([r[1] for r in last])
    lp = np.concatenate([r[2] for r in last])
    Kb = beam + 1
    kcap = -(-(Kb + max(8, Kb // 8)) // 32) * 32
    # buffers for the GEMM timing
    hid0, em0 = asr.DeviceMatrix(T * B, H), asr.DeviceMatrix(T * B, V)
    fused = desc["fused_emission"]
    em_last = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the exact bytes the last collected batch's decode consumed (the
        # parity witness of the measured path), and a check that
        # model_emissions reproduces them (the 1-GPU re-decode relies on it)
        em_last = pl.peek_emissions()
        em_chk, wk = (em0, hid0) if nsub == 1 else (asr.DeviceMatrix(T * Bp, V), asr.DeviceMatrix(T * Bp, H))
        asr.model_emissions(xs[-1], [d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout], T, Bp, em_chk, fused, work=wk,
                            recurrence=desc["recurrence"])
        same = bool(np.array_equal(em_chk.toCpu().reshape(T, Bp, V), em_last))
        em_last = (em_last, "the pipeline's own emission buffer of the timed region's last batch "
                            "(asr_pipeline_peek_emissions); model_emissions reproduces it bit for bit: "
                            + ("yes" if same else "NO"))
        if not same:
            raise SystemExit("model_emissions does not reproduce the pipeline's emissions")
    ser = None
    if (rank == 0 and desc["mode"] == asr.PIPELINE_MODES[1] and desc["decode_cus"] < 256
            and not args.no_serialized):
        dc = desc["decode_cus"]
        conc = max(1, (16 if kcap <= 64 else 9) * dc // Bp)   # the decodes the decode CUs hold
        queued = max(0, desc["inflight"] - conc)
        ms1 = serialized_decode(asr, em_last[0] if em_last is not None else pl.peek_emissions(), T, Bp, V, beam,
                                dc, conc, queued=queued)
        ser = {"ms_per_launch": round(ms1, 4), "concurrent": conc, "queued": queued, "decode_cus": dc,
               "how": f"{conc + queued} streams over the {dc} decode CUs ({conc} decodes resident at 16 per "
                      f"CU, {queued} queued, as in the pipeline), 3 decodes of the last batch's emissions back "
                      f"to back on each, nothing else running: wall / decodes (HIP events, live after the timed "
                      f"region)"}
    finish(args, asr, rank, world, first, GB, B, T, In, H, V, beam, strong, elapsed, kernel_ms,
           (lab, ln, lp), (kcap, desc["decode_waves"], 0), weights, hid0, em0, em_last,
           {"pipeline_batch": Bp, "batches_per_step": nsub, "coalesce": cg,
            "inflight_decodes": desc["inflight"], "production_streams": desc["prod_streams"],
            "decode_cus": desc["decode_cus"], "fused_emission": fused,
            "recurrence": desc["recurrence"], "streams": desc["streams"], "hw_queues": desc["hw_queues"],
            "shared_queue_streams": desc.get("shared_queue_streams"),
            "segments": desc.get("segments"), "drain_held_batches": desc.get("drain_held_batches"),
            "first_segment_share": desc.get("first_segment_share"),
            "decode_cu_gemm_rows": desc["decode_cu_gemm_rows"],
            "stages": stages, "clock": clock_fig, "cu_placement": placement, "serialized": ser, "host": host,
            "pipeline": f"native asr_pipeline ({desc['mode']}): {desc['inflight']} decodes in flight on "
                        f"{desc['decode_cus']} CUs, {desc['prod_streams']} production stream(s); "
                        f"library-owned streams, buffers and decoder schedule"},
           parity_src=(Bp, (lab_p, ln_p, lp_p)))
    pl.close()
    asr.synchronize()
    destroy_raw_streams()


def greedy_host(T, V, first, count, seed=20261015):
    """--dry-run-cpu stand-in for a rank's GPU decode: best-path (greedy) CTC
    over per-utterance random host logits (collapse repeats, drop blank 0).
    Plumbing only; never a measured or parity-checked path."""
    lab = np.zeros((count, T), np.int32)
    ln = np.zeros(count, np.int32)
    lp = np.zeros(count, np.float64)
    for b in range(count):
        e = np.random.default_rng(seed + first + b).standard_normal((T, V))
        a = e.argmax(1)
        seq = a[(a != 0) & np.r_[True, a[1:] != a[:-1]]]
        lab[b, :len(seq)] = seq
        ln[b] = len(seq)
        lp[b] = float(e.max(1).sum())
    return lab, ln, lp


def dry_run_cpu(cfg, rank, world):
    """main()'s multi-rank plumbing with no GPU: gloo rendezvous, the shard
    plan, each rank's hypotheses gathered to rank 0, merged, counted and
    checked against one process's result for the whole batch; rank 0 prints
    one JSON line (n_gpus, gather) without a throughput value."""
    T, V = cfg["T"], cfg["vocab"]
    strong = "global_batch" in cfg
    GB = cfg["global_batch"] if strong else cfg["batch"] * world
    first, B = shard_range(rank, world, GB) if strong else (shard_first(rank, cfg["batch"]), cfg["batch"])
    if world > 1:
        init_gloo(rank, world)
        dist.barrier()
    t0 = time.perf_counter()
    lab, ln, lp = greedy_host(T, V, first, B)
    elapsed = reduce_max_over_ranks(time.perf_counter() - t0, world)
    records = gather_hypotheses(pack_hypotheses(first, lab, ln, lp), world, rank)
    if rank == 0:
        hyps, lps = merge_records(records)
        if len(hyps) != GB:
            raise AssertionError(f"gathered {len(hyps)} hypotheses, expected {GB}")
        ref = pack_hypotheses(0, *greedy_host(T, V, 0, GB))
        ok = hyps == ref[1] and np.array_equal(lps, np.asarray(ref[2]))
        if not ok:
            raise AssertionError("gathered hypotheses differ from the 1-process result")
        print(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": world,
                          "dry_run": True, "scaling": "strong" if strong else "weak",
                          "host_seconds": round(elapsed, 4),
                          "config": {"global_batch": GB, "T": T, "vocab": V},
                          "gather": {"utterances": len(hyps), "digest": hyp_digest(hyps, lps)[:16],
                                     "verified_vs_1process": True}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cu_masked_streams(mode, B=0):
    """Two HIP streams restricted to disjoint sets of the GPU's CUs
    (hipExtStreamCreateWithCUMask), wrapped as torch external streams:
    (production, decode).  half: [0, n/2) decodes; fit: [0, B rounded up
    to 8) decodes (one workgroup per utterance); interleave: even CUs."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    words = (ncu + 31) // 32
    masks = []
    for half in (0, 1):
        m = [0] * words
        for cu in range(ncu):
            if mode == "half":
                take = cu < ncu // 2
            elif mode == "fit":
                take = cu < min(ncu, -(-B // 8) * 8)
            else:
                take = cu % 2 == 0
            if take == (half == 1):
                m[cu // 32] |= 1 << (cu % 32)
        masks.append((ctypes.c_uint32 * words)(*m))
    out = []
    for m in masks:
        st = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), m)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
        _RAW_STREAMS.append((hip, st.value))
        out.append(torch.cuda.ExternalStream(st.value))
    return out[0], out[1]


def cu_group_streams(D, gcu, ncu):
    """D decode streams restricted to the disjoint CU ranges [j*gcu, (j+1)*gcu)
    and one production stream on [D*gcu, ncu) (hipExtStreamCreateWithCUMask),
    wrapped as torch external streams: (production, [decode...])."""
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ncu + 31) // 32
    ranges = [(j * gcu, (j + 1) * gcu) for j in range(D)] + [(D * gcu, ncu)]
    out = []
    for lo, hi in ranges:
        m = [0] * words
        for cu in range(lo, hi):
            m[cu // 32] |= 1 << (cu % 32)
        st = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words),
                                              (ctypes.c_uint32 * words)(*m))
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
        _RAW_STREAMS.append((hip, st.value))
        out.append(torch.cuda.ExternalStream(st.value))
    return out[-1], out[:-1]


def cu_range_stream(lo, hi):
    """One HIP stream restricted to CUs [lo, hi), as a torch external stream."""
    return cu_ranges_stream([(lo, hi)])


def cu_ranges_stream(ranges):
    """One HIP stream restricted to the union of CU ranges [lo, hi)."""
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    words = (ncu + 31) // 32
    m = [0] * words
    for lo, hi in ranges:
        for cu in range(lo, hi):
            m[cu // 32] |= 1 << (cu % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), (ctypes.c_uint32 * words)(*m))
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    _RAW_STREAMS.append((hip, st.value))
    return torch.cuda.ExternalStream(st.value)


_RAW_STREAMS = []


def destroy_raw_streams():
    """Destroy the CU-masked streams before the HIP runtime tears down (a
    stream left to the runtime's exit handlers crashed a profiled run)."""
    while _RAW_STREAMS:
        hip, st = _RAW_STREAMS.pop()
        hip.hipStreamSynchronize(ctypes.c_void_p(st))
        hip.hipStreamDestroy(ctypes.c_void_p(st))


def measure_gemms(asr, d_x, d_wih, d_hid, d_wout, d_bout, d_emis, T, B, In, H, V, reps=10, fused=None):
    """MFMA utilisation of the dense stages of a step, timed live with HIP
    events on torch's current stream after the timed region: the hoisted input
    projection x.W_ih ([T*B, In] x [In, H]), the emission projection with its
    fused bias + log_softmax ([T*B, H] x [H, V]), and — when the pipeline fuses
    it (fused = (W_hh, b_ih, b_hh)) — the recurrence + emission kernel
    (asr_rnn_emit_fwd, T steps of [B x H] . [H x (H + V)]; one launch on the
    whole chip, so its utilisation is that of ceil(B / 16) CUs' worth of work
    spread over the launch time)."""
    st = torch.cuda.current_stream()
    split = asr.get_dense_arith() == asr.DENSE_SPLIT_BF16
    out = {"arith": "split_bf16" if split else "f32",
           "note": "tflops = the stage's fp32 FLOP / s.  On the split arithmetic each fp32 product is 6 bf16 "
                   "MFMA products: mfma_util = 6 x tflops over the dense bf16 peak (the matrix cores' real "
                   "use); fp32_equiv_vs_fp32_peak = tflops over the fp32 MFMA peak (can exceed 1: fp32 "
                   "results from bf16 matrix cores, not fp32 MFMA utilisation)" if split
                   else "tflops = fp32 FLOP / s; mfma_util against the fp32 MFMA peak"}
    stages = [
        ("input_gemm", lambda: asr.linear_fwd(d_x, d_wih, None, d_hid, asr.EPI_NONE, st.cuda_stream),
         2.0 * T * B * In * H),
        ("emission_gemm", lambda: asr.linear_fwd(d_hid, d_wout, d_bout, d_emis, asr.EPI_BIAS_LOGSOFTMAX,
                                                 st.cuda_stream), 2.0 * T * B * H * V)]
    if fused is not None:
        whh, bih, bhh = fused
        stages.append(("recurrence_emission", lambda: asr.rnn_emit_fwd(whh, bih, bhh, d_wout, d_bout, d_hid,
                                                                       d_emis, T, B, stream=st.cuda_stream),
                       2.0 * T * B * H * (H + V)))
    for name, fn, flops in stages:
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / reps
        tf = flops / (us * 1e-6) / 1e12
        hbm = 4.0 * (T * B * (In if name == "input_gemm" else H) + T * B * (H if name == "input_gemm" else V))
        out[name] = {"us": round(us, 2), "tflops": round(tf, 2),
                     "mfma_util": round(tf / FP32_MFMA_PEAK_TF, 4),
                     "hbm_gbs": round(hbm / (us * 1e-6) / 1e9, 1)}
        if split and name != "emission_gemm":   # fp32 work on the bf16 matrix cores, 6 products each
            out[name]["fp32_equiv_vs_fp32_peak"] = out[name]["mfma_util"]
            out[name]["bf16_mfma_tflops"] = round(SPLIT_PRODUCTS * tf, 1)
            out[name]["mfma_util"] = round(SPLIT_PRODUCTS * tf / BF16_MFMA_PEAK_TF, 4)
            out[name]["peak"] = "dense bf16 MFMA"
        if name == "recurrence_emission":   # per busy CU: one 16-utterance workgroup per CU
            busy = min(-(-B // 16), torch.cuda.get_device_properties(st.device).multi_processor_count)
            ncu = torch.cuda.get_device_properties(st.device).multi_processor_count
            peak = BF16_MFMA_PEAK_TF / SPLIT_PRODUCTS if split else FP32_MFMA_PEAK_TF
            out[name]["mfma_util_busy_cus"] = round(tf / (peak * busy / ncu), 4)
            out[name]["busy_cus"] = busy
    return out


def parity_sample_ids(B: int, S: int):
    """S utterance ids spread evenly over [0, B) (first and last included)."""
    return sorted({int(round(v)) for v in np.linspace(0, B - 1, max(1, min(S, B)))})


def cpu_baseline(asr, d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout, T, B, In, H, V, beam, emis_host, best,
                 full_T=False, emis_note=""):
    """The CPU restatement of CTCBeamSearch.cpp (oracle/ctc_oracle.cpp, the
    reference's std::set/std::map algorithm with fixes F1-F3 in fp64 log
    domain, CTCBeamSearch.cpp:50-187) timed on this host's allotted cores over
    a bounded sample of the emissions the timed region's last batch decoded
    (emis_host [T][B][V]): one utterance per thread, spread over the batch.
    When the sample covers every frame (C4: T = 1000) the oracle's answers
    are also the parity witness of the measured path: each sampled
    utterance's best labels must equal the GPU's (`best` = that batch's
    collected labels / lengths / fp64 log-probs) and its log-prob agree to
    1e-9 relative (the tests' tolerance; north_star asks 1e-4).  Decoder
    only: the reference has no CPU RNN."""
    oracle = _load("ctc_oracle", ROOT / "oracle" / "ctc_oracle.py")
    threads, quota = cpu_share()
    ids = parity_sample_ids(B, threads)
    S = len(ids)
    emis = np.ascontiguousarray(emis_host.reshape(T, B, V)[:, ids, :])
    # ~20 s of CPU at C4's shape; longer shapes decode a prefix of the frames
    # (C5), unless --cpu-full-T
    Ts = T if full_T else min(T, max(4, int(2.6e7 / (S * (beam + 1) * (V + 1)))))
    t0 = time.perf_counter()
    ref = oracle.decode(emis[:Ts], beam, 0, is_log=True, nthreads=threads, max_hyps=1)
    secs = time.perf_counter() - t0
    out = {"value": round(S * Ts / secs, 1), "unit": "frames/s", "cores": threads, "kind": "port",
           "model": cpu_model(), "host_cpus": os.cpu_count(), "cgroup_quota_cpus": quota,
           "per_core": round(S * Ts / secs / min(S, threads), 1),
           "sample": f"oracle/ctc_oracle.cpp decode of {S} utterances (ids spread over the batch) x {Ts} "
                     f"frames of the emissions the timed region's last batch decoded (beam={beam}, V={V}), "
                     f"{threads} std::threads (one utterance each), {secs:.2f} s wall; decoder only "
                     f"(the reference has no CPU RNN)"}
    parity = {"utterances": S, "frames": Ts, "checked": Ts == T}
    if Ts == T:
        lab, ln, lp = best
        bad, worst = [], 0.0
        for i, u in enumerate(ids):
            rl, rlp = ref[i][0]
            got = lab[u, :int(ln[u])].tolist()
            err = abs(float(lp[u]) - rlp) / max(1.0, abs(rlp))
            worst = max(worst, err)
            if got != [int(c) for c in rl] or not err <= 1e-9:
                bad.append(u)
        parity.update({"match": not bad, "mismatched_ids": bad[:8], "max_logp_rel_err": worst,
                       "ids": ids if S <= 16 else ids[:8] + ["..."],
                       "tolerance": "best labels identical, |dlogp| <= 1e-9 max(1, |logp|)",
                       "emissions": emis_note or "the emissions the decode consumed",
                       "checker": "oracle/ctc_oracle.cpp (CTCBeamSearch.cpp:50-187, F1-F3, fp64 log domain)"})
    else:
        parity["note"] = f"the CPU sample is a {Ts}-frame prefix of T={T}: no parity claim from it"
    out["parity"] = parity
    if V == 29 and beam == 50 and T != 1000:
        # C4 shape (T=1000, beam=50): emissions from the same model at T=1000
        T4 = 1000
        x4 = asr.DeviceMatrix.from_numpy(make_features(T4, S, In, 0))
        e4 = asr.DeviceMatrix(T4 * S, V)
        asr.model_emissions(x4, [d_wih, d_whh, d_bih, d_bhh, d_wout, d_bout], T4, S, e4,
                            fused=H % 16 == 0 and V <= 32)
        em4 = e4.toCpu().reshape(T4, S, V)
        s4 = oracle.time_decode(em4, beam, 0, is_log=True, nthreads=threads)
        out["c4_shape"] = {"value": round(S * T4 / s4, 1), "unit": "frames/s", "cores": threads,
                           "sample": f"{S} utterances x {T4} frames, beam=50, V=29, {s4:.2f} s wall"}
    return out


if __name__ == "__main__":
    main()

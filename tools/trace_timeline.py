"""Summarise a rocprofv3 kernel trace (kernel_trace.csv) of a pipelined bench
run: per kernel family the launches, mean duration and the busy time of
the union of its launches, and over the last `--window` ms of the trace the
mean number of launches of each family in flight (how many decodes /
recurrences actually overlapped) and the gap between consecutive starts.
    python tools/trace_timeline.py gpurun_out/prof_r3t_g256/trace/.../run_kernel_trace.csv
"""
import argparse
import csv
import re
from collections import defaultdict

FAMILIES = [("decode", r"ctc_wave_kernel|ctc_beam_kernel|ctc_wide_kernel"),
            ("recurrence", r"rnn_recur|rnn_step"),
            ("gemm", r"gemm_"),
            ("traceback", r"ctc_best|ctc_all|ctc_trace"),
            ("other", r".")]


def family(name):
    for f, pat in FAMILIES:
        if re.search(pat, name):
            return f
    return "other"


def union_ms(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.0, help="analyse only the last W ms of the decodes' span (0 = all)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows
          if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    ks.sort()
    dec = [k for k in ks if family(k[2]) == "decode"]   # the pipelined region: the decodes' span
    span_ks = dec or ks
    t_end = max(e for _, e, _, _ in span_ks)
    t_beg = t_end - int(a.window * 1e6) if a.window > 0 else min(s for s, _, _, _ in span_ks)
    ks = [(s, min(e, t_end), n, q) for s, e, n, q in ks if e > t_beg and s < t_end]
    span = (t_end - t_beg) / 1e6
    by = defaultdict(list)
    for s, e, n, q in ks:
        by[family(n)].append((max(s, t_beg), e, n, q))
    print(f"window {span:.3f} ms, {len(ks)} launches")
    for f, _ in FAMILIES:
        if f not in by:
            continue
        iv = [(s, e) for s, e, _, _ in by[f]]
        durs = [(e - s) / 1e6 for s, e in iv]
        inflight = sum(durs) / span
        starts = sorted(s for s, _ in iv)
        gaps = [(b - a_) / 1e6 for a_, b in zip(starts, starts[1:])]
        names = sorted({n.split("(")[0][:60] for _, _, n, _ in by[f]})
        queues = sorted({q for _, _, _, q in by[f]})
        print(f"{f:10s} n={len(iv):5d} mean={sum(durs) / len(durs):8.3f} ms busy(union)={union_ms(iv):8.3f} ms "
              f"mean in flight={inflight:5.2f} start gap={(sum(gaps) / len(gaps)) if gaps else 0:7.3f} ms "
              f"queues={len(queues)} {names[:3]}")


if __name__ == "__main__":
    main()

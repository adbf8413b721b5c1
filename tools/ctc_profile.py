"""Decoder timing sweep (waves per utterance x workload) and, with
ASR_LIB=libasr_amd_stamps.so, the per-phase shader-clock breakdown.

    python tools/ctc_profile.py            # timings
    ASR_LIB=libasr_amd_stamps.so python tools/ctc_profile.py --stamps
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")
oracle = _load("ctc_oracle", ROOT / "oracle" / "ctc_oracle.py")

PHASES = ["chunk", "P1 cand", "P2a folds>=G", "P2b select", "P2c fallback", "P3a scan",
          "P3b+barrier", "n:orphan inserts", "n:orphan filter hits", "n:extensions", "radix:pre-barrier",
          "radix:barrier", "radix:post", "-", "-", "-"]
WIDE_PHASES = ["staging+pool", "tile threshold", "tile labels+child", "stage1", "exact+stage2",
               "pool write", "slots", "n:tiles", "candidates", "n:keys in stage-1 window", "radix:pre-barrier", "radix:barrier",
               "radix:post", "-", "-", "-"]   # ctc_wide_kernel.inc (V > 63)
COUNTERS = True   # slots 13-15 of the stamps build are counters


WPOINTS = {1: "P1 cand", 2: "folds>=G", 3: "select", 4: "fallback/cu", 7: "at offsets barrier",
           5: "offsets done", 8: "own prefixes", 9: "desc written", 10: "ext built", 6: "frame end",
           11: "sel: atomics start", 12: "sel: atomics issued", 13: "sel: barrier passed",
           14: "sel: pass-0 decision"}


def bench_emissions(T, B, V, H=256):
    """Log-probability emissions of bench.py's model (RNN -> Linear +
    log_softmax, random-init weights), as the headline bench decodes them."""
    import bench
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    hid, em = asr.DeviceMatrix(T * B, H), asr.DeviceMatrix(T * B, V)
    asr.rnn_fwd(DM(bench.make_features(T, B, H, 0)), DM(w_ih), DM(w_hh), DM(b_ih.reshape(H, 1)),
                DM(b_hh.reshape(H, 1)), hid, T, B)
    asr.linear_fwd(hid, DM(w_out), DM(b_out.reshape(V, 1)), em, asr.EPI_BIAS_LOGSOFTMAX)
    return em.toCpu().reshape(T, B, V)


def run(T, B, V, beam, sigma, waves, reps, stamps, wstamps=False):
    is_log = sigma == "bench"
    emis = bench_emissions(T, B, V) if is_log else oracle.synthetic_emissions(T, B, V, sigma=sigma)
    dec = asr.CTCDecoder(V, beam, 0, waves=waves)
    ms = []
    for _ in range(reps):
        dec.decode(emis, is_log=is_log)
        try:
            dec.best(allow_overflow=True)
        except asr.AsrError:   # ablation builds (timing only) may fail their self-checks
            pass
        ms.append(dec.last_kernel_ms())
    out = {"T": T, "B": B, "V": V, "beam": beam, "sigma": sigma, "waves": dec.config()[1],
           "lds": dec.config()[2], "kernel_ms_min": round(min(ms), 4),
           "us_per_frame_step": round(1e3 * min(ms) / T, 3)}
    if wstamps:   # per-wave arrival clocks (libasr_amd_wstamps.so)
        L = asr.lib()
        nw = dec.config()[1]
        buf = np.zeros((B, 9, 16), np.uint64)
        fn = L.asr_debug_ctc_stamps
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        asr.check(fn(dec.h, buf.ctypes.data), "stamps")
        frames = buf[:, :nw, 0].astype(np.float64).sum(axis=0)   # per wave
        per = buf[:, :nw, :].astype(np.float64).sum(axis=0) / frames[:, None]
        order = sorted(WPOINTS, key=lambda i: per[0, i])
        out["arrival_cycles_by_wave"] = {WPOINTS[i]: [round(x) for x in per[:, i]] for i in order}
        # critical path: per frame, the last wave's arrival at each point
        # (relative to wave 0's frame start), averaged over frames
        crit = buf[:, 8, :].astype(np.float64).sum(axis=0) / max(1.0, buf[:, 8, 0].astype(np.float64).sum())
        out["last_wave_arrival"] = {WPOINTS[i]: round(crit[i]) for i in sorted(WPOINTS, key=lambda i: crit[i])}
    if stamps and dec.config()[1] == -1:   # one-wave kernel: phase clocks and counters
        L = asr.lib()
        buf = np.zeros((B, 16), np.uint64)
        fn = L.asr_debug_ctc_stamps
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        asr.check(fn(dec.h, buf.ctypes.data), "stamps")
        per = buf.astype(np.float64).mean(axis=0) / T
        names = ["staging", "rows+own", "folds", "labels+keys", "select", "survivors", "own build",
                 "ext build", "n:registered labels", "n:regenerated labels", "n:fallbacks", "n:extensions",
                 "n:selection passes", "n:keys >= floor"]
        out["wave_cycles_per_frame"] = {names[i]: round(per[i], 1) for i in range(8)}
        out["wave_events_per_frame"] = {names[i][2:]: round(per[i], 3) for i in range(8, 14)}
        out["cycles_total"] = round(per[:8].sum(), 1)
    elif stamps:
        L = asr.lib()
        buf = np.zeros((B, 16), np.uint64)
        fn = L.asr_debug_ctc_stamps
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        asr.check(fn(dec.h, buf.ctypes.data), "stamps")
        per = buf.astype(np.float64).mean(axis=0) / T
        PH = WIDE_PHASES if V + 1 > 64 else PHASES
        out["cycles_per_step"] = {PH[i]: round(per[i], 1) for i in range(13)
                                  if PH[i] != "-" and not PH[i].startswith("n:")}
        out["events_per_frame"] = {PH[i][2:]: round(per[i], 2) for i in range(13) if PH[i].startswith("n:")}
        if PH is WIDE_PHASES:   # slot 9: window keys | (row, column) pairs listed << 32
            out["events_per_frame"]["keys in stage-1 window"] = round(float((buf[:, 9] & 0xFFFFFFFF).mean()) / T, 2)
            out["events_per_frame"]["pairs listed"] = round(float((buf[:, 9] >> 32).mean()) / T, 2)
        ranks = (buf[:, 15] & 0xFFFFFFFF).astype(np.float64)
        out["per_frame"] = {("stage1_passes" if PH is WIDE_PHASES else "fallbacks"): round(per[13], 4),
                            "exact_passes": round(per[14], 3),
                            "ranks": round(ranks.mean() / T, 3),
                            "mean_cd": round(float((buf[:, 15] >> 32).sum() / max(1.0, ranks.sum())), 2)}
        out["cycles_total"] = round(per[:7].sum() + (per[8] if PH is WIDE_PHASES else 0.0), 1)
    dec.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--wstamps", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--waves", default="1,2,4", help="waves per utterance; -1 = the one-wave kernel")
    ap.add_argument("--cases", default="c2,c3")
    ap.add_argument("--sigmas", default="3,0.5,bench", help="synthetic emission spreads; 'bench' = bench.py's model")
    args = ap.parse_args()
    global WAVES, SIGMAS
    WAVES = [int(x) for x in args.waves.split(",")]
    SIGMAS = [x if x == "bench" else float(x) for x in args.sigmas.split(",")]
    asr.set_device(0)
    ap_cases = {"c2": (500, 64, 29, 50), "c3": (1000, 256, 29, 100),
                "s64": (300, 64, 29, 50), "s768": (300, 768, 29, 50),   # alone / three per CU
                "s4096": (300, 4096, 29, 50),   # 16 per CU (the one-wave kernel's occupancy)
                "c5": (2000, 32, 1000, 200)}   # C5: 32 utterances per GPU
    ap_cases = [ap_cases[c] for c in args.cases.split(",")]
    for (T, B, V, beam) in ap_cases:
        for sigma in SIGMAS:
            for waves in WAVES:
                print(json.dumps(run(T, B, V, beam, sigma, waves, args.reps, args.stamps, args.wstamps)), flush=True)


if __name__ == "__main__":
    main()

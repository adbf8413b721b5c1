"""Decode throughput vs workgroups per CU (the lever for batch throughput):
for each schedule (waves per utterance; -1 = the one-wave list kernel) and
batch B = k x CUs, the beam-search kernel time on bench.py's emissions and
the per-CU throughput in utterance-frames per microsecond.

    python tools/occupancy_sweep.py [--T 300] [--k 1,2,3,4] [--waves 8,4,-1] [--beam 50]
    ASR_LIB=libasr_amd_wpe3.so python tools/occupancy_sweep.py ...   # a register-budget build
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=300)
    ap.add_argument("--k", default="1,2,3,4")
    ap.add_argument("--waves", default="8,4")
    ap.add_argument("--beam", type=int, default=50)
    ap.add_argument("--V", type=int, default=29)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    asr.set_device(0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    from ctc_profile import bench_emissions
    ks = [int(x) for x in args.k.split(",")]
    Bmax = max(ks) * ncu
    emis = bench_emissions(args.T, Bmax, args.V)
    d_em = asr.DeviceMatrix.from_numpy(emis.reshape(args.T * Bmax, args.V))
    lib = os.environ.get("ASR_LIB", "libasr_amd.so")
    ref = {}
    for w in [int(x) for x in args.waves.split(",")]:
        for k in ks:
            B = k * ncu
            dec = asr.CTCDecoder(args.V, args.beam, 0, waves=w)
            ms = []
            for _ in range(args.reps):
                dec.decode_device(d_em.ptr, args.T, B, True, frame_stride=Bmax * args.V, utt_stride=args.V)
                lab, lp = dec.best()
                ms.append(dec.last_kernel_ms())
            cfg = dec.config()
            dec.close()
            key = (k,)
            same = None
            if key in ref:
                same = ref[key] == (lab, lp.tobytes())
            else:
                ref[key] = (lab, lp.tobytes())
            t = min(ms)
            print(json.dumps({"lib": lib, "waves": cfg[1], "B": B, "per_cu": k, "T": args.T,
                              "kernel_ms": round(t, 4), "us_per_frame": round(1e3 * t / args.T, 3),
                              "utt_frames_per_us_per_cu": round(B * args.T / (t * 1e3) / ncu, 4),
                              "frames_per_s": round(B * args.T / (t * 1e-3)),
                              "lds": cfg[2], "same_as_first_schedule": same}), flush=True)


if __name__ == "__main__":
    main()

"""A/B of a wide-decoder variant (ASR_LIB selects the library): decode of
bench-model emissions (V = 1000, beam = 200, 8 waves), kernel time and a
digest of every utterance's ranked beam (labels and log-probabilities), so
that two builds can be compared for speed and bit-identity.

    ASR_LIB=libasr_amd_cv_x.so python tools/wide_ab.py --T 500 --out a.json
"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import ctc_profile as cp  # noqa: E402  (loads asr_amd with ASR_LIB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--V", type=int, default=1000)
    ap.add_argument("--beam", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    asr = cp.asr
    asr.set_device(0)
    emis = cp.bench_emissions(args.T, args.B, args.V)
    dec = asr.CTCDecoder(args.V, args.beam, 0, waves=8)
    ms = []
    for _ in range(args.reps):
        dec.decode(emis, is_log=True)
        dec.best(allow_overflow=True)
        ms.append(dec.last_kernel_ms())
    m = hashlib.sha256()
    for hyps in dec.beams(args.beam + 8):
        for lab, lp in hyps:
            m.update(np.asarray(lab, np.int32).tobytes())
            m.update(np.float64(lp).tobytes())
        m.update(b"|")
    out = {"T": args.T, "B": args.B, "kernel_ms_min": round(min(ms), 4),
           "us_per_frame": round(1e3 * min(ms) / args.T, 3), "beams_sha256": m.hexdigest()}
    Path(args.out).write_text(json.dumps(out))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

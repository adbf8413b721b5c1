"""Recurrence-only timing (asr_rnn_recur_fwd, H <= 256): the VALU kernel
(one utterance per CU) vs the MFMA kernel (16 utterances per workgroup) over
batch sizes, forced with ASR_RNN_MFMA, and the automatic choice.

    python tools/rnn_recur_sweep.py [--T 1000] [--H 256] [--B 64,256,512,1024,2048]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--B", default="64,256,512,1024,2048")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    asr.set_device(0)
    rng = np.random.default_rng(0)
    T, H = a.T, a.H
    s = 1 / np.sqrt(H)
    DM = asr.DeviceMatrix.from_numpy
    whh = DM(rng.uniform(-s, s, (H, H)).astype(np.float32))
    bih, bhh = DM(np.zeros((H, 1), np.float32)), DM(np.zeros((H, 1), np.float32))
    for B in [int(x) for x in a.B.split(",")]:
        hid = asr.DeviceMatrix(T * B, H)
        row = {"T": T, "H": H, "B": B}
        for mode in ("0", "1", None):
            if mode is None:
                os.environ.pop("ASR_RNN_MFMA", None)
            else:
                os.environ["ASR_RNN_MFMA"] = mode
            best = 1e30
            for _ in range(a.reps):
                asr.synchronize()
                t0 = time.perf_counter()
                asr.rnn_recur_fwd(whh, bih, bhh, hid, T, B)
                asr.synchronize()
                best = min(best, time.perf_counter() - t0)
            row[{"0": "valu_ms", "1": "mfma_ms", None: "auto_ms"}[mode]] = round(1e3 * best, 3)
        row["utt_steps_per_us_valu"] = round(B * T / (row["valu_ms"] * 1e3), 2)
        row["utt_steps_per_us_mfma"] = round(B * T / (row["mfma_ms"] * 1e3), 2)
        print(json.dumps(row), flush=True)
        hid.free()


if __name__ == "__main__":
    main()

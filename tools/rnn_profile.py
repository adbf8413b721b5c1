"""Time the RNN forward at a given shape (default: C5 per GPU, H = in = 1024,
B = 32, T = 2000) — for rocprofv3 kernel stats of the recurrence path."""
import argparse
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
    ap.add_argument("--T", type=int, default=2000)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--H", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    asr.set_device(0)
    rng = np.random.default_rng(0)
    T, B, H = a.T, a.B, a.H
    s = 1 / np.sqrt(H)
    DM = asr.DeviceMatrix.from_numpy
    x = DM(rng.uniform(-1, 1, (T * B, H)).astype(np.float32))
    wih, whh = DM(rng.uniform(-s, s, (H, H)).astype(np.float32)), DM(rng.uniform(-s, s, (H, H)).astype(np.float32))
    bih, bhh = DM(np.zeros((H, 1), np.float32)), DM(np.zeros((H, 1), np.float32))
    hid = asr.DeviceMatrix(T * B, H)
    for r in range(a.reps):
        asr.synchronize()
        t0 = time.perf_counter()
        asr.rnn_fwd(x, wih, whh, bih, bhh, hid, T, B)
        asr.synchronize()
        print(f"rnn_fwd T={T} B={B} H={H}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()

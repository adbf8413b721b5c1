"""Time the MFMA recurrence alone (asr_rnn_recur_fwd) against the recurrence
with the emission layer fused (asr_rnn_emit_fwd) at a chip-filling shape
(default C4 one GPU: T = 1000, B = 2048, H = 256, V = 29), HIP events on
one stream, for A/B runs of the fused kernel's step schedule."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--V", type=int, default=29)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    asr.set_device(0)
    asr.rnn_set_recurrence(asr.RNN_RECUR_MFMA)
    rng = np.random.default_rng(0)
    T, B, H, V = a.T, a.B, a.H, a.V
    s = 1 / np.sqrt(H)
    DM = asr.DeviceMatrix.from_numpy
    P = DM(rng.uniform(-1, 1, (T * B, H)).astype(np.float32))
    whh = DM(rng.uniform(-s, s, (H, H)).astype(np.float32))
    bih, bhh = DM(np.zeros((H, 1), np.float32)), DM(np.zeros((H, 1), np.float32))
    wo, bo = DM(rng.uniform(-4 * s, 4 * s, (H, V)).astype(np.float32)), DM(np.zeros((V, 1), np.float32))
    hid, em = asr.DeviceMatrix(T * B, H), asr.DeviceMatrix(T * B, V)
    st = torch.cuda.current_stream()
    out = {"T": T, "B": B, "H": H, "V": V}
    for name, fn in (("recurrence", lambda: asr.rnn_recur_fwd(whh, bih, bhh, hid, T, B, stream=st.cuda_stream)),
                     ("recurrence_emission", lambda: asr.rnn_emit_fwd(whh, bih, bhh, wo, bo, P, em, T, B,
                                                                      stream=st.cuda_stream))):
        fn()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        out[name + "_ms"] = round(min(ms), 4)
        out[name + "_us_per_step"] = round(1e3 * min(ms) / T, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Recurrence step time for H > 256 (the per-frame step kernels; C5: B = 32,
H = 1024, T = 2000; BL: B = 256, H = 2048, T = 200): asr_rnn_recur_fwd alone
on an idle GPU, whole chip, HIP events; prints one JSON line per shape.
    python tools/step_time.py [B:H:T ...]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from conftest import asr  # noqa: E402
import torch  # noqa: E402

shapes = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(32, 1024, 2000), (256, 2048, 200)]
dm = asr.DeviceMatrix.from_numpy
for B, H, T in shapes:
    rng = np.random.default_rng(0)
    s = 1 / np.sqrt(H)
    W = [dm(rng.uniform(-s, s, sh).astype(np.float32)) for sh in [(H, H), (H, 1), (H, 1)]]
    P0 = rng.uniform(-1, 1, (T * B, H)).astype(np.float32)
    hid = dm(P0)
    st = torch.cuda.Stream()
    asr.rnn_recur_fwd(*W, hid, T, B, stream=st.cuda_stream)   # warm-up (hid is overwritten: timing only)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record(st)
    for _ in range(reps):
        asr.check(asr.lib().asr_rnn_recur_fwd(None, W[0].ptr, W[1].ptr, W[2].ptr, hid.ptr, T, B, H, st.cuda_stream),
                  "recur")
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"B": B, "H": H, "T": T, "ms": round(ms, 3), "us_per_step": round(1e3 * ms / T, 2)}), flush=True)

"""C5 recurrence (T=2000, B=32, H=in=1024): wall ms of asr_rnn_fwd, for rocprofv3."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from conftest import asr  # noqa: E402

T, B, H = 2000, 32, 1024
rng = np.random.default_rng(0)
s = 1 / np.sqrt(H)
dm = asr.DeviceMatrix.from_numpy
p = [dm(rng.uniform(-s, s, sh).astype(np.float32)) for sh in [(H, H), (H, H), (H, 1), (H, 1)]]
x = dm(rng.uniform(-1, 1, (T * B, H)).astype(np.float32))
hid = asr.DeviceMatrix(T * B, H)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
asr.rnn_fwd(x, *p, hid, T, B)
asr.lib().asr_device_sync()
t0 = time.perf_counter()
for _ in range(reps):
    asr.rnn_fwd(x, *p, hid, T, B)
asr.lib().asr_device_sync()
print(f"C5 rnn_fwd T={T} B={B} H={H}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms", flush=True)

"""Wall time of asr_rnn_bidir_fwd vs two asr_rnn_fwd calls (C2 / C5 shapes)."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from conftest import asr  # noqa: E402


def run(T, B, H, reps=5):
    rng = np.random.default_rng(0)
    s = 1 / np.sqrt(H)
    dm = asr.DeviceMatrix.from_numpy
    p = [tuple(dm(rng.uniform(-s, s, sh).astype(np.float32)) for sh in [(H, H), (H, H), (H, 1), (H, 1)])
         for _ in range(2)]
    x = dm(rng.uniform(-1, 1, (T * B, H)).astype(np.float32))
    out = asr.DeviceMatrix(T * B, 2 * H)
    hid = asr.DeviceMatrix(T * B, H)
    work = asr.DeviceBytes(asr.lib().asr_rnn_bidir_workspace_bytes(T, B, H))
    res = {}
    for name, fn in [("bidir", lambda: asr.rnn_bidir_fwd(x, p, out, T, B, work=work)),
                     ("2x_unidir", lambda: [asr.rnn_fwd(x, *p[d], hid, T, B) for d in range(2)])]:
        fn(); asr.lib().asr_device_sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        asr.lib().asr_device_sync()
        res[name] = (time.perf_counter() - t0) / reps * 1e3
    print(f"T={T} B={B} H={H}: " + ", ".join(f"{k} {v:.3f} ms" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    run(500, 64, 256)
    run(2000, 32, 1024, reps=2)

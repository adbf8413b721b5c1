"""The split-bf16 production kernels alone, in process (for rocprofv3 --pmc),
on the 128 production CUs at C4's 1024-utterance batch: the input projection
(M = 1,024,000, K = N = 256; REPS launches) and the fused recurrence +
emission (T = 200 steps, one launch per rep).
    python tools/gemm_probe.py [REPS] [gemm|recur|both]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import bench  # noqa: E402
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")
asr.set_device(0)
torch.cuda.set_device(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
what = sys.argv[2] if len(sys.argv) > 2 else "both"
T, B, H = 1000, 1024, 256
w = np.random.default_rng(3).uniform(-0.06, 0.06, (H, H)).astype(np.float32)
x = asr.DeviceMatrix.from_numpy(np.random.default_rng(1).uniform(-1, 1, (T * B, H)).astype(np.float32))
W = asr.DeviceMatrix.from_numpy(w)
P = asr.DeviceMatrix(T * B, H)
st = bench.cu_range_stream(128, 256)
L = asr.lib()
if what in ("gemm", "both"):
    for _ in range(reps):
        asr.check(L.asr_linear_fwd(x.ptr, W.ptr, None, P.ptr, T * B, H, H, asr.EPI_NONE, st.cuda_stream), "gemm")
if what in ("recur", "both"):
    V, T2 = 29, 200
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    dw = [DM(w_hh), DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1)), DM(w_out), DM(b_out.reshape(V, 1))]
    em = asr.DeviceMatrix(T2 * B, V)
    for _ in range(reps):
        asr.check(L.asr_rnn_emit_fwd(None, dw[0].ptr, dw[1].ptr, dw[2].ptr, dw[3].ptr, dw[4].ptr, P.ptr, None,
                                     em.ptr, T2, B, H, V, st.cuda_stream), "rnn_emit")
torch.cuda.synchronize()
bench.destroy_raw_streams()
print("ok", flush=True)

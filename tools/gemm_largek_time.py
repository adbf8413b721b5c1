"""Timing of the large-K dense GEMMs (K > 256: C5's input projection
[64000, 1024] x [1024, 1024] and emission layer [64000, 1024] x [1024, 1000]
+ log_softmax; BL's input projection [51200, 2048] x [2048, 2048]) on the
split-bf16 arithmetic against the fp32 MFMA kernels, whole chip, HIP events.

    python tools/gemm_largek_time.py
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from __graft_entry__ import PKG, _load
    asr = _load("asr_amd", PKG / "asr_amd.py")
    asr.set_device(0)
    st = torch.cuda.current_stream()
    out = {}
    rng = np.random.default_rng(0)
    for name, M, K, N, epi in (("c5_input", 64000, 1024, 1024, asr.EPI_NONE),
                               ("c5_emission", 64000, 1024, 1000, asr.EPI_BIAS_LOGSOFTMAX),
                               ("bl_input", 51200, 2048, 2048, asr.EPI_NONE)):
        x = asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (M, K)).astype(np.float32))
        W = asr.DeviceMatrix.from_numpy((rng.uniform(-1, 1, (K, N)) / np.sqrt(K)).astype(np.float32))
        b = asr.DeviceMatrix.from_numpy(rng.uniform(-0.5, 0.5, (N, 1)).astype(np.float32))
        y = asr.DeviceMatrix(M, N)
        row = {}
        for kind, label in ((asr.DENSE_SPLIT_BF16, "split_bf16"), (asr.DENSE_F32, "f32")):
            asr.set_dense_arith(kind)
            fn = lambda: asr.linear_fwd(x, W, b, y, epi, st.cuda_stream)
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                fn()
            e1.record(st)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 5
            row[label] = {"ms": round(ms, 4), "fp32_equiv_tflops": round(2.0 * M * K * N / (ms * 1e-3) / 1e12, 1)}
        asr.set_dense_arith(asr.DENSE_SPLIT_BF16)
        row["speedup"] = round(row["f32"]["ms"] / row["split_bf16"]["ms"], 3)
        out[name] = row
        print(name, json.dumps(row), flush=True)
        del x, W, b, y


if __name__ == "__main__":
    main()

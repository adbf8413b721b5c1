"""A/B timing of the split-bf16 dense kernels across library builds
(Makefile `dvariant`): the RNN input projection (M = T*B rows, K = N = 256)
and the fused recurrence + emission (T = 1000) at the C4 pipeline's shapes —
on the 128 production CUs (a 1024-utterance batch) and on the whole chip —
plus each build's error against fp64 on sampled rows / utterances.

    python tools/dense_time.py base pf tanh ...   (base = libasr_amd.so)
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def child():
    sys.path.insert(0, str(ROOT))
    import torch
    import bench
    from __graft_entry__ import PKG, _load
    asr = _load("asr_amd", PKG / "asr_amd.py")
    asr.set_device(0)
    torch.cuda.set_device(0)
    T, H, V = 1000, 256, 29
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    dw = [DM(w_ih), DM(w_hh), DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1)), DM(w_out), DM(b_out.reshape(V, 1))]
    Bfull = 2048
    xh = np.random.default_rng(1).uniform(-1, 1, (T * Bfull, H)).astype(np.float32)
    x = DM(xh)
    P = asr.DeviceMatrix(T * Bfull, H)
    em = asr.DeviceMatrix(T * Bfull, V)
    half = bench.cu_range_stream(128, 256)
    full = torch.cuda.Stream()
    out = {}

    def timed(fn, st, reps):
        fn(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn(st)
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    L = asr.lib()

    def gemm(xp, yp, M, st):
        asr.check(L.asr_linear_fwd(xp, dw[0].ptr, None, yp, M, H, H, asr.EPI_NONE, st), "gemm")

    def remit(Pp, ep, B, st):
        asr.check(L.asr_rnn_emit_fwd(None, dw[1].ptr, dw[2].ptr, dw[3].ptr, dw[4].ptr, dw[5].ptr, Pp, None, ep,
                                     T, B, H, V, st), "rnn_emit")

    for name, B, st in (("half", 1024, half), ("full", 2048, full)):
        M = T * B
        g = timed(lambda s: gemm(x.ptr, P.ptr, M, s.cuda_stream), st, 10)
        r = timed(lambda s: remit(P.ptr, em.ptr, B, s.cuda_stream), st, 3)
        out[name] = {"gemm_ms": round(g, 4), "recur_emit_ms": round(r, 4), "us_per_step": round(1e3 * r / T, 3)}
    torch.cuda.synchronize()
    # accuracy vs fp64: GEMM rows, and a full recurrence + emission of 16 utterances
    gemm(x.ptr, P.ptr, T * Bfull, 0)
    torch.cuda.synchronize()
    rows = np.random.default_rng(2).choice(T * Bfull, 256, replace=False)
    Pr = P.toCpu().reshape(T * Bfull, H)[rows]
    out["gemm_bits"] = __import__("hashlib").sha1(np.ascontiguousarray(Pr).tobytes()).hexdigest()[:16]
    Pg = Pr.astype(np.float64)
    ref = xh[rows].astype(np.float64) @ w_ih.astype(np.float64)
    out["gemm_err_rel_abs_sum"] = float(np.max(np.abs(Pg - ref) / (np.abs(xh[rows]).astype(np.float64) @
                                                                   np.abs(w_ih).astype(np.float64))))
    B = 16
    xb = np.ascontiguousarray(xh.reshape(T, Bfull, H)[:, :B, :]).reshape(T * B, H)
    xd = DM(xb)
    Pb = asr.DeviceMatrix(T * B, H)
    eb = asr.DeviceMatrix(T * B, V)
    gemm(xd.ptr, Pb.ptr, T * B, 0)
    remit(Pb.ptr, eb.ptr, B, 0)
    torch.cuda.synchronize()
    e = eb.toCpu().reshape(T, B, V).astype(np.float64)
    xb3 = xb.reshape(T, B, H).astype(np.float64)
    h = np.zeros((B, H))
    W, U = w_ih.astype(np.float64), w_hh.astype(np.float64)
    bb = (b_ih + b_hh).astype(np.float64)
    Wo, bo = w_out.astype(np.float64), b_out.astype(np.float64)
    err = 0.0
    for t in range(T):
        h = np.tanh(xb3[t] @ W + h @ U + bb)
        z = h @ Wo + bo
        z = z - z.max(1, keepdims=True)
        ls = z - np.log(np.exp(z).sum(1, keepdims=True))
        err = max(err, float(np.abs(ls - e[t]).max()))
    out["emis_err_max_abs_T1000"] = err
    out["emis_checksum"] = float(np.abs(e).sum())
    print(json.dumps(out), flush=True)
    bench.destroy_raw_streams()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    for v in sys.argv[1:] or ["base"]:
        lib = "libasr_amd.so" if v == "base" else f"libasr_amd_dv_{v}.so"
        env = dict(os.environ, ASR_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else None
        print(json.dumps({"variant": v, "result": json.loads(line) if line else None,
                          "rc": r.returncode, "err": r.stderr[-400:] if r.returncode else ""}), flush=True)


if __name__ == "__main__":
    main()

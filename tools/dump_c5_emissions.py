"""Dump C5 production emissions for the full-length wide-decoder fixture
(tests/golden/make_c5_production_golden.py).

The bench's C5 model (bench.make_weights / make_features: H = in = 1024,
V = 1000, the 32-utterance per-GPU batch at T = 2000) run through the
library on the fp32 dense arithmetic (ASR_DENSE_F32: kernels this fixture
pins, independent of the split-bf16 tuning), log_softmax emissions
[T][32][V]; utterances UIDS are written to <out>/c5_emis.npy ([T][4][V]
float32) with the sha256 of each utterance's [T][V] bytes.

    python tools/dump_c5_emissions.py gpurun_out/c5fix
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from __graft_entry__ import PKG, _load  # noqa: E402

T, B, H, V, BEAM = 2000, 32, 1024, 1000, 200
UIDS = [0, 9, 18, 27]


def production_emissions(asr):
    """[T][B][V] float32 on the host (also used by the GPU test)."""
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    W = (DM(w_ih), DM(w_hh), DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1)), DM(w_out), DM(b_out.reshape(V, 1)))
    x = DM(bench.make_features(T, B, H, 0))
    prev = asr.get_dense_arith()
    asr.set_dense_arith(asr.DENSE_F32)
    try:
        em = asr.DeviceMatrix(T * B, V)
        asr.model_emissions(x, W, T, B, em, False)
        return em.toCpu().reshape(T, B, V), em
    finally:
        asr.set_dense_arith(prev)


def digest(e_tv: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(e_tv, np.float32).tobytes()).hexdigest()


def main():
    out = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5fix")
    out.mkdir(parents=True, exist_ok=True)
    asr = _load("asr_amd", PKG / "asr_amd.py")
    asr.set_device(0)
    e, _ = production_emissions(asr)
    sub = np.ascontiguousarray(e[:, UIDS, :])
    np.save(out / "c5_emis.npy", sub)
    meta = {"T": T, "B": B, "H": H, "V": V, "beam": BEAM, "utterances": UIDS,
            "sha256": [digest(e[:, u, :]) for u in UIDS]}
    (out / "c5_emis.json").write_text(json.dumps(meta, indent=1))
    print(json.dumps(meta))


if __name__ == "__main__":
    main()

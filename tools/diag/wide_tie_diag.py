"""Diagnostic: wide-kernel .cu tie cut on few-level emissions (status per path)."""
import os
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from __graft_entry__ import PKG, _load  # noqa: E402
asr = _load("asr_amd", PKG / "asr_amd.py")
asr.set_device(0)
for V in (100, 300):
    T, B, beam = 8, 2, 12
    rng = np.random.default_rng(V)
    logit = 0.5 * rng.integers(0, 3, size=(T, B, V)).astype(np.float64)
    q = np.exp(logit)
    emis = (q / q.sum(-1, keepdims=True)).astype(np.float32)
    for sem in (asr.SEMANTICS_CUDA, asr.SEMANTICS_CPU):
        for flag in ("0", "1"):
            os.environ["ASR_CTC_WIDE_FALLBACK"] = flag
            dec = asr.CTCDecoder(V, beam, 0)
            dec.set_semantics(sem)
            dec.decode(emis)
            try:
                bm = dec.beams(max_hyps=dec.config()[0])
                print(os.environ.get("ASR_LIB", "new"), V, sem, flag, "ok", [len(x) for x in bm],
                      hash(str(bm)) % 100000, flush=True)
            except Exception as e:
                print(os.environ.get("ASR_LIB", "new"), V, sem, flag, "ERR", e, flush=True)
            dec.close()

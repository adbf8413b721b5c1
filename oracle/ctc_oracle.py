"""TEST INFRASTRUCTURE ONLY — Python handle on the CPU parity oracle.

Loads oracle/libctc_oracle.so (built from oracle/ctc_oracle.cpp, a CPU
restatement of /root/reference/CTCBeamSearch.cpp; see its header for the
fixes and how it is pinned).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use this module, and only as the checker.

Also holds the synthetic emission generator used by tests and bench (the
same inputs go to the GPU and to the oracle).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "libctc_oracle.so"
SEED0 = 20261015

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        vp, i = ctypes.c_void_p, ctypes.c_int
        for name in ("oracle_ctc_decode", "oracle_ctc_decode_prob"):
            fn = getattr(L, name)
            fn.argtypes = [vp, i, i, i, i, i, vp, i, i, i, i, vp, vp, vp, vp]
            fn.restype = i
        L.oracle_ctc_decode_ts.argtypes = [vp, i, i, i, i, i, vp, i, i, i, i, vp, vp, vp, vp, vp]
        L.oracle_ctc_decode_ts.restype = i
        L.oracle_ctc_time.argtypes = [vp, i, i, i, i, i, i, i]
        L.oracle_ctc_time.restype = ctypes.c_double
        _lib = L
    return _lib


Beam = List[Tuple[List[int], float]]


def decode(emis: np.ndarray, beam: int, blank: int = 0, codes: Optional[Sequence[int]] = None,
           is_log: bool = False, nthreads: int = 1, max_hyps: int = 512,
           prob_domain: bool = False) -> List[Beam]:
    """Ranked final beam [(labels, logp)] per utterance of emis [T][B][V]."""
    emis = np.ascontiguousarray(emis, dtype=np.float32)
    T, B, V = emis.shape
    c = None if codes is None else np.ascontiguousarray(codes, dtype=np.int32)
    nh = np.zeros(B, np.int32)
    ln = np.zeros((B, max_hyps), np.int32)
    lab = np.zeros((B, max_hyps, T), np.int32)
    lp = np.zeros((B, max_hyps), np.float64)
    fn = lib().oracle_ctc_decode_prob if prob_domain else lib().oracle_ctc_decode
    rc = fn(emis.ctypes.data, T, B, V, beam, blank, c.ctypes.data if c is not None else None,
            int(is_log), nthreads, max_hyps, T, nh.ctypes.data, ln.ctypes.data, lab.ctypes.data,
            lp.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_ctc_decode: bad arguments")
    return [[(list(lab[b, k, :ln[b, k]]), float(lp[b, k])) for k in range(min(nh[b], max_hyps))]
            for b in range(B)]


def decode_ts(emis: np.ndarray, beam: int, blank: int = 0, codes: Optional[Sequence[int]] = None,
              is_log: bool = False, nthreads: int = 1, max_hyps: int = 512):
    """Ranked final beam [(labels, logp, timesteps)] per utterance: timesteps[i]
    is the frame at which label i was appended (OracleCTC::track_ts; the
    build's definition of ctcdecode's timesteps, parity unpinned)."""
    emis = np.ascontiguousarray(emis, dtype=np.float32)
    T, B, V = emis.shape
    c = None if codes is None else np.ascontiguousarray(codes, dtype=np.int32)
    nh = np.zeros(B, np.int32)
    ln = np.zeros((B, max_hyps), np.int32)
    lab = np.zeros((B, max_hyps, T), np.int32)
    lp = np.zeros((B, max_hyps), np.float64)
    ts = np.full((B, max_hyps, T), -1, np.int32)
    rc = lib().oracle_ctc_decode_ts(emis.ctypes.data, T, B, V, beam, blank,
                                    c.ctypes.data if c is not None else None, int(is_log), nthreads,
                                    max_hyps, T, nh.ctypes.data, ln.ctypes.data, lab.ctypes.data,
                                    lp.ctypes.data, ts.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_ctc_decode_ts: bad arguments")
    return [[(list(lab[b, k, :ln[b, k]]), float(lp[b, k]), list(ts[b, k, :ln[b, k]]))
             for k in range(min(nh[b], max_hyps))] for b in range(B)]


def time_decode(emis: np.ndarray, beam: int, blank: int = 0, is_log: bool = False,
                nthreads: int = 1) -> float:
    """Wall seconds of the oracle decode (cpu_baseline leg of bench.py)."""
    emis = np.ascontiguousarray(emis, dtype=np.float32)
    T, B, V = emis.shape
    return float(lib().oracle_ctc_time(emis.ctypes.data, T, B, V, beam, blank, int(is_log), nthreads))


def synthetic_emissions(T: int, B: int, V: int, seed0: int = SEED0, sigma: float = 3.0,
                        first: int = 0, log: bool = False) -> np.ndarray:
    """[T][B][V] fp32 softmax(N(0, sigma^2) logits), computed in fp64.

    Utterance u (global index first + b) draws from its own generator
    default_rng(seed0 + u), so any shard of utterances reproduces exactly the
    rows of the full batch."""
    out = np.empty((T, B, V), np.float32)
    for b in range(B):
        rng = np.random.default_rng(seed0 + first + b)
        z = rng.normal(0.0, sigma, size=(T, V))
        z -= z.max(axis=1, keepdims=True)
        if log:
            p = z - np.log(np.exp(z).sum(axis=1, keepdims=True))
        else:
            e = np.exp(z)
            p = e / e.sum(axis=1, keepdims=True)
        out[:, b, :] = p.astype(np.float32)
    return out


def _lse(a: float, b: float) -> float:
    if a == -np.inf:
        return b
    if b == -np.inf:
        return a
    m = max(a, b)
    return m + float(np.log1p(np.exp(-abs(a - b))))


def decode_cu(emis: np.ndarray, beam: int, blank: int = 0, codes: Optional[Sequence[int]] = None,
              is_log: bool = False) -> List[List[Tuple[List[int], float]]]:
    """Pure-Python restatement of what /root/reference/CTCBeamSearch.cu
    computes when it works (small cases only):
      * initialPath (cu:337-401): one state per symbol at t = 0, pruned;
      * kernelGenNextPaths (cu:404-458): the A.2 transitions; on the last
        step the trailing blank is stripped per candidate before merging;
      * merge of identical strings (cu:150-172, 460-489) in string order —
        the .cu sums with atomicAdd in fp32 (order not fixed); here fp64 log
        domain, left fold in string order;
      * prune (cu:174-196, 491-505): stable descending sort of the
        string-sorted states, exactly min(beam, n) kept.
    Returns per utterance the final beam [(labels, log p)], best first.
    States are (labels tuple, ends_in_blank); their string is the code
    sequence plus code(blank) when ends_in_blank.  T >= 2 (for T = 1 the .cu
    returns the unstripped initial state)."""
    T, B, V = emis.shape
    code = list(range(V)) if codes is None else list(codes)
    out = []
    for b in range(B):
        le = emis[:, b, :].astype(np.float64) if is_log else np.log(emis[:, b, :].astype(np.float64))

        def skey(st):
            q, fb = st
            return tuple(code[c] for c in q) + ((code[blank],) if fb else ())

        def prune(states):
            order = sorted(states.items(), key=lambda kv: skey(kv[0]))       # string order
            order.sort(key=lambda kv: -kv[1])                                 # stable by score
            return dict(order[:beam])

        states = {}
        for c in range(V):
            st = ((), True) if c == blank else ((c,), False)
            states[st] = le[0, c]
        states = prune(states)
        for t in range(1, T):
            last = t == T - 1
            new = {}
            for (q, fb) in sorted(states, key=skey):
                s = states[(q, fb)]
                for c in range(V):
                    if c == blank:
                        nst = (q, True)
                    elif fb or not q or q[-1] != c:
                        nst = (q + (c,), False)
                    else:
                        nst = (q, False)
                    if last:
                        nst = (nst[0], False)
                    new[nst] = _lse(new.get(nst, -np.inf), s + le[t, c])
            states = prune(new)
        ranked = sorted(states.items(), key=lambda kv: (-kv[1], skey(kv[0])))
        out.append([(list(q), float(s)) for (q, _), s in ranked])
    return out

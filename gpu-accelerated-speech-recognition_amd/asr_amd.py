"""Python host mirror of the reference's C++ API over libasr_amd.so (ctypes).

The reference (jrxk/GPU-Accelerated-Speech-Recognition) exposes C++ classes
only; its callers are main.cpp / nn_test.cpp.  This module mirrors those
classes for Python callers, tests and bench.py, calling the C ABI of
include/asr_amd.h — it contains no arithmetic of its own:

    CTCBeamSearch(vocab, vocabSize, beamWidth, blankID)   CTCBeamSearch.h:107
        .decode(seqProb, timestep, batchSize)             CTCBeamSearch.cu:262
    Linear(batch_size, input_size, output_size).forward   Linear.cu:42
    RNN_Cell(batch, in, hidden).forward                   RNN_Cell.cu:65
    RNN(batch, in, hidden, time_step, num_layers).forward RNN.cu:9
    DeviceMatrix ~ cuMatrix<float> (toGpu / toCpu)        cuMatrix.h:72-105

The native library is required: importing this module on a machine where
libasr_amd.so is missing raises, there is no fallback path.
"""
from __future__ import annotations

import collections
import ctypes
import os
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# ASR_LIB selects a diagnostic variant (e.g. libasr_amd_stamps.so) for tools/.
LIB_PATH = PKG_DIR / os.environ.get("ASR_LIB", "libasr_amd.so")

ASR_OK = 0
ASR_ERR_ARG = 1
ASR_ERR_HIP = 2
ASR_ERR_OOM = 3
ASR_ERR_BEAM_OVERFLOW = 4
ASR_ERR_UNSUPPORTED = 5
ASR_ERR_STATE = 6
ASR_ERR_INTERNAL = 7

EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_LOGSOFTMAX = 0, 1, 2, 3
SEMANTICS_CPU, SEMANTICS_CUDA = 0, 1   # asr_ctc_set_semantics
ASR_CTC_WAVES_LIST = -1                # asr_ctc_set_waves: the one-wave list kernel
ASR_CTC_TS_MAX_T = 65536               # longest decode with timesteps on (16-bit frames)

# Every symbol include/asr_amd.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "asr_status_string", "asr_version", "asr_get_device_count", "asr_set_device",
    "asr_get_device", "asr_device_malloc", "asr_device_free", "asr_host_malloc",
    "asr_host_free", "asr_memcpy_h2d", "asr_memcpy_d2h", "asr_memcpy_d2d", "asr_memset",
    "asr_stream_create", "asr_stream_destroy", "asr_stream_sync", "asr_device_sync",
    "asr_matmul", "asr_matmul_ta", "asr_matmul_tb", "asr_matadd", "asr_linear_fwd",
    "asr_rnn_cell_fwd", "asr_rnn_fwd", "asr_rnn_recur_fwd", "asr_rnn_persist_stats", "asr_rnn_emit_fwd", "asr_rnn_bidir_workspace_bytes", "asr_rnn_bidir_fwd",
    "asr_ctc_create", "asr_ctc_destroy", "asr_ctc_decode",
    "asr_ctc_get_best", "asr_ctc_get_beams", "asr_ctc_last_kernel_ms", "asr_ctc_set_waves",
    "asr_ctc_get_config", "asr_ctc_decode_ex", "asr_ctc_decode_segment", "asr_ctc_set_semantics",
    "asr_ctc_set_timesteps", "asr_ctc_get_beams_ts", "asr_ctc_set_result_stream",
    "asr_ctc_set_concurrency", "asr_rnn_set_recurrence", "asr_rnn_get_recurrence",
    "asr_set_dense_arith", "asr_get_dense_arith",
    "asr_pipeline_create", "asr_pipeline_submit", "asr_pipeline_collect", "asr_pipeline_pending",
    "asr_pipeline_describe", "asr_pipeline_get_production", "asr_pipeline_get_streams", "asr_pipeline_get_queue_use",
    "asr_pipeline_peek_emissions", "asr_pipeline_get_segments", "asr_pipeline_get_drain", "asr_pipeline_get_groups",
    "asr_pipeline_get_placement", "asr_pipeline_probe_placement", "asr_pipeline_set_timing",
    "asr_pipeline_get_timeline", "asr_pipeline_destroy", "asr_pipeline_create_coalesced", "asr_pipeline_get_coalesce",
]
# asr_pipeline_get_placement roles (ASR_PIPE_ROLE_*)
PIPE_ROLES = {0: "decode", 1: "production", 2: "decode_cu_gemm", 3: "gemm"}
ASR_MAX_XCC = 16


class AsrError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {status_string(status)} (status {status})")


_lib: Optional[ctypes.CDLL] = None
_vp = ctypes.c_void_p
_i = ctypes.c_int
_sz = ctypes.c_size_t
_f = ctypes.c_float


def lib() -> ctypes.CDLL:
    """Load libasr_amd.so (built by `make` in this directory)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} not found: build it with __graft_entry__.build() "
                           "or `make -C gpu-accelerated-speech-recognition_amd`")
    L = ctypes.CDLL(str(LIB_PATH))
    L.asr_status_string.restype = ctypes.c_char_p
    L.asr_status_string.argtypes = [_i]
    L.asr_version.restype = ctypes.c_char_p
    sig = {
        "asr_get_device_count": [ctypes.POINTER(_i)],
        "asr_set_device": [_i],
        "asr_get_device": [ctypes.POINTER(_i)],
        "asr_device_malloc": [ctypes.POINTER(_vp), _sz],
        "asr_device_free": [_vp],
        "asr_host_malloc": [ctypes.POINTER(_vp), _sz],
        "asr_host_free": [_vp],
        "asr_memcpy_h2d": [_vp, _vp, _sz, _vp],
        "asr_memcpy_d2h": [_vp, _vp, _sz, _vp],
        "asr_memcpy_d2d": [_vp, _vp, _sz, _vp],
        "asr_memset": [_vp, _i, _sz, _vp],
        "asr_stream_create": [ctypes.POINTER(_vp)],
        "asr_stream_destroy": [_vp],
        "asr_stream_sync": [_vp],
        "asr_device_sync": [],
        "asr_matmul": [_vp, _vp, _vp, _i, _i, _i, _vp],
        "asr_matmul_ta": [_vp, _vp, _vp, _i, _i, _i, _vp],
        "asr_matmul_tb": [_vp, _vp, _vp, _i, _i, _i, _vp],
        "asr_matadd": [_vp, _vp, _vp, _i, _i, _f, _vp],
        "asr_linear_fwd": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp],
        "asr_rnn_cell_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp],
        "asr_rnn_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp],
        "asr_rnn_recur_fwd": [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp],
        "asr_rnn_persist_stats": [ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)],
        "asr_rnn_set_recurrence": [_i],
        "asr_rnn_get_recurrence": [ctypes.POINTER(_i)],
        "asr_set_dense_arith": [_i],
        "asr_get_dense_arith": [ctypes.POINTER(_i)],
        "asr_rnn_emit_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp],
        "asr_pipeline_create": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)],
        "asr_pipeline_create_coalesced": [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)],
        "asr_pipeline_get_coalesce": [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)],
        "asr_pipeline_submit": [_vp, _vp],
        "asr_pipeline_collect": [_vp, _vp, _i, _vp, _vp, _vp],
        "asr_pipeline_pending": [_vp, ctypes.POINTER(_i)],
        "asr_pipeline_describe": [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                                  ctypes.POINTER(_i)],
        "asr_pipeline_destroy": [_vp],
        "asr_pipeline_get_production": [_vp, ctypes.POINTER(_i), ctypes.POINTER(ctypes.c_longlong),
                                        ctypes.POINTER(_i)],
        "asr_pipeline_get_streams": [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)],
        "asr_pipeline_get_queue_use": [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)],
        "asr_pipeline_get_placement": [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                                       ctypes.POINTER(_i)],
        "asr_pipeline_probe_placement": [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i)],
        "asr_pipeline_set_timing": [_vp, _i],
        "asr_pipeline_get_timeline": [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(_f)],
        "asr_pipeline_peek_emissions": [_vp, ctypes.POINTER(_vp)],
        "asr_pipeline_get_segments": [_vp, ctypes.POINTER(_i)],
        "asr_pipeline_get_drain": [_vp, ctypes.POINTER(_i), ctypes.POINTER(ctypes.c_double)],
        "asr_pipeline_get_groups": [_vp, ctypes.POINTER(_i)],
        "asr_rnn_bidir_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp],
        "asr_ctc_create": [_vp, _i, _i, _i, _i, ctypes.POINTER(_vp)],
        "asr_ctc_destroy": [_vp],
        "asr_ctc_decode": [_vp, _vp, _i, _i, _i, _vp],
        "asr_ctc_get_best": [_vp, _vp, _i, _vp, _vp],
        "asr_ctc_get_beams": [_vp, _i, _i, _vp, _vp, _vp, _vp],
        "asr_ctc_last_kernel_ms": [_vp, ctypes.POINTER(_f)],
        "asr_ctc_set_waves": [_vp, _i],
        "asr_ctc_set_concurrency": [_vp, _i],
        "asr_ctc_get_config": [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)],
        "asr_ctc_decode_ex": [_vp, _vp, _i, _i, ctypes.c_long, ctypes.c_long, _vp, _i, _vp],
        "asr_ctc_decode_segment": [_vp, _vp, _i, _i, _i, _i, ctypes.c_long, ctypes.c_long, _vp, _i, _vp],
        "asr_ctc_set_semantics": [_vp, _i],
        "asr_ctc_set_timesteps": [_vp, _i],
        "asr_ctc_set_result_stream": [_vp, _vp],
        "asr_ctc_get_beams_ts": [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _i
    L.asr_rnn_bidir_workspace_bytes.argtypes = [_i, _i, _i]
    L.asr_rnn_bidir_workspace_bytes.restype = _sz
    _lib = L
    return L


def status_string(status: int) -> str:
    return lib().asr_status_string(status).decode()


def check(rc: int, what: str) -> None:
    if rc != ASR_OK:
        raise AsrError(rc, what)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = _i(0)
    check(lib().asr_get_device_count(ctypes.byref(n)), "asr_get_device_count")
    return n.value


def set_device(d: int) -> None:
    check(lib().asr_set_device(d), "asr_set_device")


def synchronize() -> None:
    check(lib().asr_device_sync(), "asr_device_sync")


class DeviceMatrix:
    """fp32 row-major device buffer (cuMatrix<float> device side)."""

    def __init__(self, rows: int, cols: int = 1, data: Optional[np.ndarray] = None):
        self.rows, self.cols = int(rows), int(cols)
        self.nbytes = 4 * self.rows * self.cols
        p = _vp()
        check(lib().asr_device_malloc(ctypes.byref(p), self.nbytes), "asr_device_malloc")
        self.ptr = p.value or 0
        if data is not None:
            self.toGpu(data)

    @classmethod
    def from_numpy(cls, a: np.ndarray) -> "DeviceMatrix":
        a = np.ascontiguousarray(a, dtype=np.float32)
        r = a.shape[0] if a.ndim else 1
        return cls(r, a.size // max(r, 1), a)

    def toGpu(self, a: np.ndarray, stream: int = 0) -> None:
        a = np.ascontiguousarray(a, dtype=np.float32)
        assert a.size * 4 == self.nbytes, (a.shape, self.rows, self.cols)
        check(lib().asr_memcpy_h2d(self.ptr, _ptr(a), self.nbytes, stream), "asr_memcpy_h2d")

    def toCpu(self, stream: int = 0) -> np.ndarray:
        out = np.empty((self.rows, self.cols), dtype=np.float32)
        check(lib().asr_memcpy_d2h(_ptr(out), self.ptr, self.nbytes, stream), "asr_memcpy_d2h")
        return out

    def free(self) -> None:
        if self.ptr:
            lib().asr_device_free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBytes:
    """Untyped device allocation (workspace / generic buffers)."""

    def __init__(self, nbytes: int):
        p = _vp()
        check(lib().asr_device_malloc(ctypes.byref(p), int(nbytes)), "asr_device_malloc")
        self.ptr, self.nbytes = p.value or 0, int(nbytes)

    def __del__(self):
        try:
            if self.ptr:
                lib().asr_device_free(self.ptr)
        except Exception:
            pass


# --------------------------------------------------------------------- dense
def linear_fwd(x: DeviceMatrix, W: DeviceMatrix, b: Optional[DeviceMatrix], y: DeviceMatrix,
               epilogue: int = EPI_BIAS_RELU, stream: int = 0) -> DeviceMatrix:
    M, K = x.rows, x.cols
    N = W.cols
    assert W.rows == K and y.rows == M and y.cols == N
    check(lib().asr_linear_fwd(x.ptr, W.ptr, b.ptr if b else None, y.ptr, M, K, N, epilogue,
                               stream), "asr_linear_fwd")
    return y


def rnn_fwd(x: DeviceMatrix, W_ih: DeviceMatrix, W_hh: DeviceMatrix, b_ih: DeviceMatrix,
            b_hh: DeviceMatrix, hid: DeviceMatrix, T: int, B: int,
            h0: Optional[DeviceMatrix] = None, stream: int = 0) -> DeviceMatrix:
    inp, H = W_ih.rows, W_ih.cols
    check(lib().asr_rnn_fwd(x.ptr, h0.ptr if h0 else None, W_ih.ptr, W_hh.ptr, b_ih.ptr,
                            b_hh.ptr, hid.ptr, T, B, inp, H, stream), "asr_rnn_fwd")
    return hid


def rnn_recur_fwd(W_hh: DeviceMatrix, b_ih: DeviceMatrix, b_hh: DeviceMatrix, hid: DeviceMatrix,
                  T: int, B: int, h0: Optional[DeviceMatrix] = None, stream: int = 0) -> DeviceMatrix:
    """The recurrence stage alone (asr_rnn_recur_fwd): hid holds x.W_ih on entry,
    the hidden states on return."""
    H = W_hh.cols
    check(lib().asr_rnn_recur_fwd(h0.ptr if h0 else None, W_hh.ptr, b_ih.ptr, b_hh.ptr, hid.ptr,
                                  T, B, H, stream), "asr_rnn_recur_fwd")
    return hid


def rnn_persist_stats() -> tuple:
    """(launches, recoveries) of the one-launch H > 256 recurrence in this
    process (asr_rnn_persist_stats): recoveries are launches that gave up
    waiting for their workgroups and were finished by the recovery kernel."""
    n, r = ctypes.c_longlong(0), ctypes.c_longlong(0)
    check(lib().asr_rnn_persist_stats(ctypes.byref(n), ctypes.byref(r)), "asr_rnn_persist_stats")
    return n.value, r.value


def rnn_emit_fwd(W_hh: DeviceMatrix, b_ih: DeviceMatrix, b_hh: DeviceMatrix, W_out: DeviceMatrix,
                 b_out: DeviceMatrix, P: DeviceMatrix, emis: DeviceMatrix, T: int, B: int,
                 h0: Optional[DeviceMatrix] = None, hid: Optional[DeviceMatrix] = None,
                 stream: int = 0) -> DeviceMatrix:
    """Recurrence + emission projection + log_softmax in one kernel
    (asr_rnn_emit_fwd): P holds x.W_ih (unchanged), emis [T*B, V] receives the
    log-probabilities, hid (optional) the hidden states."""
    H, V = W_hh.cols, W_out.cols
    assert P.rows == T * B and P.cols == H and emis.rows == T * B and emis.cols == V
    check(lib().asr_rnn_emit_fwd(h0.ptr if h0 else None, W_hh.ptr, b_ih.ptr, b_hh.ptr, W_out.ptr,
                                 b_out.ptr, P.ptr, hid.ptr if hid else None, emis.ptr, T, B, H, V,
                                 stream), "asr_rnn_emit_fwd")
    return emis


def rnn_bidir_fwd(x: DeviceMatrix, params: Sequence[Tuple[DeviceMatrix, ...]], out: DeviceMatrix,
                  T: int, B: int, h0: Optional[DeviceMatrix] = None,
                  work: Optional["DeviceBytes"] = None, stream: int = 0) -> DeviceMatrix:
    """nn.RNN(bidirectional=True) (baseline/model.py:30): params[d] = (W_ih, W_hh,
    b_ih, b_hh) for d = 0 (forward in t) and d = 1 (reverse); h0 [2*B, H];
    out [T*B, 2H] = (h_fwd, h_bwd) per row."""
    inp, H = params[0][0].rows, params[0][0].cols
    assert len(params) == 2 and x.rows == T * B and x.cols == inp
    assert out.rows == T * B and out.cols == 2 * H
    need = lib().asr_rnn_bidir_workspace_bytes(T, B, H)
    if work is None or work.nbytes < need:
        work = DeviceBytes(need)
    arr = [(_vp * 2)(*(params[d][k].ptr for d in range(2))) for k in range(4)]
    check(lib().asr_rnn_bidir_fwd(x.ptr, h0.ptr if h0 else None, arr[0], arr[1], arr[2], arr[3],
                                  out.ptr, work.ptr, T, B, inp, H, stream), "asr_rnn_bidir_fwd")
    if stream == 0:
        check(lib().asr_stream_sync(None), "asr_stream_sync")
    return out


RNN_RECUR_AUTO, RNN_RECUR_VALU, RNN_RECUR_MFMA = 0, 1, 2


def rnn_set_recurrence(kind: int) -> None:
    """Process-wide recurrence kernel choice (asr_rnn_set_recurrence)."""
    check(lib().asr_rnn_set_recurrence(int(kind)), "asr_rnn_set_recurrence")


def rnn_get_recurrence() -> int:
    """The process-wide recurrence kernel choice (asr_rnn_get_recurrence)."""
    k = _i()
    check(lib().asr_rnn_get_recurrence(ctypes.byref(k)), "asr_rnn_get_recurrence")
    return k.value


DENSE_F32, DENSE_SPLIT_BF16 = 0, 1


def set_dense_arith(arith: int) -> None:
    """Process-wide arithmetic of the dense contractions (asr_set_dense_arith):
    DENSE_SPLIT_BF16 (default, fp32-accurate three-piece bf16 MFMA) or DENSE_F32."""
    check(lib().asr_set_dense_arith(int(arith)), "asr_set_dense_arith")


def get_dense_arith() -> int:
    a = _i()
    check(lib().asr_get_dense_arith(ctypes.byref(a)), "asr_get_dense_arith")
    return a.value


def rnn_cell_fwd(x: DeviceMatrix, h_prev: DeviceMatrix, W_ih: DeviceMatrix,
                 W_hh: DeviceMatrix, b_ih: DeviceMatrix, b_hh: DeviceMatrix,
                 h_out: DeviceMatrix, stream: int = 0) -> DeviceMatrix:
    B, inp = x.rows, x.cols
    H = W_ih.cols
    check(lib().asr_rnn_cell_fwd(x.ptr, h_prev.ptr, W_ih.ptr, W_hh.ptr, b_ih.ptr, b_hh.ptr,
                                 h_out.ptr, B, inp, H, stream), "asr_rnn_cell_fwd")
    return h_out


class Linear:
    """Linear.h: y = relu(x.W + b), W [in, out] row-major (Linear.cu:42-49)."""

    def __init__(self, batch_size: int, input_size: int, output_size: int,
                 weight: Optional[np.ndarray] = None, bias: Optional[np.ndarray] = None,
                 epilogue: int = EPI_BIAS_RELU):
        self.batch_size, self.input_size, self.output_size = batch_size, input_size, output_size
        w = np.zeros((input_size, output_size), np.float32) if weight is None else weight
        b = np.zeros((output_size,), np.float32) if bias is None else bias
        self.w = DeviceMatrix.from_numpy(np.asarray(w, np.float32).reshape(input_size, output_size))
        self.b = DeviceMatrix.from_numpy(np.asarray(b, np.float32).reshape(output_size, 1))
        self.outputs = DeviceMatrix(batch_size, output_size)
        self.epilogue = epilogue

    def forward(self, inputs: DeviceMatrix, stream: int = 0) -> DeviceMatrix:
        return linear_fwd(inputs, self.w, self.b, self.outputs, self.epilogue, stream)


class RNN:
    """RNN.h: tanh RNN, num_layers stacked, time-major [T*B, H] hiddens."""

    def __init__(self, batch_size: int, input_size: int, hidden_size: int, time_step: int,
                 num_layers: int = 1, params: Optional[Sequence[Tuple[np.ndarray, ...]]] = None):
        self.B, self.inp, self.H, self.T, self.L = batch_size, input_size, hidden_size, time_step, num_layers
        self.layers = []
        for l in range(num_layers):
            i = input_size if l == 0 else hidden_size
            if params is None:
                p = (np.zeros((i, hidden_size), np.float32), np.zeros((hidden_size, hidden_size), np.float32),
                     np.zeros(hidden_size, np.float32), np.zeros(hidden_size, np.float32))
            else:
                p = params[l]
            w_ih, w_hh, b_ih, b_hh = (DeviceMatrix.from_numpy(np.asarray(a, np.float32).reshape(
                (i, hidden_size) if k == 0 else (hidden_size, hidden_size) if k == 1 else (hidden_size, 1)))
                for k, a in enumerate(p))
            self.layers.append((w_ih, w_hh, b_ih, b_hh))
        self.hiddens = [DeviceMatrix(time_step * batch_size, hidden_size) for _ in range(num_layers)]

    def forward(self, inputs: DeviceMatrix, stream: int = 0) -> DeviceMatrix:
        x = inputs
        for l, (w_ih, w_hh, b_ih, b_hh) in enumerate(self.layers):
            rnn_fwd(x, w_ih, w_hh, b_ih, b_hh, self.hiddens[l], self.T, self.B, None, stream)
            x = self.hiddens[l]
        return self.hiddens[-1]


# ----------------------------------------------------------------------- CTC
class CTCDecoder:
    """Handle over asr_ctc_*: decode time-major emissions [T][B][V]."""

    def __init__(self, V: int, beam_width: int, blank_id: int = 0,
                 codes: Optional[Sequence[int]] = None, max_states: int = 0, waves: int = 0):
        self.V, self.beam, self.blank = V, beam_width, blank_id
        self.codes = None if codes is None else np.ascontiguousarray(codes, dtype=np.int32)
        h = _vp()
        check(lib().asr_ctc_create(_ptr(self.codes) if self.codes is not None else None, V,
                                   beam_width, blank_id, max_states, ctypes.byref(h)),
              "asr_ctc_create")
        self.h = h.value
        if waves:
            check(lib().asr_ctc_set_waves(self.h, waves), "asr_ctc_set_waves")
        self._emis: Optional[DeviceBytes] = None
        self.T = self.B = 0

    def config(self) -> Tuple[int, int, int]:
        ms, w, lds = _i(), _i(), _i()
        check(lib().asr_ctc_get_config(self.h, ctypes.byref(ms), ctypes.byref(w), ctypes.byref(lds)),
              "asr_ctc_get_config")
        return ms.value, w.value, lds.value

    def set_waves(self, waves: int) -> None:
        check(lib().asr_ctc_set_waves(self.h, waves), "asr_ctc_set_waves")

    def set_concurrency(self, n: int) -> None:
        """Scheduling hint: n decodes of this batch size run at once on the
        device (asr_ctc_set_concurrency); results are unchanged."""
        check(lib().asr_ctc_set_concurrency(self.h, int(n)), "asr_ctc_set_concurrency")

    def set_semantics(self, semantics: int) -> None:
        """SEMANTICS_CPU (default, the parity target) or SEMANTICS_CUDA
        (CTCBeamSearch.cu: exactly beam states, strip-then-merge last step)."""
        check(lib().asr_ctc_set_semantics(self.h, semantics), "asr_ctc_set_semantics")

    def set_result_stream(self, stream: int) -> None:
        """Run the best-path traceback and its copy to host memory on `stream`
        (a hipStream_t handle; 0: the decode's own stream)."""
        check(lib().asr_ctc_set_result_stream(self.h, ctypes.c_void_p(stream or None)), "asr_ctc_set_result_stream")

    def set_timesteps(self, on: bool) -> None:
        """Record each label's append frame in later decodes (beams_ts)."""
        check(lib().asr_ctc_set_timesteps(self.h, int(bool(on))), "asr_ctc_set_timesteps")

    def decode_device(self, d_emis: int, T: int, B: int, is_log: bool, stream: int = 0,
                      lengths: Optional[Sequence[int]] = None, frame_stride: Optional[int] = None,
                      utt_stride: Optional[int] = None) -> None:
        """Decode device emissions: element (t, b, v) at d_emis[t*frame_stride +
        b*utt_stride + v] (default time-major [T][B][V]); lengths[b] <= T."""
        fs = B * self.V if frame_stride is None else int(frame_stride)
        us = self.V if utt_stride is None else int(utt_stride)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.int32)
        if ln is not None:
            assert ln.shape == (B,), (ln.shape, B)
        check(lib().asr_ctc_decode_ex(self.h, d_emis, T, B, fs, us,
                                      _ptr(ln) if ln is not None else None, int(bool(is_log)), stream),
              "asr_ctc_decode_ex")
        self.T, self.B = T, B

    def decode_segment(self, d_emis: int, T: int, t0: int, t1: int, B: int, is_log: bool, stream: int = 0,
                       lengths: Optional[Sequence[int]] = None, frame_stride: Optional[int] = None,
                       utt_stride: Optional[int] = None) -> None:
        """Frames [t0, t1) of a T-frame batch (asr_ctc_decode_segment): d_emis
        addresses frame t0 (element (t, b, v) at d_emis + ((t - t0)*frame_stride
        + b*utt_stride + v) floats); segments in order from 0 to T, then
        best() / beams() as after decode_device."""
        fs = B * self.V if frame_stride is None else int(frame_stride)
        us = self.V if utt_stride is None else int(utt_stride)
        ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.int32)
        if ln is not None:
            assert ln.shape == (B,), (ln.shape, B)
        check(lib().asr_ctc_decode_segment(self.h, d_emis, T, t0, t1, B, fs, us,
                                           _ptr(ln) if ln is not None else None, int(bool(is_log)), stream),
              "asr_ctc_decode_segment")
        self.T, self.B = T, B

    def decode(self, emis: np.ndarray, is_log: bool = False, stream: int = 0,
               lengths: Optional[Sequence[int]] = None, batch_major: bool = False) -> None:
        """Upload emissions (fp32 [T][B][V], or [B][T][V] with batch_major) and
        enqueue the decode; lengths[b] frames of utterance b are used."""
        emis = np.ascontiguousarray(emis, dtype=np.float32)
        if batch_major:
            B, T, V = emis.shape
            fs, us = V, T * V
        else:
            T, B, V = emis.shape
            fs, us = B * V, V
        assert V == self.V, (V, self.V)
        if self._emis is None or self._emis.nbytes < emis.nbytes:
            self._emis = DeviceBytes(emis.nbytes)
        check(lib().asr_memcpy_h2d(self._emis.ptr, _ptr(emis), emis.nbytes, stream), "asr_memcpy_h2d")
        self.decode_device(self._emis.ptr, T, B, is_log, stream, lengths, fs, us)

    def best_arrays(self, allow_overflow: bool = False) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Best hypotheses as arrays: labels [B][T] int32 (row b valid up to
        lengths[b]), lengths [B], fp64 log-probs [B].  Reuses host buffers:
        copy them before the next call if they must persist."""
        B, T = self.B, self.T
        if getattr(self, "_best_bufs", None) is None or self._best_bufs[0].shape != (B, max(T, 1)):
            self._best_bufs = (np.zeros((B, max(T, 1)), np.int32), np.zeros(B, np.int32),
                               np.zeros(B, np.float64))
        lab, ln, lp = self._best_bufs
        rc = lib().asr_ctc_get_best(self.h, _ptr(lab), max(T, 1), _ptr(ln), _ptr(lp))
        if not (allow_overflow and rc == ASR_ERR_BEAM_OVERFLOW):
            check(rc, "asr_ctc_get_best")
        return lab, ln, lp

    def best(self, allow_overflow: bool = False) -> Tuple[List[List[int]], np.ndarray]:
        """Best label sequence and fp64 log-prob of every utterance."""
        lab, ln, lp = self.best_arrays(allow_overflow)
        return [lab[b, :ln[b]].tolist() for b in range(self.B)], lp.copy()

    def beams(self, max_hyps: int) -> List[List[Tuple[List[int], float]]]:
        """Ranked final beam (logp desc, string asc) of every utterance."""
        B, T = self.B, self.T
        nh = np.zeros(B, np.int32)
        ln = np.zeros((B, max_hyps), np.int32)
        lab = np.zeros((B, max_hyps, max(T, 1)), np.int32)
        lp = np.zeros((B, max_hyps), np.float64)
        check(lib().asr_ctc_get_beams(self.h, max_hyps, max(T, 1), _ptr(nh), _ptr(ln), _ptr(lab),
                                      _ptr(lp)), "asr_ctc_get_beams")
        return [[(lab[b, k, :ln[b, k]].tolist(), float(lp[b, k])) for k in range(min(nh[b], max_hyps))]
                for b in range(B)]

    def beams_ts(self, max_hyps: int) -> List[List[Tuple[List[int], float, List[int]]]]:
        """Ranked final beam with each label's append frame: [(labels, logp,
        timesteps)] per utterance (timesteps mode must have been on)."""
        B, T = self.B, self.T
        nh = np.zeros(B, np.int32)
        ln = np.zeros((B, max_hyps), np.int32)
        lab = np.zeros((B, max_hyps, max(T, 1)), np.int32)
        lp = np.zeros((B, max_hyps), np.float64)
        ts = np.zeros((B, max_hyps, max(T, 1)), np.int32)
        check(lib().asr_ctc_get_beams_ts(self.h, max_hyps, max(T, 1), _ptr(nh), _ptr(ln), _ptr(lab),
                                         _ptr(lp), _ptr(ts)), "asr_ctc_get_beams_ts")
        return [[(lab[b, k, :ln[b, k]].tolist(), float(lp[b, k]), ts[b, k, :ln[b, k]].tolist())
                 for k in range(min(nh[b], max_hyps))] for b in range(B)]

    def last_kernel_ms(self) -> float:
        ms = _f()
        check(lib().asr_ctc_last_kernel_ms(self.h, ctypes.byref(ms)), "asr_ctc_last_kernel_ms")
        return ms.value

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().asr_ctc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PipelineConfig(ctypes.Structure):
    """asr_pipeline_config (include/asr_amd.h)."""
    _fields_ = [(n, ctypes.c_int) for n in ("T", "B", "in_", "H", "V", "beam", "blank", "inflight",
                                           "prod_streams", "decode_cus", "segments")]


PIPELINE_MODES = {0: "CU groups (small batches)", 1: "chip-filling batches", 2: "CU groups (H > 256)"}


def model_emissions(x: "DeviceMatrix", weights, T: int, B: int, emis: "DeviceMatrix", fused: bool,
                    work: Optional["DeviceMatrix"] = None, stream: int = 0,
                    recurrence: Optional[int] = None) -> "DeviceMatrix":
    """One batch's emissions the way a Pipeline produces them
    (asr_pipeline_get_production): fused — input projection GEMM, then the
    recurrence with the emission layer fused (asr_rnn_emit_fwd); otherwise
    asr_rnn_fwd then asr_linear_fwd(..., log_softmax), with the recurrence
    kind the pipeline pinned (`recurrence`, Pipeline.describe()["recurrence"];
    None / AUTO: the process-wide choice), restored afterwards.  weights =
    (W_ih, W_hh, b_ih, b_hh, W_out, b_out); work [T*B, H] is scratch
    (allocated if None)."""
    W_ih, W_hh, b_ih, b_hh, W_out, b_out = weights
    work = work if work is not None else DeviceMatrix(T * B, W_hh.cols)
    if fused:
        linear_fwd(x, W_ih, None, work, EPI_NONE, stream)
        rnn_emit_fwd(W_hh, b_ih, b_hh, W_out, b_out, work, emis, T, B, stream=stream)
        return emis
    prev = None
    if recurrence not in (None, RNN_RECUR_AUTO):
        prev = rnn_get_recurrence()
        rnn_set_recurrence(recurrence)
    try:
        rnn_fwd(x, W_ih, W_hh, b_ih, b_hh, work, T, B, stream=stream)
    finally:
        if prev is not None:
            rnn_set_recurrence(prev)
    linear_fwd(work, W_out, b_out, emis, EPI_BIAS_LOGSOFTMAX, stream)
    return emis


class Pipeline:
    """asr_pipeline_*: RNN -> Linear + log_softmax -> CTC decode over a stream of
    equal-shape batches, the library overlapping production and decodes on its
    own streams.  submit(x) queues a batch (features stay valid until its
    results are collected); collect() returns the oldest batch's
    (labels [B][T], lengths [B], logp [B], decode_ms)."""

    def __init__(self, T: int, B: int, inp: int, H: int, V: int, beam: int, weights, blank: int = 0,
                 inflight: int = 0, prod_streams: int = 0, decode_cus: int = 0, segments: int = 0,
                 coalesce: int = 1):
        """coalesce > 1: dynamic batching (asr_pipeline_create_coalesced):
        `coalesce` consecutive submits of B utterances run as one batch; the
        schedule (inflight, prod_streams, ...) is that batch's."""
        self.T, self.B = T, B
        self.coalesce = max(1, int(coalesce))
        self.cfg = PipelineConfig(T, B, inp, H, V, beam, blank, inflight, prod_streams, decode_cus, segments)
        self._w = weights   # (W_ih, W_hh, b_ih, b_hh, W_out, b_out) DeviceMatrix: kept alive
        h = _vp()
        if self.coalesce > 1:
            check(lib().asr_pipeline_create_coalesced(ctypes.byref(self.cfg), self.coalesce,
                                                      *[w.ptr for w in weights], ctypes.byref(h)),
                  "asr_pipeline_create_coalesced")
        else:
            check(lib().asr_pipeline_create(ctypes.byref(self.cfg), *[w.ptr for w in weights], ctypes.byref(h)),
                  "asr_pipeline_create")
        self.h = h.value
        self._lab = np.zeros((B, max(T, 1)), np.int32)
        self._len = np.zeros(B, np.int32)
        self._lp = np.zeros(B, np.float64)
        self._inputs = collections.deque()   # submitted features, alive until their batch is collected
        self._kept = []                      # features of failed submits (alive until close)

    def describe(self):
        m, d, p, c, w = _i(), _i(), _i(), _i(), _i()
        check(lib().asr_pipeline_describe(self.h, ctypes.byref(m), ctypes.byref(d), ctypes.byref(p),
                                          ctypes.byref(c), ctypes.byref(w)), "asr_pipeline_describe")
        fz, gr, rk = _i(), ctypes.c_longlong(), _i()
        check(lib().asr_pipeline_get_production(self.h, ctypes.byref(fz), ctypes.byref(gr), ctypes.byref(rk)),
              "asr_pipeline_get_production")
        ns, hq, sg, gp = _i(), _i(), _i(), _i()
        check(lib().asr_pipeline_get_streams(self.h, ctypes.byref(ns), ctypes.byref(hq)), "asr_pipeline_get_streams")
        check(lib().asr_pipeline_get_segments(self.h, ctypes.byref(sg)), "asr_pipeline_get_segments")
        check(lib().asr_pipeline_get_groups(self.h, ctypes.byref(gp)), "asr_pipeline_get_groups")
        qs, qd = _i(), _i()
        check(lib().asr_pipeline_get_queue_use(self.h, ctypes.byref(qs), ctypes.byref(qd)),
              "asr_pipeline_get_queue_use")
        hb, f0 = _i(), ctypes.c_double()
        check(lib().asr_pipeline_get_drain(self.h, ctypes.byref(hb), ctypes.byref(f0)), "asr_pipeline_get_drain")
        return {"mode": PIPELINE_MODES.get(m.value, m.value), "inflight": d.value, "prod_streams": p.value,
                "decode_cus": c.value, "decode_waves": w.value, "fused_emission": bool(fz.value),
                "decode_cu_gemm_rows": gr.value, "recurrence": rk.value, "streams": ns.value,
                "hw_queues": hq.value, "segments": sg.value, "groups": gp.value,
                "drain_held_batches": hb.value, "first_segment_share": round(f0.value, 4),
                "shared_queue_streams": qs.value, "dedicated_queue_streams": qd.value,
                "coalesce": self.coalesce}

    def placement(self):
        """[(role name, cu_lo, cu_hi)] of every stream the pipeline created."""
        n = _i()
        check(lib().asr_pipeline_get_placement(self.h, 0, ctypes.byref(n), None, None, None),
              "asr_pipeline_get_placement")
        cnt = n.value
        role, lo, hi = (_i * max(1, cnt))(), (_i * max(1, cnt))(), (_i * max(1, cnt))()
        check(lib().asr_pipeline_get_placement(self.h, cnt, ctypes.byref(n), role, lo, hi),
              "asr_pipeline_get_placement")
        return [(PIPE_ROLES.get(role[i], role[i]), lo[i], hi[i]) for i in range(cnt)]

    def probe_placement(self, role: str):
        """Physical CUs per XCD that the first stream of `role` reaches (one
        probe launch; synchronises that stream): a list, one count per XCD."""
        r = {v: k for k, v in PIPE_ROLES.items()}[role]
        cnt, nx = (_i * ASR_MAX_XCC)(), _i()
        check(lib().asr_pipeline_probe_placement(self.h, r, cnt, ctypes.byref(nx)), "asr_pipeline_probe_placement")
        return [cnt[i] for i in range(nx.value)]

    def set_timing(self, on: bool = True) -> None:
        """Record per-batch production / decode timing events from the next
        submit on (call on a drained pipeline; clears the timeline)."""
        check(lib().asr_pipeline_set_timing(self.h, 1 if on else 0), "asr_pipeline_set_timing")

    def timeline(self):
        """(batch ids [n], stamps [n, 4] ms: production start / end, decode
        start / end) of the batches collected since set_timing."""
        n = _i()
        check(lib().asr_pipeline_get_timeline(self.h, 0, ctypes.byref(n), None, None), "asr_pipeline_get_timeline")
        cnt = n.value
        b = np.zeros(max(1, cnt), np.int64)
        t = np.zeros((max(1, cnt), 4), np.float32)
        check(lib().asr_pipeline_get_timeline(self.h, cnt, ctypes.byref(n),
                                              b.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                                              t.ctypes.data_as(ctypes.POINTER(_f))), "asr_pipeline_get_timeline")
        return b[:cnt], t[:cnt]

    def submit(self, x: "DeviceMatrix") -> None:
        """Queue a batch.  x is kept alive here until its batch is collected
        (asr_pipeline_submit reads it until then); after a failed submit it
        is kept until close(): queued work of the batch may still read it."""
        rc = lib().asr_pipeline_submit(self.h, x.ptr)
        if rc != ASR_OK:
            self._kept.append(x)
            check(rc, "asr_pipeline_submit")
        self._inputs.append(x)

    def pending(self) -> int:
        n = _i()
        check(lib().asr_pipeline_pending(self.h, ctypes.byref(n)), "asr_pipeline_pending")
        return n.value

    def collect(self, out=None):
        """(labels [B][T] int32, lengths [B], logp [B] fp64, decode_ms) of the
        oldest batch; the arrays are reused by the next call unless the caller
        passes its own (out = (labels, lengths, logp) of those shapes / dtypes)."""
        ms = _f()
        lab, ln, lp = (self._lab, self._len, self._lp) if out is None else out
        assert lab.dtype == np.int32 and lab.shape == self._lab.shape and lab.flags.c_contiguous
        assert ln.dtype == self._len.dtype and ln.shape == self._len.shape
        assert lp.dtype == np.float64 and lp.shape == self._lp.shape
        rc = lib().asr_pipeline_collect(self.h, _ptr(lab), lab.shape[1], _ptr(ln), _ptr(lp), ctypes.byref(ms))
        n = _i()
        if lib().asr_pipeline_pending(self.h, ctypes.byref(n)) == ASR_OK:
            while len(self._inputs) > n.value:   # collected batches' features may go
                self._inputs.popleft()
        check(rc, "asr_pipeline_collect")
        return lab, ln, lp, ms.value

    def peek_emissions(self) -> np.ndarray:
        """Host copy of the emissions [T][B][V] the last collected batch's
        decode consumed (asr_pipeline_peek_emissions)."""
        ptr = _vp()
        check(lib().asr_pipeline_peek_emissions(self.h, ctypes.byref(ptr)), "asr_pipeline_peek_emissions")
        g, col = self.coalesce, _i()
        if g > 1:   # the whole coalesced batch, then this submit's columns
            check(lib().asr_pipeline_get_coalesce(self.h, None, None, ctypes.byref(col)), "asr_pipeline_get_coalesce")
        out = np.empty((self.T, g * self.B, self.cfg.V), np.float32)
        check(lib().asr_memcpy_d2h(_ptr(out), ptr.value, out.nbytes, None), "asr_memcpy_d2h")
        if g > 1:
            out = np.ascontiguousarray(out[:, col.value * self.B:(col.value + 1) * self.B, :])
        return out

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().asr_pipeline_destroy(self.h)   # synchronises the pipeline's streams
            self.h = None
        self._inputs = collections.deque()
        self._kept = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CTCBeamSearch:
    """CTCBeamSearch.h:107 — CTCBeamSearch(vocab, vocabSize, beamWidth, blankID).

    decode(seqProb, timestep, batchSize) takes probabilities [T*B, V]
    (time-major rows, CTCBeamSearch.cu:67-69) and returns, per utterance, the
    best string and its probability as float (cu:283-298); `logprobs` holds
    the fp64 log-probabilities of the last decode.
    """

    def __init__(self, vocab: Sequence[str], vocabSize: int, beamWidth: int, blankID: int):
        self.vocab = [str(c) for c in list(vocab)[:vocabSize]]
        self.vocabSize, self.beamWidth, self.blankID = vocabSize, beamWidth, blankID
        codes = [ord(c) & 0xFF if len(c) == 1 else i for i, c in enumerate(self.vocab)]
        self._dec = CTCDecoder(vocabSize, beamWidth, blankID, codes)
        self.logprobs: Optional[np.ndarray] = None

    def decode(self, seqProb: np.ndarray, timestep: int, batchSize: int) -> List[Tuple[str, float]]:
        seqProb = np.asarray(seqProb, np.float32)
        if seqProb.shape[-1] != self.vocabSize:
            raise ValueError("Error: inconsistent vocabulary size in CTC decoder")
        self._dec.decode(seqProb.reshape(timestep, batchSize, self.vocabSize), is_log=False)
        labels, lp = self._dec.best()
        self.logprobs = lp
        return [("".join(self.vocab[i] for i in lab), float(np.exp(l))) for lab, l in zip(labels, lp)]


class CTCBeamDecoder:
    """Batch interface of the Python baseline's decoder (baseline/main.py:10,
    29, 46: ctcdecode.CTCBeamDecoder(labels, beam_width=, blank_id=,
    num_processes=, log_probs_input=True).decode(probs[B,T,V], seq_lens)) on
    this library's decoder.  ctcdecode itself is not available here, so the
    search semantics are the reference C++ decoder's (CTCBeamSearch.cpp with
    F1-F3), not ctcdecode's; no language model (model_path must
    be None).  decode returns (beam_results [B, beam_width, T] int32 label
    ids, beam_scores [B, beam_width] float32 = -log p (lower is better),
    timesteps [B, beam_width, T] int32, out_lens [B, beam_width] int32);
    hypotheses beyond an utterance's final beam have length 0 and score +inf.
    timesteps[b, k, i] is the frame at which label i of hypothesis k was
    FIRST APPENDED in the surviving search lineage (asr_ctc_set_timesteps).
    This differs from ctcdecode, which reports the frame of its trie node's
    best emission; the two are not pinned against each other (ctcdecode is
    unavailable here).  -1 past a hypothesis' length.  Tracking costs a second
    node table per decode, so it is on only with timesteps=True (the
    default, as ctcdecode always returns them); timesteps=False returns an
    all -1 array and decodes on the plain path.  probs may be a numpy array
    or a torch tensor (a GPU tensor is decoded in place, no copy)."""

    def __init__(self, labels: Sequence[str], model_path: Optional[str] = None, alpha: float = 0.0,
                 beta: float = 0.0, cutoff_top_n: int = 40, cutoff_prob: float = 1.0,
                 beam_width: int = 100, num_processes: int = 4, blank_id: int = 0,
                 log_probs_input: bool = False, timesteps: bool = True):
        if model_path is not None:
            raise NotImplementedError("language-model scoring is not supported")
        self.labels = list(labels)
        self.beam_width, self.blank_id, self.log_probs_input = beam_width, blank_id, log_probs_input
        self.track_timesteps = bool(timesteps)
        self._dec = CTCDecoder(len(self.labels), beam_width, blank_id)
        self._dec.set_timesteps(self.track_timesteps)

    def decode(self, probs, seq_lens=None):
        B, T, V = (int(x) for x in probs.shape)
        lens = None if seq_lens is None else np.asarray(
            seq_lens.cpu().numpy() if hasattr(seq_lens, "cpu") else seq_lens, dtype=np.int32)
        if hasattr(probs, "is_cuda") and probs.is_cuda:   # torch GPU tensor: zero-copy
            import torch
            p = probs if probs.dtype == torch.float32 else probs.float()
            if p.stride(2) != 1:   # the kernel reads a frame's V labels contiguously
                p = p.contiguous()
            self._dec.decode_device(p.data_ptr(), T, B, self.log_probs_input,
                                    torch.cuda.current_stream().cuda_stream, lens,
                                    p.stride(1), p.stride(0))
        else:
            arr = probs.cpu().numpy() if hasattr(probs, "cpu") else np.asarray(probs)
            self._dec.decode(arr, is_log=self.log_probs_input, lengths=lens, batch_major=True)
        K = self.beam_width
        if self.track_timesteps:
            beams = self._dec.beams_ts(max_hyps=self._dec.config()[0])
        else:
            beams = [[(lab, lp, None) for lab, lp in u] for u in self._dec.beams(self._dec.config()[0])]
        results = np.zeros((B, K, T), np.int32)
        scores = np.full((B, K), np.inf, np.float32)
        timesteps = np.full((B, K, T), -1, np.int32)
        out_lens = np.zeros((B, K), np.int32)
        for b, hyps in enumerate(beams):
            for k, (lab, lp, ts) in enumerate(hyps[:K]):
                results[b, k, :len(lab)] = lab
                scores[b, k] = -lp
                if ts is not None:
                    timesteps[b, k, :len(ts)] = ts
                out_lens[b, k] = len(lab)
        return results, scores, timesteps, out_lens

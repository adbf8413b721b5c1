"""GPU parity of the one-wave list kernel (asr_ctc_set_waves(ASR_CTC_WAVES_LIST),
csrc/ctc_wave_kernel.inc) against the CPU oracle: the same cases as
test_ctc_gpu.py, the same bar (labels and ranks identical, log-probs within
1e-9 relative)."""
import numpy as np
import pytest

from conftest import asr, cpu_threads, oracle
from test_ctc_gpu import assert_beams_equal, gpu_beams

pytestmark = pytest.mark.gpu
LIST = -1   # ASR_CTC_WAVES_LIST


def test_list_kernel_selected():
    dec = asr.CTCDecoder(29, 50, 0, waves=LIST)
    assert dec.config()[1] == LIST
    dec.close()


@pytest.mark.parametrize("T,B,V,beam,sigma", [
    (1, 4, 5, 3, 3.0), (2, 3, 4, 2, 3.0), (10, 8, 4, 2, 3.0), (25, 6, 6, 4, 3.0),
    (50, 8, 29, 10, 3.0), (100, 1, 29, 10, 3.0), (60, 16, 29, 50, 3.0), (60, 16, 29, 50, 0.5),
    (80, 8, 29, 100, 3.0), (80, 8, 29, 100, 0.3), (30, 4, 63, 20, 3.0), (30, 4, 63, 20, 0.5),
    (40, 4, 2, 5, 3.0), (20, 3, 31, 64, 1.0),
])
def test_random_parity(T, B, V, beam, sigma):
    emis = oracle.synthetic_emissions(T, B, V, seed0=2000 + T + V + beam, sigma=sigma)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam, waves=LIST), ref, f"T={T} B={B} V={V} beam={beam} s={sigma}")


def test_blank_last_and_codes_order():
    T, B, V, beam = 40, 6, 9, 7
    emis = oracle.synthetic_emissions(T, B, V, seed0=5)
    codes = [ord("a") + i for i in range(V - 1)] + [ord("~")]
    ref = oracle.decode(emis, beam, V - 1, codes=codes)
    assert_beams_equal(gpu_beams(emis, beam, V - 1, codes, waves=LIST), ref, "blank=V-1")


def test_log_input_and_zeros():
    emis = oracle.synthetic_emissions(50, 5, 29, seed0=9, log=True)
    ref = oracle.decode(emis, 20, 0, is_log=True)
    assert_beams_equal(gpu_beams(emis, 20, is_log=True, waves=LIST), ref, "is_log")
    emis = oracle.synthetic_emissions(30, 4, 7, seed0=3)
    emis[5, :, 2] = 0.0
    emis[:, 1, 4] = 0.0
    emis[0, 2, :] = 0.0
    emis[0, 2, 3] = 1.0
    ref = oracle.decode(emis, 5, 0)
    assert_beams_equal(gpu_beams(emis, 5, waves=LIST), ref, "zeros")


def test_ties_uniform_emissions():
    T, V, beam = 6, 4, 3
    emis = np.full((T, 2, V), 1.0 / V, np.float32)
    ref = oracle.decode(emis, beam, 0)
    assert_beams_equal(gpu_beams(emis, beam, max_states=128, waves=LIST), ref, "ties")


def test_blank_dominant():
    """Peaked, blank-dominated frames (the list kernel's best case)."""
    T, B, V, beam = 200, 8, 29, 50
    emis = oracle.synthetic_emissions(T, B, V, seed0=31, sigma=4.0)
    emis[:, :, 0] *= 30.0
    emis /= emis.sum(axis=2, keepdims=True)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam, waves=LIST), ref, "blank-dominant")


def test_lengths_batch_api():
    T, B, V, beam = 60, 6, 29, 20
    emis = oracle.synthetic_emissions(T, B, V, seed0=44)
    lengths = [60, 1, 0, 33, 59, 17]
    dec = asr.CTCDecoder(V, beam, 0, waves=LIST)
    dec.decode(emis, lengths=lengths)
    best, lp = dec.best()
    for b, n in enumerate(lengths):
        ref = oracle.decode(np.ascontiguousarray(emis[:n, b:b + 1, :]), beam, 0)[0] if n else [([], 0.0)]
        assert best[b] == ref[0][0], f"utterance {b} (T={n})"
        assert abs(lp[b] - ref[0][1]) <= 1e-9 * max(1.0, abs(ref[0][1]))
    dec.close()


def test_c2_shape_best():
    T, B, V, beam = 500, 64, 29, 50
    emis = oracle.synthetic_emissions(T, B, V)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads(), max_hyps=beam + 1)
    dec = asr.CTCDecoder(V, beam, 0, waves=LIST)
    dec.decode(emis)
    best, lp = dec.best()
    for b in range(B):
        assert best[b] == ref[b][0][0], f"utterance {b}"
        assert abs(lp[b] - ref[b][0][1]) <= 1e-9 * abs(ref[b][0][1])
    dec.close()


@pytest.mark.parametrize("sigma,beam", [(3.0, 50), (0.5, 50), (1.0, 100)])
def test_same_bits_as_workgroup_kernel(sigma, beam):
    """The one-wave kernel keeps the workgroup kernel's arithmetic (prefix
    scores, fold order, exact selection), so the ranked beams of a batch are
    the same labels and the same fp64 bits — only slot order differs."""
    T, B, V = 120, 96, 29
    emis = oracle.synthetic_emissions(T, B, V, seed0=777 + beam, sigma=sigma)
    got = {}
    for w in (8, LIST):
        dec = asr.CTCDecoder(V, beam, 0, waves=w)
        dec.decode(emis)
        got[w] = (dec.beams(max_hyps=dec.config()[0]), dec.best())
        dec.close()
    assert got[8][0] == got[LIST][0]
    assert got[8][1][0] == got[LIST][1][0]
    assert np.array_equal(np.asarray(got[8][1][1]), np.asarray(got[LIST][1][1]))

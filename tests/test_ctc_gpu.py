"""GPU parity of the HIP CTC beam search against the CPU oracle.

Bar (BASELINE.json north_star): decoded label sequences and beam ranks
identical to the reference CTCBeamSearch.cpp semantics; path log-probs within
1e-4.  The test tolerance is tighter: |dlogp| <= 1e-9 * max(1, |logp|)
(both sides compute in fp64; they differ only by libm vs device-libm ulps).
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN, asr, cpu_threads, oracle

pytestmark = pytest.mark.gpu
TOL = 1e-9


def assert_beams_equal(got, ref, what=""):
    assert len(got) == len(ref), what
    for b, (g, r) in enumerate(zip(got, ref)):
        assert [l for l, _ in g] == [l for l, _ in r], f"{what} utterance {b}: labels/ranks differ"
        for (_, x), (_, y) in zip(g, r):
            assert abs(x - y) <= TOL * max(1.0, abs(y)), f"{what} utterance {b}: {x} vs {y}"


def gpu_beams(emis, beam, blank=0, codes=None, is_log=False, waves=0, max_states=0):
    dec = asr.CTCDecoder(emis.shape[2], beam, blank, codes, max_states=max_states, waves=waves)
    dec.decode(emis, is_log=is_log)
    beams = dec.beams(max_hyps=dec.config()[0])
    best, lp = dec.best()
    # best() must be rank 0 of the ranked beam
    for b in range(emis.shape[1]):
        assert best[b] == beams[b][0][0]
        assert lp[b] == beams[b][0][1]
    dec.close()
    return beams


def test_main_cpp_vector():
    g = json.loads((GOLDEN / "main_cpp_ctc.json").read_text())
    emis = np.array(g["emissions"], np.float32).reshape(g["T"], 1, g["V"])
    codes = [ord(c) for c in g["vocab"]]
    got = gpu_beams(emis, g["beam"], g["blank"], codes)[0]
    assert ["".join(g["vocab"][i] for i in l) for l, _ in got] == [x[0] for x in g["expected_log"]]
    for (_, x), (_, e) in zip(got, g["expected_log"]):
        assert abs(x - e) <= 1e-12
    # the drop-in class returns (string, float prob) like CTCBeamSearch::decode
    ctc = asr.CTCBeamSearch(g["vocab"], g["V"], g["beam"], g["blank"])
    res = ctc.decode(emis.reshape(g["T"], g["V"]), g["T"], 1)
    assert res[0][0] == "cbacbc"
    assert res[0][1] == pytest.approx(g["survey_A6"]["prob"], rel=1e-6)


@pytest.mark.parametrize("T,B,V,beam", [
    (1, 4, 5, 3), (2, 3, 4, 2), (10, 8, 4, 2), (25, 6, 6, 4), (50, 8, 29, 10),
    (100, 1, 29, 10),            # BASELINE configs[0] shape (C1)
    (60, 16, 29, 50), (80, 8, 29, 100), (30, 4, 63, 20), (40, 4, 2, 5), (20, 3, 31, 64),
])
def test_random_parity(T, B, V, beam):
    emis = oracle.synthetic_emissions(T, B, V, seed0=1000 + T + V + beam)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam), ref, f"T={T} B={B} V={V} beam={beam}")


@pytest.mark.parametrize("waves", [1, 2, 4, 8])
def test_waves_bitwise_equal(waves):
    emis = oracle.synthetic_emissions(70, 8, 29, seed0=77)
    ref = oracle.decode(emis, 50, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, 50, waves=waves), ref, f"waves={waves}")


def test_blank_last_and_codes_order():
    """Blank id != 0 and a blank code above the symbols flips the fold order."""
    T, B, V, beam = 40, 6, 9, 7
    emis = oracle.synthetic_emissions(T, B, V, seed0=5)
    codes = [ord("a") + i for i in range(V - 1)] + [ord("~")]
    ref = oracle.decode(emis, beam, V - 1, codes=codes)
    assert_beams_equal(gpu_beams(emis, beam, V - 1, codes), ref, "blank=V-1")
    codes2 = [ord("~")] + [ord("a") + i for i in range(V - 1)]   # blank 0, largest code
    ref2 = oracle.decode(emis, beam, 0, codes=codes2)
    assert_beams_equal(gpu_beams(emis, beam, 0, codes2), ref2, "blank code max")


def test_log_input():
    emis = oracle.synthetic_emissions(50, 5, 29, seed0=9, log=True)
    ref = oracle.decode(emis, 20, 0, is_log=True)
    assert_beams_equal(gpu_beams(emis, 20, is_log=True), ref, "is_log")


def test_zero_probabilities():
    emis = oracle.synthetic_emissions(30, 4, 7, seed0=3)
    emis[5, :, 2] = 0.0
    emis[:, 1, 4] = 0.0
    emis[0, 2, :] = 0.0
    emis[0, 2, 3] = 1.0
    ref = oracle.decode(emis, 5, 0)
    assert_beams_equal(gpu_beams(emis, 5), ref, "zeros")


def test_ties_uniform_emissions():
    """All-equal emissions: many exact ties at the cutoff are all kept."""
    T, V, beam = 6, 4, 3
    emis = np.full((T, 2, V), 1.0 / V, np.float32)
    ref = oracle.decode(emis, beam, 0)
    assert max(len(r) for r in ref) > beam + 1
    assert_beams_equal(gpu_beams(emis, beam, max_states=128), ref, "ties")


def test_overflow_is_reported():
    """An explicit max_states too small for the ties is an error, never a
    silently different beam."""
    T, V, beam = 6, 4, 3
    emis = np.full((T, 1, V), 1.0 / V, np.float32)
    dec = asr.CTCDecoder(V, beam, 0, max_states=4)
    dec.decode(emis)
    with pytest.raises(asr.AsrError) as e:
        dec.best()
    assert e.value.status == asr.ASR_ERR_BEAM_OVERFLOW


def test_overflow_retried_with_automatic_capacity():
    """With the automatic capacity, tie overflow re-decodes with more room."""
    T, V, beam = 8, 4, 3
    emis = np.full((T, 3, V), 1.0 / V, np.float32)
    ref = oracle.decode(emis, beam, 0)
    assert max(len(r) for r in ref) > 64   # two doublings of the default 32 states
    dec = asr.CTCDecoder(V, beam, 0)
    dec.decode(emis)
    best, lp = dec.best()
    assert best == [r[0][0] for r in ref]
    assert_beams_equal(dec.beams(256), ref, "retry")


def test_shard_invariance():
    """Decoding any utterance range reproduces the full batch (multi-GPU sharding)."""
    full = oracle.synthetic_emissions(40, 12, 29, seed0=21)
    dec = asr.CTCDecoder(29, 20, 0)
    dec.decode(full)
    a, la = dec.best()
    dec.decode(np.ascontiguousarray(full[:, 5:9, :]))
    b, lb = dec.best()
    assert a[5:9] == b and np.array_equal(la[5:9], lb)


def test_c2_shape_best():
    """BASELINE configs[1] decode shape: B=64, T=500, V=29, beam=50."""
    T, B, V, beam = 500, 64, 29, 50
    emis = oracle.synthetic_emissions(T, B, V)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads(), max_hyps=beam + 1)
    dec = asr.CTCDecoder(V, beam, 0)
    dec.decode(emis)
    best, lp = dec.best()
    for b in range(B):
        assert best[b] == ref[b][0][0], f"utterance {b}"
        assert abs(lp[b] - ref[b][0][1]) <= TOL * abs(ref[b][0][1])
    beams = dec.beams(beam + 1)
    assert_beams_equal([x[:beam + 1] for x in beams[:8]], [r[:beam + 1] for r in ref[:8]], "C2")


def test_overflow_retry_with_next_batch_queued():
    """An automatic-capacity handle whose decode overflows (more tied
    survivors than max_states) re-decodes the caller's emission buffer when
    the results are fetched (asr_amd.h lifetime rule: the buffer stays valid
    and unmodified until then).  Here another handle's decode of a different
    buffer is queued on the same stream before the overflowing results are
    read; both results must still be the oracle's."""
    T, V, beam = 4, 5, 5
    uni = np.full((T, 2, V), 1.0 / V, np.float32)
    ref_u = oracle.decode(uni, beam, 0, max_hyps=4096)
    other = oracle.synthetic_emissions(30, 3, V, seed0=31)
    ref_o = oracle.decode(other, beam, 0)
    dA = asr.DeviceMatrix.from_numpy(uni.reshape(T * 2, V))
    dB = asr.DeviceMatrix.from_numpy(other.reshape(30 * 3, V))
    h1, h2 = asr.CTCDecoder(V, beam, 0), asr.CTCDecoder(V, beam, 0)
    assert h1.config()[0] < max(len(r) for r in ref_u)   # the default capacity overflows
    h1.decode_device(dA.ptr, T, 2, is_log=False)
    h2.decode_device(dB.ptr, 30, 3, is_log=False)         # next batch queued first
    best1, lp1 = h1.best()
    assert best1 == [r[0][0] for r in ref_u]
    assert_beams_equal(h1.beams(max_hyps=4096), ref_u, "overflow retry")
    assert_beams_equal(h2.beams(max_hyps=h2.config()[0]), ref_o, "next batch")
    h1.close()
    h2.close()

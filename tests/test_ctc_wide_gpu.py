"""GPU parity of the large-vocabulary decoder (V > 63: ctc_wide_kernel.inc)
against the CPU oracle — BASELINE C5 shapes (V=1000, beam=200) at short T.

Same bar as tests/test_ctc_gpu.py: labels and beam ranks identical, fp64
log-probs equal to 1e-9 relative.
"""
import numpy as np
import pytest

from conftest import asr, cpu_threads, oracle
from test_ctc_gpu import assert_beams_equal, gpu_beams

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,B,V,beam", [
    (12, 4, 64, 8),         # smallest wide shape (V+1 = 65 columns)
    (20, 4, 100, 20),
    (25, 3, 300, 50),       # C5-like width, C2 beam
    (40, 2, 129, 5),
    (10, 2, 1000, 200),     # BASELINE C5 vocabulary and beam
    (8, 2, 4096, 50),       # largest vocabulary
    (6, 2, 4096, 200),      # ... and beam: little LDS left for window segments (fallback path)
])
def test_wide_random_parity(T, B, V, beam):
    emis = oracle.synthetic_emissions(T, B, V, seed0=3000 + T + V + beam)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam), ref, f"T={T} B={B} V={V} beam={beam}")


def test_wide_flat_emissions():
    """Flat distributions (sigma 0.5): many label tiles per frame."""
    T, B, V, beam = 15, 3, 400, 30
    emis = oracle.synthetic_emissions(T, B, V, sigma=0.5, seed0=41)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam), ref, "flat")


def test_wide_uniform_ties():
    """All-equal emissions over 150 labels: 149 states tie at the cutoff,
    across three label tiles; all are kept (F2)."""
    T, V, beam = 2, 150, 10
    emis = np.full((T, 2, V), 1.0 / V, np.float32)
    ref = oracle.decode(emis, beam, 0, max_hyps=1000)
    assert max(len(r) for r in ref) > 2 * 64
    assert_beams_equal(gpu_beams(emis, beam, max_states=256), ref, "uniform")


def test_wide_tie_overflow_is_reported():
    """4761 tied states (uniform, V=70, T=3) exceed any capacity: reported."""
    emis = np.full((3, 1, 70), 1.0 / 70, np.float32)
    dec = asr.CTCDecoder(70, 10, 0, max_states=256)
    dec.decode(emis)
    with pytest.raises(asr.AsrError) as e:
        dec.best()
    assert e.value.status == asr.ASR_ERR_BEAM_OVERFLOW
    dec.close()


def test_wide_blank_last_and_codes_order():
    T, B, V, beam = 20, 3, 90, 12
    emis = oracle.synthetic_emissions(T, B, V, seed0=11)
    codes = [1000 + i for i in range(V - 1)] + [5]     # blank code below every symbol
    ref = oracle.decode(emis, beam, V - 1, codes=codes)
    assert_beams_equal(gpu_beams(emis, beam, V - 1, codes), ref, "blank=V-1")
    codes2 = [7000] + [100 + 3 * i for i in range(V - 1)]   # blank 0, largest code
    ref2 = oracle.decode(emis, beam, 0, codes=codes2)
    assert_beams_equal(gpu_beams(emis, beam, 0, codes2), ref2, "blank code max")


def test_wide_log_input_and_zeros():
    T, B, V, beam = 18, 3, 200, 16
    emis = oracle.synthetic_emissions(T, B, V, seed0=12)
    emis[3, :, 5:40] = 0.0
    emis[0, 1, :] = 0.0
    emis[0, 1, 7] = 1.0
    ref = oracle.decode(emis, beam, 0)
    assert_beams_equal(gpu_beams(emis, beam), ref, "zeros")
    lemis = np.log(np.maximum(oracle.synthetic_emissions(T, B, V, seed0=13), 1e-30)).astype(np.float32)
    ref2 = oracle.decode(lemis, beam, 0, is_log=True)
    assert_beams_equal(gpu_beams(lemis, beam, is_log=True), ref2, "is_log")


def test_wide_long_utterance_best():
    """Longer T: node records hold 4 x 16-bit labels; best path and score."""
    T, B, V, beam = 120, 2, 500, 20
    emis = oracle.synthetic_emissions(T, B, V, seed0=14)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads(), max_hyps=beam + 1)
    dec = asr.CTCDecoder(V, beam, 0)
    dec.decode(emis)
    best, lp = dec.best()
    for b in range(B):
        assert best[b] == ref[b][0][0]
        assert abs(lp[b] - ref[b][0][1]) <= 1e-9 * abs(ref[b][0][1])
    dec.close()


def test_wide_blank_dominant_frames():
    """The blank often carries the largest emission (as in trained CTC
    models): the selection's key bound must include it."""
    T, B, V, beam = 40, 2, 300, 100
    emis = oracle.synthetic_emissions(T, B, V, seed0=15).astype(np.float64)
    emis[::2, :, 0] *= 50.0                 # every other frame: blank dominant
    emis /= emis.sum(axis=2, keepdims=True)
    emis = emis.astype(np.float32)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
    assert_beams_equal(gpu_beams(emis, beam), ref, "blank dominant")


def test_wide_c5_longer():
    """BASELINE C5 vocabulary and beam over 40 frames (best path and score)."""
    T, B, V, beam = 40, 1, 1000, 200
    emis = oracle.synthetic_emissions(T, B, V, seed0=16)
    ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads(), max_hyps=beam + 1)
    assert_beams_equal([x[:beam + 1] for x in gpu_beams(emis, beam)], ref, "C5 T=40")


@pytest.mark.parametrize("semantics", [asr.SEMANTICS_CPU, asr.SEMANTICS_CUDA])
def test_wide_tile0_precompute_matches_in_kernel(monkeypatch, semantics):
    """V > 65: the first tile's threshold of every frame comes from
    ctc_tile0_kernel (a one-wave radix selection per frame before the
    decode); ASR_CTC_TILE0=0 makes the decode kernel select it itself.
    Both give the same beams, bit for bit: on frames whose 12 best labels
    are continuous and the rest take 6 log levels (ties at every tile
    threshold, few at the beam cutoff), and on continuous emissions."""
    T, B, V, beam = 30, 3, 500, 40
    rng = np.random.default_rng(5)
    logit = 0.5 * rng.integers(0, 6, size=(T, B, V)).astype(np.float64)
    for t in range(T):
        for b in range(B):
            logit[t, b, rng.permutation(V)[:12]] = 4.0 + 3.0 * rng.random(12)
    q = np.exp(logit)
    cases = {"tied tail": (q / q.sum(-1, keepdims=True)).astype(np.float32),
             "continuous": oracle.synthetic_emissions(T, B, V, seed0=77)}
    for name, emis in cases.items():
        got = {}
        for flag in ("1", "0"):
            monkeypatch.setenv("ASR_CTC_TILE0", flag)
            dec = asr.CTCDecoder(V, beam, 0)
            dec.set_semantics(semantics)
            dec.decode(emis)
            got[flag] = dec.beams(max_hyps=dec.config()[0])
            dec.close()
        assert got["1"] == got["0"], name
        if semantics == asr.SEMANTICS_CPU:
            ref = oracle.decode(emis, beam, 0, nthreads=cpu_threads())
            assert_beams_equal(got["1"], ref, name)

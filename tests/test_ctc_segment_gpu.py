"""Segmented (streaming) decode, asr_ctc_decode_segment: frames [t0, t1) at a
time with the beam carried on the device between segments (VERDICT r3 next
#3: a T-segmented handoff between production and decode).  The reference
decodes whole utterances only (CTCBeamSearch.cu:262-312; CPU path
CTCBeamSearch.cpp:50-187), so the contract is: a segmented decode is
bit-identical to the whole decode of the same frames — labels, ranks and
fp64 log-probs of the full final beam — for any split, with variable
utterance lengths ending inside, at and before segment boundaries; and the
whole decode is the oracle's (checked on a subset here as well)."""
import numpy as np
import pytest

from conftest import asr, cpu_threads, oracle
from test_ctc_gpu import assert_beams_equal

pytestmark = pytest.mark.gpu


def _segmented(d_em, T, B, V, beam, cuts, is_log, lengths=None, fs=None, us=None):
    fs = B * V if fs is None else fs
    us = V if us is None else us
    d = asr.CTCDecoder(V, beam, 0)
    bounds = [0] + list(cuts) + [T]
    for t0, t1 in zip(bounds, bounds[1:]):
        d.decode_segment(d_em.ptr + 4 * t0 * fs, T, t0, t1, B, is_log, lengths=lengths if t0 == 0 else None,
                         frame_stride=fs, utt_stride=us)
    beams = d.beams(max_hyps=d.config()[0])
    lab, lp = d.best()
    # the one-wave kernel carries the beam for V <= 63, the wide kernel (8 waves) above
    assert d.config()[1] == (asr.ASR_CTC_WAVES_LIST if V + 1 <= 64 else 8)
    d.close()
    return beams, lab, lp


def _whole(d_em, T, B, V, beam, is_log, lengths=None, waves=asr.ASR_CTC_WAVES_LIST, fs=None, us=None):
    d = asr.CTCDecoder(V, beam, 0, waves=waves)
    d.decode_device(d_em.ptr, T, B, is_log, lengths=lengths, frame_stride=fs, utt_stride=us)
    beams = d.beams(max_hyps=d.config()[0])
    lab, lp = d.best()
    d.close()
    return beams, lab, lp


def _same(a, b, what):
    assert a[1] == b[1], f"{what}: best labels differ"
    assert np.array_equal(a[2], b[2]), f"{what}: best log-probs differ"
    assert len(a[0]) == len(b[0])
    for u, (x, y) in enumerate(zip(a[0], b[0])):
        assert [l for l, _ in x] == [l for l, _ in y], f"{what}: utterance {u} ranked labels differ"
        assert [s for _, s in x] == [s for _, s in y], f"{what}: utterance {u} ranked scores differ"


@pytest.mark.parametrize("T,B,V,beam,cuts,sigma", [
    (120, 37, 29, 50, [40, 80], 3.0),
    (120, 37, 29, 50, [1, 2, 3, 119], 3.0),        # one-frame segments at both ends
    (97, 64, 29, 50, [13, 50, 51, 90], 0.5),       # flat emissions: many ties near the cutoff
    (80, 20, 47, 50, [33], 3.0),                   # V > 32: 64-bit child masks
    (60, 16, 29, 100, [7, 30], 3.0),               # beam 100: two rows per lane
    (64, 8, 5, 10, [8, 16, 24, 32, 40, 48, 56], 2.0),
])
def test_segmented_equals_whole(T, B, V, beam, cuts, sigma):
    emis = oracle.synthetic_emissions(T, B, V, seed0=777 + T, sigma=sigma)
    d_em = asr.DeviceMatrix.from_numpy(emis.reshape(T * B, V))
    seg = _segmented(d_em, T, B, V, beam, cuts, False)
    whole = _whole(d_em, T, B, V, beam, False)
    _same(seg, whole, f"cuts {cuts}")
    # and the whole decode is the oracle's (a subset)
    sub = list(range(0, B, max(1, B // 4)))[:4]
    ref = oracle.decode(np.ascontiguousarray(emis[:, sub, :]), beam, 0, nthreads=cpu_threads(), max_hyps=256)
    assert_beams_equal([seg[0][u] for u in sub], ref, f"segmented vs oracle, cuts {cuts}")


@pytest.mark.parametrize("T,B,V,beam,cuts,sigma,lengths", [
    (60, 6, 100, 20, [20, 40], 3.0, None),
    (48, 5, 1000, 200, [1, 24, 47], 2.0, None),          # C5's vocabulary and beam, one-frame segments
    (50, 7, 300, 40, [25], 1.0, [50, 25, 24, 26, 0, 1, 49]),   # lengths ending at / around the cut
])
def test_segmented_wide_equals_whole(T, B, V, beam, cuts, sigma, lengths):
    """V > 63: the wide kernel (8 waves per utterance, vocabulary tiles, the
    first tile of each frame precomputed per segment) carries its beam across
    segments too — the C5 pipeline hands the decode two T-segments.  Bit-
    identical to the whole decode, which is the oracle's on a subset."""
    emis = oracle.synthetic_emissions(T, B, V, seed0=919 + V, sigma=sigma)
    d_em = asr.DeviceMatrix.from_numpy(emis.reshape(T * B, V))
    seg = _segmented(d_em, T, B, V, beam, cuts, False, lengths=lengths)
    whole = _whole(d_em, T, B, V, beam, False, lengths=lengths, waves=0)
    _same(seg, whole, f"wide, cuts {cuts}")
    if V <= 300 and lengths is None:
        sub = [0, B - 1]
        ref = oracle.decode(np.ascontiguousarray(emis[:, sub, :]), beam, 0, nthreads=2, max_hyps=256)
        assert_beams_equal([seg[0][u] for u in sub], ref, f"wide segmented vs oracle, cuts {cuts}")


def test_segmented_with_lengths_and_strides():
    """Utterances ending inside a segment, exactly at a boundary, before the
    first cut, and with no frames at all; batch-major [B][T][V] strides."""
    T, B, V, beam = 90, 12, 29, 50
    cuts = [30, 60]
    lengths = [90, 30, 60, 31, 29, 0, 1, 59, 61, 89, 45, 15]
    emis = oracle.synthetic_emissions(T, B, V, seed0=4242, log=True)
    bm = np.ascontiguousarray(emis.transpose(1, 0, 2))     # [B][T][V]
    d_em = asr.DeviceMatrix.from_numpy(bm.reshape(B * T, V))
    seg = _segmented(d_em, T, B, V, beam, cuts, True, lengths=lengths, fs=V, us=T * V)
    whole = _whole(d_em, T, B, V, beam, True, lengths=lengths, fs=V, us=T * V)
    _same(seg, whole, "lengths")
    for b, n in enumerate(lengths):   # each utterance is the oracle's decode of its own frames
        if n == 0:
            assert seg[1][b] == [] and seg[2][b] == 0.0
            continue
        ref = oracle.decode(np.ascontiguousarray(emis[:n, b:b + 1, :]), beam, 0, is_log=True, max_hyps=1)
        assert seg[1][b] == [int(c) for c in ref[0][0][0]], f"utterance {b} (length {n})"
        assert abs(seg[2][b] - ref[0][0][1]) <= 1e-9 * max(1.0, abs(ref[0][0][1]))


def test_segment_errors():
    T, B, V, beam = 20, 4, 29, 10
    emis = oracle.synthetic_emissions(T, B, V, seed0=5)
    d_em = asr.DeviceMatrix.from_numpy(emis.reshape(T * B, V))
    d = asr.CTCDecoder(V, beam, 0)
    with pytest.raises(asr.AsrError) as e:          # must start at frame 0
        d.decode_segment(d_em.ptr, T, 5, 10, B, False)
    assert e.value.status == asr.ASR_ERR_STATE
    d.decode_segment(d_em.ptr, T, 0, 10, B, False)
    with pytest.raises(asr.AsrError) as e:          # results only after the last segment
        d.best()
    assert e.value.status == asr.ASR_ERR_STATE
    with pytest.raises(asr.AsrError) as e:          # out of order
        d.decode_segment(d_em.ptr, T, 12, 20, B, False)
    assert e.value.status == asr.ASR_ERR_STATE
    with pytest.raises(asr.AsrError) as e:          # a different batch shape mid-decode
        d.decode_segment(d_em.ptr + 4 * 10 * B * V, T, 10, 20, B - 1, False)
    assert e.value.status == asr.ASR_ERR_ARG
    d.decode_segment(d_em.ptr + 4 * 10 * B * V, T, 10, 20, B, False)
    lab, lp = d.best()
    d.close()
    assert (lab, lp.tolist()) == (lambda r: (r[1], r[2].tolist()))(_whole(d_em, T, B, V, beam, False))
    for setup in ("cu", "ts"):
        d = asr.CTCDecoder(V, beam, 0)
        if setup == "cu":
            d.set_semantics(asr.SEMANTICS_CUDA)
        else:
            d.set_timesteps(True)
        with pytest.raises(asr.AsrError) as e:
            d.decode_segment(d_em.ptr, T, 0, 10, B, False)
        assert e.value.status == asr.ASR_ERR_UNSUPPORTED
        d.close()
    Vw = 100   # the large-vocabulary kernel segments too (round 5), in CPU semantics only
    ew = asr.DeviceMatrix.from_numpy(oracle.synthetic_emissions(T, B, Vw, seed0=6).reshape(T * B, Vw))
    d = asr.CTCDecoder(Vw, beam, 0)
    d.set_semantics(asr.SEMANTICS_CUDA)
    with pytest.raises(asr.AsrError) as e:
        d.decode_segment(ew.ptr, T, 0, 10, B, False)
    assert e.value.status == asr.ASR_ERR_UNSUPPORTED
    d.close()


def test_segmented_overflow_retry_equals_whole():
    """a segmented decode whose beam overflows the automatic
    capacity (flat emissions: more tied survivors than max_states) is
    re-decoded whole at the results fetch, from the first segment's
    emission pointer and lengths; the result is the oracle's and the
    whole decode's, bit for bit."""
    T, B, V, beam = 8, 3, 4, 3
    uni = np.full((T, B, V), 1.0 / V, np.float32)
    ref = oracle.decode(uni, beam, 0, max_hyps=4096)
    d_em = asr.DeviceMatrix.from_numpy(uni.reshape(T * B, V))
    d = asr.CTCDecoder(V, beam, 0)
    assert d.config()[0] < max(len(r) for r in ref)   # the default capacity overflows
    for t0, t1 in ((0, 3), (3, 5), (5, T)):
        d.decode_segment(d_em.ptr + 4 * t0 * B * V, T, t0, t1, B, False)
    lab, lp = d.best()
    assert lab == [r[0][0] for r in ref]
    assert_beams_equal(d.beams(max_hyps=4096), ref, "segmented overflow retry")
    d.close()
    whole = _whole(d_em, T, B, V, beam, False, waves=0)
    assert lab == whole[1] and np.array_equal(lp, whole[2])

"""Timesteps mode (asr_ctc_set_timesteps): the frame at which every label of
every final hypothesis was appended — the ctcdecode `timesteps` output of the
Python baseline (baseline/main.py:46).  ctcdecode is not available here, so
the definition is the build's own (a continuing prefix keeps its labels'
frames, a new prefix is its parent's frames plus the current frame) and is
pinned against the oracle's restatement of it (OracleCTC::track_ts), decoded
on the same emissions: labels, ranks and frames identical."""
import numpy as np
import pytest

from conftest import asr, cpu_threads, oracle
from test_ctc_gpu import TOL

pytestmark = pytest.mark.gpu


def gpu_beams_ts(emis, beam, is_log=False, lengths=None, waves=0, max_states=0):
    dec = asr.CTCDecoder(emis.shape[2], beam, 0, max_states=max_states, waves=waves)
    dec.set_timesteps(True)
    dec.decode(emis, is_log=is_log, lengths=lengths)
    out = dec.beams_ts(max_hyps=256)   # the overflow retry may hold more than config()[0]
    plain = dec.beams(max_hyps=256)
    dec.close()
    # the labels and scores are those of the plain ranked beam
    assert [[(l, s) for l, s, _ in u] for u in out] == plain
    return out


def assert_ts_equal(got, ref, what):
    assert len(got) == len(ref)
    for b, (g, r) in enumerate(zip(got, ref)):
        assert [h[0] for h in g] == [h[0] for h in r], f"{what} utterance {b}: labels/ranks differ"
        for (_, x, tg), (_, y, tr) in zip(g, r):
            assert abs(x - y) <= TOL * max(1.0, abs(y))
            assert tg == tr, f"{what} utterance {b}: timesteps {tg[:12]}... vs {tr[:12]}..."


def check_monotone(beams, T):
    for u in beams:
        for lab, _, ts in u:
            assert len(ts) == len(lab)
            assert all(0 <= a < b < T for a, b in zip(ts, ts[1:])) and (not ts or 0 <= ts[0] < T)


@pytest.mark.parametrize("T,B,V,beam,sigma", [(60, 8, 29, 50, 3.0), (40, 6, 29, 10, 0.5), (50, 4, 8, 6, 3.0),
                                              (30, 4, 63, 20, 3.0)])
def test_timesteps_workgroup_kernel(T, B, V, beam, sigma):
    emis = oracle.synthetic_emissions(T, B, V, seed0=31 + V, sigma=sigma)
    got = gpu_beams_ts(emis, beam)
    ref = oracle.decode_ts(emis, beam, 0, nthreads=cpu_threads())
    assert_ts_equal(got, ref, f"T={T} V={V} beam={beam}")
    check_monotone(got, T)


def test_timesteps_long_utterance_many_blocks():
    """T = 300: hypotheses of ~270 labels span ~34 node records each."""
    T, B, V, beam = 300, 4, 29, 16
    emis = oracle.synthetic_emissions(T, B, V, seed0=77)
    got = gpu_beams_ts(emis, beam)
    ref = oracle.decode_ts(emis, beam, 0, nthreads=cpu_threads())
    assert_ts_equal(got, ref, "T=300")
    assert max(len(h[0]) for u in got for h in u) > 64


@pytest.mark.parametrize("T,B,V,beam", [(30, 4, 100, 16), (20, 2, 300, 40)])
def test_timesteps_wide_kernel(T, B, V, beam):
    emis = oracle.synthetic_emissions(T, B, V, seed0=5 + V)
    got = gpu_beams_ts(emis, beam)
    ref = oracle.decode_ts(emis, beam, 0, nthreads=cpu_threads())
    assert_ts_equal(got, ref, f"wide V={V}")
    check_monotone(got, T)


def test_timesteps_variable_lengths_and_list_schedule():
    """Per-utterance lengths; a handle asking for the one-wave list kernel
    runs the workgroup kernel while timesteps are on."""
    T, B, V, beam = 50, 5, 29, 12
    emis = oracle.synthetic_emissions(T, B, V, seed0=3)
    lens = [50, 1, 17, 33, 0]
    got = gpu_beams_ts(emis, beam, lengths=lens, waves=asr.ASR_CTC_WAVES_LIST)
    for b, n in enumerate(lens):
        if n == 0:
            continue
        ref = oracle.decode_ts(np.ascontiguousarray(emis[:n, b:b + 1, :]), beam, 0)
        assert_ts_equal([got[b]], ref, f"utterance {b} (length {n})")


def test_timesteps_through_overflow_retry():
    """Uniform emissions tie every candidate: the automatic capacity re-decodes
    with more room, and the retry handle tracks timesteps too."""
    T, B, V, beam = 8, 3, 4, 3   # > 64 tied states: two doublings of the default capacity
    emis = np.full((T, B, V), 1.0 / V, np.float32)
    got = gpu_beams_ts(emis, beam)
    ref = oracle.decode_ts(emis, beam, 0)
    assert max(len(r) for r in ref) > 64
    assert_ts_equal(got, ref, "uniform")


def test_timesteps_frame_limit_guard():
    """Frames are kept in 16 bits: with timesteps on, T > 65536 is refused
    before anything is enqueued (no silent wrap of frames >= 65536)."""
    dec = asr.CTCDecoder(29, 8, 0)
    dec.set_timesteps(True)
    buf = asr.DeviceBytes(4 * 29)   # never read: the guard runs first
    with pytest.raises(asr.AsrError) as ei:
        dec.decode_device(buf.ptr, asr.ASR_CTC_TS_MAX_T + 1, 1, is_log=True, frame_stride=1, utt_stride=1)
    assert ei.value.status == asr.ASR_ERR_UNSUPPORTED
    dec.close()


def test_beams_ts_requires_timesteps_mode():
    emis = oracle.synthetic_emissions(10, 2, 29, seed0=1)
    dec = asr.CTCDecoder(29, 8, 0)
    dec.decode(emis)
    with pytest.raises(asr.AsrError):
        dec.beams_ts(max_hyps=4)
    dec.close()

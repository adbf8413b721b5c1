"""Batch API: per-utterance lengths, batch-major emissions and the
ctcdecode-style CTCBeamDecoder mirror (the Python
baseline's decoder call baseline/main.py:29, 46).  Parity against the CPU
oracle decoding each utterance's own frames."""
import numpy as np
import pytest
import torch

from conftest import asr, cpu_threads, oracle
from test_ctc_gpu import assert_beams_equal

pytestmark = pytest.mark.gpu


def per_utterance_ref(emis_tbv, lengths, beam, is_log=False):
    out = []
    for b, n in enumerate(lengths):
        out.append(oracle.decode(np.ascontiguousarray(emis_tbv[:n, b:b + 1, :]), beam, 0,
                                 is_log=is_log)[0])
    return out


@pytest.mark.parametrize("V,beam", [(29, 10), (29, 50), (100, 16)])
def test_variable_lengths(V, beam):
    T, B = 60, 6
    emis = oracle.synthetic_emissions(T, B, V, seed0=500 + V)
    lengths = [60, 1, 30, 17, 45, 59]
    dec = asr.CTCDecoder(V, beam, 0)
    dec.decode(emis, lengths=lengths)
    got = dec.beams(dec.config()[0])
    assert_beams_equal(got, per_utterance_ref(emis, lengths, beam), f"lengths V={V}")
    best, lp = dec.best()
    assert [len(x) for x in best] == [len(g[0][0]) for g in got]
    dec.close()


def test_zero_length_utterance():
    emis = oracle.synthetic_emissions(10, 2, 29, seed0=7)
    dec = asr.CTCDecoder(29, 8, 0)
    dec.decode(emis, lengths=[10, 0])
    best, lp = dec.best()
    assert best[1] == [] and lp[1] == 0.0          # only the empty prefix (score log 1)
    ref = oracle.decode(np.ascontiguousarray(emis[:, :1, :]), 8, 0)
    assert best[0] == ref[0][0][0]
    dec.close()


def test_batch_major_equals_time_major():
    T, B, V = 40, 5, 29
    emis = oracle.synthetic_emissions(T, B, V, seed0=8)
    dec = asr.CTCDecoder(V, 20, 0)
    dec.decode(emis)
    a = dec.beams(dec.config()[0])
    dec.decode(np.ascontiguousarray(emis.transpose(1, 0, 2)), batch_major=True)
    b = dec.beams(dec.config()[0])
    assert a == b
    dec.close()


def test_ctcdecode_style_mirror_numpy_and_torch_gpu():
    T, B, V, beam = 50, 4, 29, 10
    emis = oracle.synthetic_emissions(T, B, V, seed0=9, log=True)     # log-probs, like model.py
    probs_btv = np.ascontiguousarray(emis.transpose(1, 0, 2))
    lens = np.array([50, 20, 35, 50], np.int32)
    dec = asr.CTCBeamDecoder(["$"] + [chr(65 + i) for i in range(V - 1)], beam_width=beam,
                             blank_id=0, num_processes=4, log_probs_input=True)
    res, scores, steps, out_lens = dec.decode(torch.from_numpy(probs_btv), torch.from_numpy(lens))
    assert res.shape == (B, beam, T) and scores.shape == (B, beam) and out_lens.shape == (B, beam)
    assert steps.shape == (B, beam, T)
    ref = per_utterance_ref(emis, lens, beam, is_log=True)
    for b in range(B):
        for k in range(beam):
            lab, lp = ref[b][k]
            assert out_lens[b, k] == len(lab)
            assert list(res[b, k, :len(lab)]) == lab
            assert abs(float(scores[b, k]) + lp) <= 1e-5 * max(1.0, abs(lp))
    # timesteps: each label's append frame, as the oracle tracks it
    for b in range(B):
        ref_ts = oracle.decode_ts(np.ascontiguousarray(emis[:lens[b], b:b + 1, :]), beam, 0, is_log=True)[0]
        for k in range(beam):
            lab, _, ts = ref_ts[k]
            assert list(steps[b, k, :len(lab)]) == ts, f"utterance {b} hypothesis {k}: timesteps differ"
            assert all(steps[b, k, len(lab):] == -1)
    # a GPU tensor is decoded in place (no host copy) and gives the same beams
    res2, scores2, _, lens2 = dec.decode(torch.from_numpy(probs_btv).cuda(), torch.from_numpy(lens))
    assert np.array_equal(res, res2) and np.array_equal(scores, scores2) and np.array_equal(out_lens, lens2)
    # timesteps=False: the same beams on the plain path, timesteps all -1
    dec3 = asr.CTCBeamDecoder(["$"] + [chr(65 + i) for i in range(V - 1)], beam_width=beam,
                              blank_id=0, log_probs_input=True, timesteps=False)
    res3, scores3, steps3, lens3 = dec3.decode(torch.from_numpy(probs_btv), torch.from_numpy(lens))
    assert np.array_equal(res, res3) and np.array_equal(scores, scores3) and np.array_equal(out_lens, lens3)
    assert (steps3 == -1).all()

"""BASELINE configs at full size on MI355X:

  C3  decode-only, B=256, T=1000, V=29, beam=100 (configs[2]);
  C4  one GPU's shard, B=256, T=1000, H=256, V=29, beam=50, end to end
      RNN -> Linear + log_softmax -> decode (configs[3]);
  C5  one GPU's shard, B=32, T=2000, H=1024, V=1000, beam=200, end to end
      (configs[4]);
  BL  the reference's own Python-harness workload, baseline/config.json:1-28
      (B=256, T=200, H=2048, V=47, beam=100), end to end.

Checked three ways:
  * against the CPU oracle (the CTCBeamSearch.cpp restatement): utterance
    subsets at full length from the committed fixture
    tests/golden/full_configs.json (tests/golden/make_full_config_golden.py
    decodes the same synthetic rows in the dev container), or decoded here on
    the GPU-produced emissions for the end-to-end cases — labels and ranks
    identical, log-probs within 1e-9 relative;
  * size-independent properties over the whole batch: best() is rank 0 of the
    ranked beam, ranks are sorted, labels are valid non-blank ids, no beam
    overflow is reported, and decoding the batch in two shards gives the
    full batch's rows bit for bit (what utterance sharding over GPUs relies
    on);
  * a second kernel schedule (4 waves per utterance instead of 8, V <= 63)
    must agree bit for bit; the automatic schedule is asserted (8 waves at
    B <= CUs, the packed 4-wave kernel at C4's one-GPU batch of 2048).
"""
import hashlib
import json
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, asr, cpu_threads, oracle
from test_ctc_gpu import assert_beams_equal

pytestmark = pytest.mark.gpu
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (the bench's model weights and per-utterance features)

FULL = json.loads((GOLDEN / "full_configs.json").read_text())


def labels_digest(beam):
    m = hashlib.sha256()
    for lab, _ in beam:
        m.update(np.asarray(lab, np.int32).tobytes())
        m.update(b"|")
    return m.hexdigest()


def decode_best(emis_dev_or_host, T, B, V, beam, is_log, waves=0):
    dec = asr.CTCDecoder(V, beam, 0, waves=waves)
    if isinstance(emis_dev_or_host, np.ndarray):
        dec.decode(emis_dev_or_host, is_log=is_log)
    else:
        dec.decode_device(emis_dev_or_host, T, B, is_log)
    lab, ln, lp = dec.best_arrays()
    out = [lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()
    return dec, out


def check_properties(dec, best, V, blank=0):
    """best() = rank 0 of the ranked beam; ranks sorted; labels valid."""
    labels, lp = best
    beams = dec.beams(max_hyps=dec.config()[0])
    for b, hyps in enumerate(beams):
        assert hyps, f"utterance {b}: empty final beam"
        assert hyps[0][0] == labels[b] and hyps[0][1] == lp[b], f"utterance {b}: best != rank 0"
        scores = [s for _, s in hyps]
        assert all(x >= y for x, y in zip(scores, scores[1:])), f"utterance {b}: ranks not sorted"
        assert np.isfinite(lp[b]) and lp[b] <= 0.0
        for lab, _ in hyps[:4]:
            assert all(0 <= c < V and c != blank for c in lab)
    return beams


def check_shards(emis, T, B, V, beam, is_log, best, waves=0):
    """Two shards decoded separately equal the full batch's rows bit for bit."""
    labels, lp = best
    h = B // 2
    for lo, hi in ((0, h), (h, B)):
        d, (l2, p2) = decode_best(np.ascontiguousarray(emis[:, lo:hi, :]), T, hi - lo, V, beam, is_log, waves)
        d.close()
        assert l2 == labels[lo:hi], f"shard [{lo},{hi}) labels differ from the full batch"
        assert np.array_equal(p2, lp[lo:hi]), f"shard [{lo},{hi}) log-probs differ from the full batch"


def check_fixture(name, emis_subset, dec_beams=None):
    g = FULL[name]
    d = asr.CTCDecoder(g["V"], g["beam"], 0)
    d.decode(emis_subset)
    beams = d.beams(max_hyps=d.config()[0])
    d.close()
    for i, u in enumerate(g["utterances"]):
        got = beams[i]
        assert [l for l, _ in got[:1]] == [g["best_labels"][i]], f"{name} utterance {u}: best differs"
        assert len(got) == g["n_hyps"][i], f"{name} utterance {u}: beam size differs"
        assert labels_digest(got) == g["beam_labels_sha256"][i], f"{name} utterance {u}: ranked beam differs"
        for (_, x), y in zip(got, g["beam_logp"][i]):
            assert abs(x - y) <= 1e-9 * max(1.0, abs(y)), f"{name} utterance {u}: {x} vs {y}"
    return beams


def test_c3_full_size():
    g = FULL["C3"]
    T, B, V, beam = g["T"], g["B"], g["V"], g["beam"]
    emis = oracle.synthetic_emissions(T, B, V, seed0=g["seed0"], sigma=g["sigma"])
    dec, best = decode_best(emis, T, B, V, beam, False)
    assert dec.config()[1] == 8
    check_properties(dec, best, V)
    dec.close()
    # oracle: 16 full-length utterances spread over the batch
    check_fixture("C3", np.ascontiguousarray(emis[:, g["utterances"], :]))
    sub_best = [best[0][u] for u in g["utterances"]]
    assert sub_best == g["best_labels"]
    check_shards(emis, T, B, V, beam, False, best)
    d4, best4 = decode_best(emis, T, B, V, beam, False, waves=4)
    d4.close()
    assert best4[0] == best[0] and np.array_equal(best4[1], best[1]), "4-wave schedule differs"


def _e2e(T, B, H, V, first=0):
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    x = DM(bench.make_features(T, B, H, first))
    hid, em = asr.DeviceMatrix(T * B, H), asr.DeviceMatrix(T * B, V)
    asr.rnn_fwd(x, DM(w_ih), DM(w_hh), DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1)), hid, T, B)
    asr.linear_fwd(hid, DM(w_out), DM(b_out.reshape(V, 1)), em, asr.EPI_BIAS_LOGSOFTMAX)
    asr.synchronize()
    e = em.toCpu().reshape(T, B, V)
    assert np.all(np.isfinite(e)) and np.all(e <= 0.0)
    # rows are log-probabilities: logsumexp over the vocabulary is 0
    assert np.abs(np.log(np.exp(e.astype(np.float64)).sum(-1))).max() < 1e-5
    return em, e


def test_c4_shard_full_size_e2e():
    T, B, H, V, beam = 1000, 256, 256, 29, 50
    em, e = _e2e(T, B, H, V)
    dec, best = decode_best(em.ptr, T, B, V, beam, True)
    assert dec.config()[1] == 8   # one utterance per CU: the 8-wave kernel
    check_properties(dec, best, V)
    dec.close()
    # oracle on the GPU-produced emissions, 8 full-length utterances
    sub = [0, 37, 64, 101, 128, 165, 200, 255]
    es = np.ascontiguousarray(e[:, sub, :])
    ref = oracle.decode(es, beam, 0, is_log=True, nthreads=cpu_threads(), max_hyps=128)
    d = asr.CTCDecoder(V, beam, 0)
    d.decode(es, is_log=True)
    assert_beams_equal(d.beams(max_hyps=d.config()[0]), ref, "C4 shard subset")
    d.close()
    assert [best[0][u] for u in sub] == [r[0][0] for r in ref]
    check_shards(e, T, B, V, beam, True, best)
    d4, best4 = decode_best(em.ptr, T, B, V, beam, True, waves=4)
    d4.close()
    assert best4[0] == best[0] and np.array_equal(best4[1], best[1]), "4-wave schedule differs"


def test_c4_one_gpu_full_batch_packed_schedule():
    """C4 on ONE GPU (the bench's N=1 line): 2048 utterances, 8 per CU, so
    the library's automatic schedule is the one-wave kernel, a dozen and more
    to a CU (runtime.hip auto_waves); it must agree bit for bit with the
    8-wave and the packed 4-wave schedules on the whole batch, and its first
    256 rows with a 256-utterance decode (one per CU, 8 waves: the 8-GPU
    shard shape)."""
    T, B, H, V, beam = 1000, 2048, 256, 29, 50
    em, e = _e2e(T, B, H, V)
    dec, best = decode_best(em.ptr, T, B, V, beam, True)
    assert dec.config()[1] == asr.ASR_CTC_WAVES_LIST, "automatic schedule at 8 per CU: the one-wave kernel"
    ms_auto = dec.last_kernel_ms()
    dec.close()
    times = {}
    for w in (8, 4):
        dw, bw = decode_best(em.ptr, T, B, V, beam, True, waves=w)
        assert dw.config()[1] == w
        times[w] = dw.last_kernel_ms()
        dw.close()
        assert bw[0] == best[0] and np.array_equal(bw[1], best[1]), f"{w}-wave schedule differs"
    ds = asr.CTCDecoder(V, beam, 0)   # rows [0, 256) in place: frame stride B*V
    ds.decode_device(em.ptr, T, 256, True, frame_stride=B * V, utt_stride=V)
    l256, p256 = ds.best()
    assert ds.config()[1] == 8
    ds.close()
    assert l256 == best[0][:256] and np.array_equal(p256, best[1][:256]), "256-utterance shard differs"
    print(f"C4 2048 x 1000 decode: auto (one wave) {ms_auto:.2f} ms, 4 waves {times[4]:.2f} ms, "
          f"8 waves {times[8]:.2f} ms")
    assert ms_auto < times[4] < times[8], "the automatic schedule should be the fastest at 8 per CU"


def test_c5_decode_fixture():
    g = FULL["C5_decode"]
    emis = np.concatenate([oracle.synthetic_emissions(g["T"], 1, g["V"], seed0=g["seed0"], first=u)
                           for u in g["utterances"]], axis=1)
    check_fixture("C5_decode", emis)


def test_c5_shard_full_size_e2e():
    T, B, H, V, beam = 2000, 32, 1024, 1000, 200
    em, e = _e2e(T, B, H, V)
    dec, best = decode_best(em.ptr, T, B, V, beam, True)
    check_properties(dec, best, V)
    dec.close()
    check_shards(e, T, B, V, beam, True, best)
    # oracle on a prefix of the GPU-produced emissions (the restatement does
    # ~1 frame/s per thread at V=1000, beam=200)
    Tp, sub = 24, [0, 31]
    es = np.ascontiguousarray(e[:Tp, sub, :])
    ref = oracle.decode(es, beam, 0, is_log=True, nthreads=2, max_hyps=512)
    d = asr.CTCDecoder(V, beam, 0)
    d.decode(es, is_log=True)
    assert_beams_equal(d.beams(max_hyps=d.config()[0]), ref, "C5 prefix")
    d.close()


def test_baseline_harness_workload_e2e():
    """baseline/config.json:1-28: seg_len 200, batch 256, rnn_hidden_size 2048,
    vocab 46 + blank, beam 100 (the reference's own Python harness)."""
    T, B, H, V, beam = 200, 256, 2048, 47, 100
    em, e = _e2e(T, B, H, V)
    dec, best = decode_best(em.ptr, T, B, V, beam, True)
    check_properties(dec, best, V)
    dec.close()
    check_shards(e, T, B, V, beam, True, best)
    sub = [0, 85, 170, 255]
    es = np.ascontiguousarray(e[:, sub, :])
    ref = oracle.decode(es, beam, 0, is_log=True, nthreads=cpu_threads(), max_hyps=256)
    d = asr.CTCDecoder(V, beam, 0)
    d.decode(es, is_log=True)
    assert_beams_equal(d.beams(max_hyps=d.config()[0]), ref, "BL subset")
    d.close()


@pytest.mark.parametrize("B", [2048, 1024])
def test_c4_pipeline_full_size_vs_oracle(B):
    """The bench's headline path exactly: the native
    pipeline at C4's one-GPU shape (T = 1000, H = 256, V = 29, beam 50; B =
    2048 as one batch, and 1024: the pipeline batch bench.py feeds C4's 2048
    utterances per GPU in on the split-bf16 arithmetic) with its automatic
    schedule — split-bf16 fused recurrence + emission kernel, the one-wave
    decoder 16 to a decode CU — against the oracle on 8 full-length
    utterances spread over the batch, decoded from the very emission bytes
    the pipeline's decode consumed (asr_pipeline_peek_emissions).  The whole
    batch must also equal a sequential decode of model_emissions (the same
    production, one call at a time)."""
    T, H, V, beam = 1000, 256, 29, 50
    (w_ih, w_hh, b_ih, b_hh), (w_out, b_out) = bench.make_weights(H, H, V)
    DM = asr.DeviceMatrix.from_numpy
    W = [DM(w_ih), DM(w_hh), DM(b_ih.reshape(H, 1)), DM(b_hh.reshape(H, 1)), DM(w_out), DM(b_out.reshape(V, 1))]
    x = DM(bench.make_features(T, B, H, 0))
    p = asr.Pipeline(T, B, H, H, V, beam, W)
    d = p.describe()
    assert d["mode"] == "chip-filling batches" and d["fused_emission"], d
    for _ in range(3):   # three batches in flight through the ring
        p.submit(x)
    outs = []
    while p.pending():
        lab, ln, lp, ms = p.collect()
        outs.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    assert d["decode_waves"] == asr.ASR_CTC_WAVES_LIST or p.describe()["decode_waves"] == asr.ASR_CTC_WAVES_LIST
    e = p.peek_emissions()
    p.close()
    for o in outs[1:]:
        assert o[0] == outs[0][0] and np.array_equal(o[1], outs[0][1]), "batches of the same input differ"
    labels, lp = outs[-1]
    # the pipeline's emissions are what model_emissions (one call at a time) gives
    em = asr.DeviceMatrix(T * B, V)
    asr.model_emissions(x, W, T, B, em, True)
    assert np.array_equal(em.toCpu().reshape(T, B, V), e), "model_emissions differs from the pipeline's emissions"
    sub = sorted({int(round(v)) for v in np.linspace(0, B - 1, 8)})
    ref = oracle.decode(np.ascontiguousarray(e[:, sub, :]), beam, 0, is_log=True, nthreads=cpu_threads(),
                        max_hyps=1)
    for i, u in enumerate(sub):
        assert labels[u] == [int(c) for c in ref[i][0][0]], f"utterance {u}: best labels differ from the oracle"
        assert abs(lp[u] - ref[i][0][1]) <= 1e-9 * max(1.0, abs(ref[i][0][1])), (u, lp[u], ref[i][0][1])


C5P = GOLDEN / "c5_production.json"


@pytest.mark.skipif(not C5P.exists(), reason="tests/golden/c5_production.json not generated")
def test_c5_production_full_length_vs_oracle(monkeypatch):
    """C5 on PRODUCTION emissions: the bench's C5 model
    (H = 1024, V = 1000, 32 utterances, T = 2000) through the library's fp32
    dense arithmetic, log_softmax emissions — where every frame appends a
    label and the wide kernel's orphan adoption fires — against the CPU
    oracle's decode of the same bytes over their first g["T"] frames
    (tests/golden/c5_production.json, written in the dev container by
    tests/golden/make_c5_production_golden.py from tools/dump_c5_emissions.py's
    dump; the emission digests tie the fixture to these bytes; the oracle's
    string work grows ~T^1.75 on such emissions, ~3 h per utterance at T =
    1000).  Four utterances:
      * the wide kernel, whole decode: best labels, beam size, ranked labels
        (digest) and every rank's log-prob within 1e-9 relative;
      * the same in two T-segments (the C5 pipeline's hand-off), bit for bit;
      * with every orphan adoption forced through the one-thread scan that
        runs past 128 filter hits per frame (ASR_CTC_WIDE_ADOPT_CAP=1), bit
        for bit;
      * the four rows inside the whole 32-utterance batch, bit for bit.
    Then the full T = 2000 of the four utterances: whole = two T-segments
    (property, bit for bit)."""
    sys.path.insert(0, str(ROOT / "tools"))
    import dump_c5_emissions as c5
    g = json.loads(C5P.read_text())
    e, em = c5.production_emissions(asr)
    T, B, V, beam = g["T"], g["B"], g["V"], g["beam"]
    Tp = g.get("T_production", T)
    assert e.shape == (Tp, B, V)
    uids = g["utterances"]
    for u, d in zip(uids, g["emis_sha256"]):
        assert c5.digest(e[:, u, :]) == d, f"utterance {u}: emissions differ from the fixture's (regenerate it)"
    sub = np.ascontiguousarray(e[:T, uids, :])
    d_sub = asr.DeviceMatrix.from_numpy(sub.reshape(T * len(uids), V))

    def run(segments, d_src=None, Tr=None, ns=None):
        d_src = d_sub if d_src is None else d_src
        Tr = T if Tr is None else Tr
        n = len(uids)
        d = asr.CTCDecoder(V, beam, 0)
        if segments:
            cut = Tr * 5 // 9
            for t0, t1 in ((0, cut), (cut, Tr)):
                d.decode_segment(d_src.ptr + 4 * t0 * n * V, Tr, t0, t1, n, True)
        else:
            d.decode_device(d_src.ptr, Tr, n, True)
        assert d.config()[1] == 8   # the wide kernel
        beams = d.beams(max_hyps=d.config()[0])
        d.close()
        return beams

    whole = run(False)
    for i, u in enumerate(uids):
        got = whole[i]
        assert got[0][0] == g["best_labels"][i], f"utterance {u}: best differs from the oracle"
        assert len(got) == g["n_hyps"][i], f"utterance {u}: beam size differs"
        assert labels_digest(got) == g["beam_labels_sha256"][i], f"utterance {u}: ranked beam differs"
        for (_, x), y in zip(got, g["beam_logp"][i]):
            assert abs(x - y) <= 1e-9 * max(1.0, abs(y)), f"utterance {u}: {x} vs {y}"

    def same(a, what):
        for i in range(len(uids)):
            assert [l for l, _ in a[i]] == [l for l, _ in whole[i]], f"{what}: utterance {uids[i]} labels"
            assert [s for _, s in a[i]] == [s for _, s in whole[i]], f"{what}: utterance {uids[i]} scores"

    same(run(True), "two T-segments")
    monkeypatch.setenv("ASR_CTC_WIDE_ADOPT_CAP", "1")
    same(run(False), "adoptions through the one-thread scan")
    monkeypatch.delenv("ASR_CTC_WIDE_ADOPT_CAP")
    # the four rows inside the whole 32-utterance batch (its first T frames)
    dec = asr.CTCDecoder(V, beam, 0)
    dec.decode_device(em.ptr, T, B, True)
    lab, lp = dec.best()
    dec.close()
    for i, u in enumerate(uids):
        assert lab[u] == whole[i][0][0] and lp[u] == whole[i][0][1], f"utterance {u} in the batch"
    if Tp > T:   # C5's full T: whole = two T-segments, bit for bit
        full = asr.DeviceMatrix.from_numpy(np.ascontiguousarray(e[:, uids, :]).reshape(Tp * len(uids), V))
        a, b = run(False, full, Tp), run(True, full, Tp)
        for i in range(len(uids)):
            assert [l for l, _ in a[i]] == [l for l, _ in b[i]] and [x for _, x in a[i]] == [x for _, x in b[i]], uids[i]

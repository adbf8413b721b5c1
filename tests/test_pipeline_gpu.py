"""Native throughput pipeline (asr_pipeline_*): RNN -> Linear + log_softmax ->
CTC decode over a stream of batches, production and decodes overlapped on
library-owned streams.  Every batch's results must be exactly those of the
same batch run one call at a time (asr_rnn_fwd, asr_linear_fwd,
asr_ctc_decode), in every schedule the library picks (CU groups for small
batches, chip-filling batches, H > 256), for any submit / collect
interleaving (the pipeline fetches results itself when the caller falls a
whole buffer ring behind)."""
import numpy as np
import pytest

from conftest import asr

pytestmark = pytest.mark.gpu


def _weights(inp, H, V, seed):
    rng = np.random.default_rng(seed)
    s = 1 / np.sqrt(H)
    host = [rng.uniform(-s, s, (inp, H)), rng.uniform(-s, s, (H, H)), rng.uniform(-0.1, 0.1, (H, 1)),
            rng.uniform(-0.1, 0.1, (H, 1)), rng.uniform(-4 * s, 4 * s, (H, V)), rng.uniform(-0.5, 0.5, (V, 1))]
    return [asr.DeviceMatrix.from_numpy(np.asarray(a, np.float32)) for a in host]


def _sequential(x, W, T, B, inp, H, V, beam, recur, fused=False):
    asr.rnn_set_recurrence(recur)
    try:
        em = asr.DeviceMatrix(T * B, V)
        asr.model_emissions(x, W, T, B, em, fused)
        dec = asr.CTCDecoder(V, beam, 0)
        dec.decode_device(em.ptr, T, B, is_log=True)
        lab, ln, lp = dec.best_arrays()
        out = ([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy())
        dec.close()
        return out
    finally:
        asr.rnn_set_recurrence(asr.RNN_RECUR_AUTO)


@pytest.mark.parametrize("T,B,inp,H,V,beam,mode,recur", [
    (60, 16, 64, 64, 29, 10, "CU groups (small batches)", asr.RNN_RECUR_AUTO),
    (40, 256, 48, 64, 29, 50, "chip-filling batches", asr.RNN_RECUR_MFMA),
    (40, 512, 48, 64, 47, 50, "chip-filling batches", asr.RNN_RECUR_MFMA),   # V > 32: not fused
    (30, 300, 32, 64, 29, 100, "chip-filling batches", asr.RNN_RECUR_MFMA),  # beam 100 (C3-like): fused
    (12, 300, 32, 384, 47, 60, "chip-filling batches", asr.RNN_RECUR_AUTO),  # H > 256 (BL-like)
    (20, 8, 32, 384, 29, 8, "CU groups (H > 256)", asr.RNN_RECUR_AUTO),
    # H > 256 with the wide decoder (C5-like): two T-segments, the one-launch recurrence
    (24, 16, 32, 384, 100, 12, "CU groups (H > 256)", asr.RNN_RECUR_AUTO),
])
def test_pipeline_matches_sequential(T, B, inp, H, V, beam, mode, recur):
    W = _weights(inp, H, V, seed=T + B + H)
    rng = np.random.default_rng(7)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(7)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["mode"] == mode, d
    got = []

    def take():
        lab, ln, lp, ms = p.collect()
        assert ms > 0.0
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))

    # submit ahead of collecting, past the buffer ring (the pipeline then
    # fetches the oldest results itself), then interleave
    for x in xs[:5]:
        p.submit(x)
    take()
    take()
    for x in xs[5:]:
        p.submit(x)
    while p.pending():
        take()
    p.close()
    assert len(got) == len(xs)
    for i, x in enumerate(xs):
        ref = _sequential(x, W, T, B, inp, H, V, beam, recur, d["fused_emission"])
        assert got[i][0] == ref[0], f"batch {i}: labels differ ({d})"
        assert np.array_equal(got[i][1], ref[1]), f"batch {i}: log-probs differ ({d})"


def test_pipeline_explicit_schedule_and_shared_cus():
    """Explicit knobs: every stream on every CU (decode_cus = -1) and a given
    number of decodes in flight; same results."""
    T, B, inp, H, V, beam = 30, 300, 32, 48, 29, 20
    W = _weights(inp, H, V, seed=3)
    x = asr.DeviceMatrix.from_numpy(np.random.default_rng(1).uniform(-1, 1, (T * B, inp)).astype(np.float32))
    p = asr.Pipeline(T, B, inp, H, V, beam, W, inflight=2, prod_streams=1, decode_cus=-1)
    d = p.describe()
    assert d["inflight"] == 2 and d["prod_streams"] == 1 and d["decode_cus"] >= 256
    for _ in range(3):
        p.submit(x)
    outs = []
    for _ in range(3):
        lab, ln, lp, _ = p.collect()
        outs.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    assert d["fused_emission"]   # chip-filling batch, V <= 32
    ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
    for o in outs:
        assert o[0] == ref[0] and np.array_equal(o[1], ref[1])


@pytest.mark.parametrize("gsplit", ["0.3", "1.0"])
def test_pipeline_input_projection_on_decode_cus(gsplit, monkeypatch):
    """ASR_PIPELINE_GSPLIT: part (or all) of each batch's input projection on
    the decode CUs' stream; rows are independent, so the results are the
    sequential fused production's bits."""
    monkeypatch.setenv("ASR_PIPELINE_GSPLIT", gsplit)
    T, B, inp, H, V, beam = 24, 600, 64, 256, 29, 30
    W = _weights(inp, H, V, seed=11)
    rng = np.random.default_rng(5)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(4)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["mode"] == "chip-filling batches" and d["fused_emission"], d
    assert d["decode_cu_gemm_rows"] == int(float(gsplit) * T * B) // 128 * 128, d
    for x in xs:
        p.submit(x)
    got = []
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    for g, x in zip(got, xs):
        ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])


@pytest.mark.parametrize("B,stage", [(16, "head"), (16, "tail"), (300, "produce"), (300, "decode")])
def test_pipeline_failure_is_reported(B, stage, monkeypatch):
    """A batch whose production cannot be queued is not accepted (the error
    comes back, the pipeline is unchanged); a failure in an accepted batch's
    later work fails the pipeline from that batch on — its collect and every
    later call return the error, never another batch's stale results — while
    earlier batches are still collected normally.  The
    library's test hook ASR_PIPELINE_FAULT=<batch>:<stage> fails one stage
    of one batch once."""
    T, inp, H, V, beam = 20, 32, 64, 29, 10
    monkeypatch.setenv("ASR_PIPELINE_FAULT", f"2:{stage}")
    W = _weights(inp, H, V, seed=5)
    rng = np.random.default_rng(9)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(5)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert (d["mode"] == "CU groups (small batches)") == (B == 16), d

    def ref(x):
        return _sequential(x, W, T, B, inp, H, V, beam, d["recurrence"], d["fused_emission"])

    def take():
        lab, ln, lp, _ = p.collect()
        return [lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()

    p.submit(xs[0])
    p.submit(xs[1])
    if stage in ("head", "produce"):   # batch 2 is refused, nothing else changes
        with pytest.raises(asr.AsrError) as ei:
            p.submit(xs[2])
        assert ei.value.status == asr.ASR_ERR_INTERNAL
        assert p.pending() == 2
        p.submit(xs[3])   # accepted as batch 2
        got = [take() for _ in range(3)]
        for g, x in zip(got, (xs[0], xs[1], xs[3])):
            r = ref(x)
            assert g[0] == r[0] and np.array_equal(g[1], r[1])
    else:
        # tail: batch 2's emission GEMM + decode are queued by the submit of
        # batch 3 (split schedule); decode: by batch 2's own submit
        if stage == "tail":
            p.submit(xs[2])
            with pytest.raises(asr.AsrError):
                p.submit(xs[3])
        else:
            with pytest.raises(asr.AsrError):
                p.submit(xs[2])
        for i in range(2):   # batches 0 and 1 were fine
            g, r = take(), ref(xs[i])
            assert g[0] == r[0] and np.array_equal(g[1], r[1])
        with pytest.raises(asr.AsrError) as ei:   # batch 2: the error, not stale results
            p.collect()
        assert ei.value.status == asr.ASR_ERR_INTERNAL
        with pytest.raises(asr.AsrError):
            p.submit(xs[4])
    p.close()


@pytest.mark.parametrize("segments,B", [(2, 300), (3, 600), (5, 256)])
def test_pipeline_segmented_handoff(segments, B):
    """T-segmented handoff (asr_pipeline_config.segments): the fused
    production publishes each segment's emissions and the decode of that
    segment starts behind it (asr_ctc_decode_segment), the recurrence
    carrying h across segments.  Same bits as the sequential fused
    production + whole decode, batch for batch."""
    T, inp, H, V, beam = 37, 48, 64, 29, 40
    W = _weights(inp, H, V, seed=segments)
    rng = np.random.default_rng(segments)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(4)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W, segments=segments)
    d = p.describe()
    assert d["mode"] == "chip-filling batches" and d["fused_emission"] and d["segments"] == segments, d
    for x in xs:
        p.submit(x)
    got = []
    while p.pending():
        lab, ln, lp, ms = p.collect()
        assert ms > 0.0
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    assert p.describe()["decode_waves"] == asr.ASR_CTC_WAVES_LIST
    p.close()
    for g, x in zip(got, xs):
        ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])


def test_pipeline_persistent_recurrence_fault_recovers(monkeypatch):
    """The pipeline path of the fail-safe one-launch recurrence (H > 256,
    C5-like): batch 1's recurrence launches run with one workgroup stalled
    (ASR_RNN_PERSIST_FAULT), give up and are finished by their recovery
    kernels; every batch — the faulted one and the later ones — collects the
    sequential path's bits, and nothing fails the pipeline."""
    T, B, inp, H, V, beam = 24, 16, 32, 384, 100, 12
    W = _weights(inp, H, V, seed=41)
    rng = np.random.default_rng(41)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(4)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["mode"] == "CU groups (H > 256)", d
    n0, r0 = asr.rnn_persist_stats()
    got = []
    for i, x in enumerate(xs):
        if i == 1:
            monkeypatch.setenv("ASR_RNN_PERSIST_FAULT", "5")
        p.submit(x)
        monkeypatch.delenv("ASR_RNN_PERSIST_FAULT", raising=False)
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    n1, r1 = asr.rnn_persist_stats()
    assert n1 - n0 == 4 * d["segments"], (n0, n1, d)   # one launch per batch and T-segment
    assert r1 - r0 >= 1, (r0, r1)                      # batch 1's segments that reached frame 5
    for g, x in zip(got, xs):
        ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_AUTO)
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])


@pytest.mark.parametrize("drain,seg0,B", [("-1", "", 300), ("-1", "0.3", 300), ("2", "0.25", 600), ("", "0.4", 256)])
def test_pipeline_drain_schedule(drain, seg0, B, monkeypatch):
    """The drain schedule (ASR_PIPELINE_DRAIN: the last decode segment of the
    newest batches held back, released onto its decode stream by newer
    batches or onto its production stream when the caller drains) and an
    uneven first T-segment (ASR_PIPELINE_SEG0) only move work between streams
    and CUs: every batch equals the sequential fused production + whole
    decode, with submits ahead of collects, interleaved, and a drain in the
    middle (collect everything, then submit more)."""
    if drain:
        monkeypatch.setenv("ASR_PIPELINE_DRAIN", drain)
    if seg0:
        monkeypatch.setenv("ASR_PIPELINE_SEG0", seg0)
    T, inp, H, V, beam = 41, 48, 64, 29, 40
    W = _weights(inp, H, V, seed=B + 3)
    rng = np.random.default_rng(B)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(3)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W, segments=2)
    d = p.describe()
    assert d["mode"] == "chip-filling batches" and d["segments"] == 2, d
    order = [0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2]
    got = []

    def take():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))

    for i in order[:9]:   # a ring's worth ahead, then collects interleaved
        p.submit(xs[i])
        if p.pending() > 6:
            take()
    while p.pending():    # the caller drains
        take()
    for i in order[9:]:   # and the pipeline goes on
        p.submit(xs[i])
    while p.pending():
        take()
    p.close()
    assert len(got) == len(order)
    refs = [_sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True) for x in xs]
    for g, i in zip(got, order):
        assert g[0] == refs[i][0] and np.array_equal(g[1], refs[i][1]), f"input {i}"


@pytest.mark.parametrize("group", ["2", "3"])
def test_pipeline_production_groups(group, monkeypatch):
    """H > 256 (C5-like): the recurrences of G consecutive batches run as one
    (one per-frame MFMA step launch for all of them); a partial group is
    produced when its results are asked for.  Same bits as one batch at a
    time (asr_rnn_fwd + asr_linear_fwd + asr_ctc_decode)."""
    monkeypatch.setenv("ASR_PIPELINE_GROUP", group)
    T, B, inp, H, V, beam = 16, 16, 32, 384, 70, 12
    W = _weights(inp, H, V, seed=int(group))
    rng = np.random.default_rng(int(group))
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(5)]
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["mode"] == "CU groups (H > 256)" and d["groups"] == int(group), d
    got = []
    for i, x in enumerate(xs):
        p.submit(x)
        if i == 1:   # batch 0 asked for before its group is complete
            lab, ln, lp, _ = p.collect()
            got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    assert len(got) == len(xs)
    for g, x in zip(got, xs):
        ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_AUTO)
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])


def test_pipeline_fits_hw_queues(monkeypatch):
    """HIP maps only the UNMASKED streams onto its GPU_MAX_HW_QUEUES hardware
    queues; a CU-masked stream gets a queue of its own (round 6, run r6b: C4
    / 256 per GPU / C2 at 4 queues with the 24-queue schedule kept ran as
    fast as at 24).  So asr_pipeline_create fits only its unmasked streams
    to the count it reads: the chip-filling schedule, whose decode and
    production streams are masked, keeps its decodes, productions and the
    decode CUs' share of the input projection at 4 queues, with no stream
    sharing HIP's queues; with every stream on every CU (decode_cus = -1)
    the unmasked streams are fitted to the 4 queues; explicit counts are
    kept.  The results are the same bits either way.  (The decode CUs'
    share is requested explicitly: the split-bf16 arithmetic's default is
    none.)"""
    monkeypatch.setenv("ASR_PIPELINE_GSPLIT", "0.3")
    T, B, inp, H, V, beam = 24, 600, 64, 256, 29, 30
    W = _weights(inp, H, V, seed=13)
    x = asr.DeviceMatrix.from_numpy(np.random.default_rng(2).uniform(-1, 1, (T * B, inp)).astype(np.float32))
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    full = asr.Pipeline(T, B, inp, H, V, beam, W).describe()
    assert full["hw_queues"] == 24 and full["decode_cu_gemm_rows"] > 0, full
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["hw_queues"] == 4 and d["shared_queue_streams"] == 0, d
    assert d["dedicated_queue_streams"] == d["streams"] > 4, d
    for k in ("inflight", "prod_streams", "decode_cu_gemm_rows"):
        assert d[k] == full[k], (k, d, full)
    for _ in range(3):
        p.submit(x)
    got = []
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
    for g in got:
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])
    u = asr.Pipeline(T, B, inp, H, V, beam, W, decode_cus=-1)   # every stream unmasked: fitted
    du = u.describe()
    u.close()
    assert du["dedicated_queue_streams"] == 0 and 0 < du["shared_queue_streams"] <= 4, du
    q = asr.Pipeline(T, B, inp, H, V, beam, W, inflight=3, prod_streams=3, decode_cus=-1)   # explicit: kept
    dq = q.describe()
    q.close()
    assert dq["inflight"] == 3 and dq["prod_streams"] == 3 and dq["shared_queue_streams"] > 4, dq


def _covers(pl, ncu):
    """Every CU is in a decode range or the production range, and no decode
    range overlaps the production range."""
    rs = pl.placement()
    dec = [(lo, hi) for r, lo, hi in rs if r == "decode"]
    prod = [(lo, hi) for r, lo, hi in rs if r == "production"]
    assert dec and prod, rs
    cov = np.zeros(ncu, bool)
    for lo, hi in dec + prod:
        cov[lo:hi] = True
    assert cov.all(), (rs, np.flatnonzero(~cov))
    for dlo, dhi in dec:
        for plo, phi in prod:
            if (dlo, dhi) != (0, ncu) and (plo, phi) != (0, ncu):
                assert dhi <= plo or phi <= dlo, rs
    return rs


@pytest.mark.parametrize("T,B,inp,H,V,beam,mode", [
    (24, 48, 64, 256, 29, 50, "CU groups (small batches)"),
    (16, 32, 32, 384, 29, 8, "CU groups (H > 256)"),
])
def test_pipeline_groups_fit_hw_queues(monkeypatch, T, B, inp, H, V, beam, mode):
    """the CU groups are laid out from the decode count that the
    hardware-queue fit leaves (only the unmasked GEMM streams count against
    HIP's default of 4 queues; the masked decode groups and production keep
    their own): every CU is then in a decode group or in production, never
    in neither, and the results are the sequential ones."""
    import torch
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    W = _weights(inp, H, V, seed=B + H)
    x = asr.DeviceMatrix.from_numpy(np.random.default_rng(5).uniform(-1, 1, (T * B, inp)).astype(np.float32))
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    full = asr.Pipeline(T, B, inp, H, V, beam, W)
    full_d = full.describe()
    assert full_d["mode"] == mode
    _covers(full, ncu)
    full.close()
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    d = p.describe()
    assert d["hw_queues"] == 4 and d["shared_queue_streams"] <= 4, d
    assert d["inflight"] == full_d["inflight"], (d, full_d)
    rs = _covers(p, ncu)
    ndec = len({(lo, hi) for r, lo, hi in rs if r == "decode"})
    assert ndec == min(d["inflight"], len([r for r in rs if r[0] == "decode"])), (rs, d)
    for _ in range(3):
        p.submit(x)
    got = []
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    p.close()
    ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_AUTO)
    for g in got:
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])


def test_pipeline_timeline_and_probe():
    """asr_pipeline_set_timing / get_timeline: one record per batch collected
    after the call, stamps ordered within each stage; the results are those
    of an untimed run.  asr_pipeline_probe_placement: the decode and
    production roles reach CUs on every XCD, at most their ranges' CUs."""
    T, B, inp, H, V, beam = 24, 600, 64, 256, 29, 30
    W = _weights(inp, H, V, seed=21)
    x = asr.DeviceMatrix.from_numpy(np.random.default_rng(3).uniform(-1, 1, (T * B, inp)).astype(np.float32))
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    p.submit(x)
    p.collect()
    p.set_timing(True)
    n = 5
    got = []
    for _ in range(n):
        p.submit(x)
    while p.pending():
        lab, ln, lp, _ = p.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
    bid, st = p.timeline()
    assert list(bid) == list(range(1, 1 + n)), bid
    assert (st >= 0).all() and (st[:, 1] >= st[:, 0]).all() and (st[:, 3] >= st[:, 2]).all(), st
    assert (st[:, 3] >= st[:, 0]).all(), st
    ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
    for g in got:
        assert g[0] == ref[0] and np.array_equal(g[1], ref[1])
    rs = p.placement()
    for role in ("decode", "production"):
        lo, hi = next((lo, hi) for r, lo, hi in rs if r == role)
        per = p.probe_placement(role)
        assert len(per) >= 1 and all(c > 0 for c in per) and sum(per) <= hi - lo, (role, per, lo, hi)
    p.close()


def test_pipeline_latches_dense_arith():
    """A pipeline keeps the dense arithmetic it was created under
    (asr_set_dense_arith changes the process-wide setting for later calls
    only): batches submitted and collected after a switch to fp32 are the
    split-bf16 production's bits, equal to a sequential split-bf16 decode;
    a pipeline created after the switch runs fp32 and its emissions differ."""
    T, B, inp, H, V, beam = 24, 600, 64, 256, 29, 30
    W = _weights(inp, H, V, seed=17)
    x = asr.DeviceMatrix.from_numpy(np.random.default_rng(9).uniform(-1, 1, (T * B, inp)).astype(np.float32))
    assert asr.get_dense_arith() == asr.DENSE_SPLIT_BF16
    ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
    em_split = asr.DeviceMatrix(T * B, V)
    asr.model_emissions(x, W, T, B, em_split, True, recurrence=asr.RNN_RECUR_MFMA)
    p = asr.Pipeline(T, B, inp, H, V, beam, W)
    p.submit(x)
    asr.set_dense_arith(asr.DENSE_F32)
    try:
        p.submit(x)
        got = []
        while p.pending():
            lab, ln, lp, _ = p.collect()
            got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
        assert np.array_equal(p.peek_emissions(), em_split.toCpu().reshape(T, B, V))
        p.close()
        for g in got:
            assert g[0] == ref[0] and np.array_equal(g[1], ref[1])
        q = asr.Pipeline(T, B, inp, H, V, beam, W)
        q.submit(x)
        q.collect()
        assert not np.array_equal(q.peek_emissions(), em_split.toCpu().reshape(T, B, V))
        q.close()
    finally:
        asr.set_dense_arith(asr.DENSE_SPLIT_BF16)


@pytest.mark.parametrize("group,B,n,interleave", [(4, 64, 10, False), (2, 256, 5, False), (3, 96, 7, True)])
def test_pipeline_coalesced_matches_sequential(group, B, n, interleave):
    """Dynamic batching (asr_pipeline_create_coalesced): `group` submits of B
    utterances run as one chip-filling batch of group * B; every submit's
    results are the sequential fused production + decode of its own B
    utterances, bit for bit and in submission order, with a partial batch (n
    not a multiple of group, or collects interleaved with submits) completed
    by zero-feature padding; peek_emissions returns the submit's own
    columns, the bytes model_emissions computes for it alone."""
    T, inp, H, V, beam = 41, 48, 64, 29, 30
    W = _weights(inp, H, V, seed=group)
    rng = np.random.default_rng(group + B)
    xs = [asr.DeviceMatrix.from_numpy(rng.uniform(-1, 1, (T * B, inp)).astype(np.float32)) for _ in range(n)]
    pl = asr.Pipeline(T, B, inp, H, V, beam, W, coalesce=group)
    d = pl.describe()
    assert d["coalesce"] == group and d["mode"] == "chip-filling batches" and d["fused_emission"], d
    got, ems = [], []

    def take():
        lab, ln, lp, ms = pl.collect()
        got.append(([lab[b, :ln[b]].tolist() for b in range(B)], lp.copy()))
        ems.append(pl.peek_emissions())

    for i, x in enumerate(xs):
        pl.submit(x)
        if interleave and i % 3 == 1:
            take()
    while pl.pending():
        take()
    pl.close()
    assert len(got) == n
    asr.rnn_set_recurrence(asr.RNN_RECUR_MFMA)
    try:
        for i, x in enumerate(xs):
            ref = _sequential(x, W, T, B, inp, H, V, beam, asr.RNN_RECUR_MFMA, fused=True)
            assert got[i][0] == ref[0] and np.array_equal(got[i][1], ref[1]), f"submit {i}"
            em = asr.DeviceMatrix(T * B, V)
            asr.model_emissions(x, W, T, B, em, True, recurrence=d["recurrence"])
            assert np.array_equal(em.toCpu().reshape(T, B, V), ems[i]), f"submit {i}: emissions"
    finally:
        asr.rnn_set_recurrence(asr.RNN_RECUR_AUTO)

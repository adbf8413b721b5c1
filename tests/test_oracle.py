"""CPU tests of the parity oracle (oracle/ctc_oracle.cpp) — no GPU needed.

Pins the restatement of /root/reference/CTCBeamSearch.cpp three ways:
golden values of the reference's own test vector (main.cpp:51-60),
exhaustive CTC enumeration (no pruning => exact prefix probabilities), and
agreement with the literal fp32 probability-domain arithmetic at short T.
"""
import itertools
import json
import math

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, oracle


def _collapse(path, blank):
    out, prev = [], None
    for s in path:
        if s != prev and s != blank:
            out.append(s)
        prev = s
    return tuple(out)


def brute_force(emis, blank):
    """Exact P(prefix) for one utterance by enumerating all V^T alignments."""
    T, V = emis.shape
    le = np.log(emis.astype(np.float64))
    acc = {}
    for path in itertools.product(range(V), repeat=T):
        lp = float(sum(le[t, s] for t, s in enumerate(path)))
        q = _collapse(path, blank)
        acc.setdefault(q, []).append(lp)
    return {q: float(np.logaddexp.reduce(v)) for q, v in acc.items()}


def test_main_cpp_golden():
    g = json.loads((GOLDEN / "main_cpp_ctc.json").read_text())
    emis = np.array(g["emissions"], np.float32).reshape(g["T"], 1, g["V"])
    codes = [ord(c) for c in g["vocab"]]
    got = oracle.decode(emis, g["beam"], g["blank"], codes)[0]
    s = lambda lab: "".join(g["vocab"][i] for i in lab)
    assert [s(l) for l, _ in got] == [x[0] for x in g["expected_log"]]
    for (l, lp), (_, e) in zip(got, g["expected_log"]):
        assert lp == pytest.approx(e, abs=1e-12)
    # compiled fixed reference gave cbacbc / -5.681380 / 0.0034088497
    assert s(got[0][0]) == g["survey_A6"]["best"]
    assert got[0][1] == pytest.approx(g["survey_A6"]["logp"], abs=5e-6)
    prob = oracle.decode(emis, g["beam"], g["blank"], codes, prob_domain=True)[0]
    assert prob[0][1] == pytest.approx(g["survey_A6"]["prob"], rel=1e-7)
    assert [s(l) for l, _ in prob] == g["survey_A6"]["beam"]


@pytest.mark.parametrize("T,V,seed", [(1, 4, 0), (2, 3, 1), (4, 4, 2), (6, 3, 3), (6, 4, 4), (5, 5, 5)])
def test_exhaustive_enumeration(T, V, seed):
    """With a beam wider than the state space the decoder is exact."""
    rng = np.random.default_rng(seed)
    e = rng.random((T, V)).astype(np.float32) + 0.05
    e /= e.sum(1, keepdims=True)
    exact = brute_force(e.astype(np.float64), blank=0)
    got = oracle.decode(e.reshape(T, 1, V), beam=10 ** 6, blank=0, max_hyps=10 ** 4)[0]
    assert len(got) == len(exact)
    for lab, lp in got:
        assert lp == pytest.approx(exact[tuple(lab)], abs=1e-9)


@pytest.mark.parametrize("blank", [0, 2])
def test_exhaustive_nonzero_blank(blank):
    rng = np.random.default_rng(11)
    T, V = 5, 4
    e = rng.dirichlet(np.ones(V), size=T).astype(np.float32)
    exact = brute_force(e.astype(np.float64), blank=blank)
    got = oracle.decode(e.reshape(T, 1, V), beam=10 ** 6, blank=blank, max_hyps=10 ** 4)[0]
    assert {tuple(l): lp for l, lp in got} == pytest.approx(exact, abs=1e-9)


@pytest.mark.parametrize("T,V,beam,seed", [(12, 5, 3, 0), (20, 29, 10, 1), (30, 8, 6, 2)])
def test_log_domain_matches_prob_domain(T, V, beam, seed):
    """The log-domain restatement ranks like the reference's fp32 products."""
    emis = oracle.synthetic_emissions(T, 3, V, seed0=100 + seed, sigma=2.0)
    lg = oracle.decode(emis, beam, 0)
    pr = oracle.decode(emis, beam, 0, prob_domain=True)
    for a, b in zip(lg, pr):
        assert [l for l, _ in a] == [l for l, _ in b]
        for (_, x), (_, p) in zip(a, b):
            assert math.exp(x) == pytest.approx(p, rel=2e-4)


def test_prune_keeps_ties():
    """F2/F1: all states tied at the cutoff survive (uniform emissions)."""
    T, V, beam = 3, 3, 2
    emis = np.full((T, 1, V), 1.0 / V, np.float32)
    got = oracle.decode(emis, beam, 0)[0]
    assert len(got) >= beam + 1
    lg = oracle.decode(emis, 100, 0)[0]   # unpruned
    assert len(lg) >= len(got)


def test_beam_at_least_vocab():
    """beam >= V: the literal reference threw at t=0 (cpp:107); F2 keeps all."""
    emis = oracle.synthetic_emissions(5, 2, 4)
    got = oracle.decode(emis, beam=500, blank=0)
    exact = [brute_force(emis[:, b, :].astype(np.float64), 0) for b in range(2)]
    for g, ex in zip(got, exact):
        assert {tuple(l): lp for l, lp in g} == pytest.approx(ex, abs=1e-9)


def test_zero_probabilities():
    """Exact zeros give -inf scores that still count as states (prob 0)."""
    emis = oracle.synthetic_emissions(6, 2, 5)
    emis[2, :, 3] = 0.0
    emis[:, 1, 1] = 0.0
    got = oracle.decode(emis, beam=3, blank=0)
    assert all(len(g) >= 1 for g in got)


def test_synthetic_shard_invariance():
    full = oracle.synthetic_emissions(5, 6, 7)
    part = oracle.synthetic_emissions(5, 3, 7, first=3)
    assert np.array_equal(full[:, 3:, :], part)


def test_threads_deterministic():
    emis = oracle.synthetic_emissions(40, 8, 29)
    a = oracle.decode(emis, 10, 0, nthreads=1)
    b = oracle.decode(emis, 10, 0, nthreads=4)
    assert a == b


def test_oracle_under_sanitizers():
    """ASan + UBSan build of the CPU restatement over its edge cases (SURVEY
    §5 'Race detection'; oracle/sanitize_main.cpp).  Host code only."""
    import subprocess
    odir = ROOT / "oracle"
    subprocess.run(["make", "-s", "-C", str(odir), "sanitize"], check=True)
    r = subprocess.run([str(odir / "ctc_oracle_sanitize")], capture_output=True, text=True,
                       timeout=300, env={**__import__("os").environ, "ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle sanitizer run: ok" in r.stdout


def test_oracle_timesteps_properties():
    """The oracle's timesteps (ctcdecode's output, the build's definition):
    one per label, strictly increasing frames < T, the same beams as the
    plain decode, and a label's frame never later than where a hypothesis
    sharing that prefix appended it (prefixes share frames)."""
    T, B, V, beam = 40, 3, 7, 8
    emis = oracle.synthetic_emissions(T, B, V, seed0=12)
    ts = oracle.decode_ts(emis, beam, 0, nthreads=2)
    plain = oracle.decode(emis, beam, 0, nthreads=2)
    for u_ts, u in zip(ts, plain):
        assert [(l, s) for l, s, _ in u_ts] == u
        for lab, _, fr in u_ts:
            assert len(fr) == len(lab)
            assert all(0 <= a < b < T for a, b in zip(fr, fr[1:]))
    # T = 1: every hypothesis is one label appended at frame 0
    one = oracle.decode_ts(emis[:1], beam, 0)
    assert all(fr == [0] * len(lab) for u in one for lab, _, fr in u)


def test_c5_production_fixture_consistent():
    """tests/golden/c5_production.json (the oracle's decode of the first T
    frames of four C5 production-emission utterances, checked against the
    wide kernel by test_full_configs_gpu.py) is self-consistent: a full beam
    (beam + ties) per utterance, ranked by log-probability, the best
    hypothesis first, labels inside the vocabulary with no blank, at most one
    label per frame."""
    p = GOLDEN / "c5_production.json"
    if not p.exists():
        pytest.skip("fixture not generated")
    g = json.loads(p.read_text())
    assert g["T"] <= g["T_production"] and g["V"] == 1000 and g["beam"] == 200
    n = len(g["utterances"])
    assert len(g["emis_sha256"]) == len(g["best_labels"]) == len(g["beam_logp"]) == len(g["n_hyps"]) == n
    for i in range(n):
        lp = g["beam_logp"][i]
        assert len(lp) == g["n_hyps"][i] >= g["beam"]
        assert all(a >= b for a, b in zip(lp, lp[1:]))
        assert lp[0] == g["best_logp"][i] and math.isfinite(lp[0])
        lab = g["best_labels"][i]
        assert 0 < len(lab) <= g["T"]
        assert all(0 < c < g["V"] for c in lab)   # blank 0 never emitted

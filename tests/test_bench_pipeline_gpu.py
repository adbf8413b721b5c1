"""bench.py's pipelines decode the same hypotheses: D batches in flight on
disjoint CU groups (8-wave decode workgroups one per CU, or 4-wave ones two
to a CU), the production split over two streams, HIP-graph
production replays and the sequential loop all gather the same digest
(labels + fp64 log-probs of every utterance) — the scheduling changes when
work runs, never what it computes.  Each bench run is one subprocess (a few
seconds at T = 100), run one after another."""
import json
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(*args, config="C2", env=None):
    import os
    cmd = [sys.executable, str(ROOT / "bench.py"), "--no-cpu-baseline", "--steps", "6", "--warmup", "2",
           "--T", "100", "--config", config, *args]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                         env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    return line


def test_inflight_and_split_production_match_sequential():
    """The CU-group schedules (ASR_PIPELINE_MODE=0 keeps C2's 64-utterance
    batches on them) against the sequential loop: the same unfused production
    (recurrence, then the emission GEMM), the same bits."""
    groups = {"ASR_PIPELINE_MODE": "0"}
    seq = _bench("--no-pipeline")
    one = ("--coalesce", "1")   # 64-utterance batches (no dynamic batching)
    runs = {
        "packed": _bench("--packed", *one),   # 4-wave decode workgroups two to a CU, 5 batches in flight
        "d1": _bench("--inflight", "1", *one, env=groups),
        "d3_split_all": _bench("--inflight", "3", *one, env=groups),   # auto: production split, GEMMs on all CUs
        "d2_unsplit_graph": _bench("--inflight", "2", "--prod-split", "off", "--graph-production", "on",
                                   "--prod-streams", "2", *one),
    }
    assert seq["gather"]["utterances"] == 64
    for name, r in runs.items():
        assert r["gather"] == seq["gather"], name
    assert runs["d3_split_all"]["config"]["inflight_decodes"] == 3
    assert runs["packed"]["config"]["decode_waves"] == 4 and runs["packed"]["config"]["inflight_decodes"] == 5
    assert runs["d2_unsplit_graph"]["config"]["production_streams"] == 2


def test_c2_chip_filling_schedule_independent():
    """C2's default native schedule (64-utterance batches on the chip-filling
    schedule: one-wave decodes, 10 in flight, fused production) gathers the
    same digest at 1, 3 and the default decodes in flight and with the
    production in one T-segment — placement and overlap never change a bit."""
    base = _bench("--coalesce", "1")
    assert base["config"]["inflight_decodes"] == 10 and base["config"]["decode_waves"] == -1, base["config"]
    assert base["config"]["fused_emission"] is True
    for args in (("--inflight", "1"), ("--inflight", "3"), ("--segments", "1")):
        r = _bench(*args, "--coalesce", "1")
        assert r["gather"] == base["gather"], args
    # the default: dynamic batching (ten 64-utterance submits per launch), the same bits
    co = _bench()
    assert co["config"]["coalesce"] == 10, co["config"]
    assert co["gather"] == base["gather"]


def test_c4_self_launched_ranks_match_one_rank():
    """The driver's multi-GPU form, `bench.py --gpus 2` with no rank
    variables: two rank processes (sharing this box's one GPU: ranks wrap)
    shard C4's 2048 utterances; rank 0 gathers and re-decodes every shard on
    its own device (verified_vs_1gpu), and the digest equals one rank's."""
    one = _bench(config="C4")
    two = _bench("--gpus", "2", config="C4")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["gather"]["utterances"] == two["gather"]["utterances"] == 2048
    assert two["gather"]["verified_vs_1gpu"] is True
    assert two["gather"]["digest"] == one["gather"]["digest"]
    assert two["scaling"] == "strong" and two["config"]["batch_per_gpu"] == 1024

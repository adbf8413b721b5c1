"""Writes tests/golden/full_configs.json: CPU-oracle decodes of utterance
subsets of the BASELINE configs at full length, used by
tests/test_full_configs_gpu.py (the GPU box does not have time to run the
std::set/std::map restatement over 1000-frame utterances at beam 100, or
V=1000 at beam 200, inside a test).

Inputs are the same synthetic emissions the tests generate
(oracle.synthetic_emissions, softmax of N(0, 3^2) logits, one generator per
global utterance index), so a subset decoded here equals those
rows of the full batch decoded on the GPU.

    python tests/golden/make_full_config_golden.py [--threads N]
"""
import argparse
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from __graft_entry__ import _load  # noqa: E402

oracle = _load("ctc_oracle", ROOT / "oracle" / "ctc_oracle.py")

# name: (T, B of the full batch, V, beam, utterance ids checked)
CASES = {
    "C3": (1000, 256, 29, 100, list(range(0, 256, 16))),          # BASELINE configs[2]
    "C5_decode": (200, 32, 1000, 200, [0, 31]),                    # configs[4]: V, beam; T prefix
}


def labels_digest(beam):
    """sha256 over the ranked final beam's label sequences (ids, in rank order)."""
    m = hashlib.sha256()
    for lab, _ in beam:
        m.update(np.asarray(lab, np.int32).tobytes())
        m.update(b"|")
    return m.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    out_path = Path(__file__).resolve().parent / "full_configs.json"
    out = json.loads(out_path.read_text()) if out_path.exists() else {}
    for name, (T, B, V, beam, uids) in CASES.items():
        if args.only and name != args.only:
            continue
        emis = np.concatenate([oracle.synthetic_emissions(T, 1, V, first=u) for u in uids], axis=1)
        t0 = time.time()
        ref = oracle.decode(emis, beam, 0, nthreads=args.threads, max_hyps=1024)
        secs = time.time() - t0
        out[name] = {
            "T": T, "B": B, "V": V, "beam": beam, "sigma": 3.0, "seed0": oracle.SEED0,
            "utterances": uids, "oracle_seconds": round(secs, 1),
            "best_labels": [[int(c) for c in r[0][0]] for r in ref],
            "best_logp": [r[0][1] for r in ref],
            "n_hyps": [len(r) for r in ref],
            "beam_labels_sha256": [labels_digest(r) for r in ref],
            "beam_logp": [[lp for _, lp in r] for r in ref],
        }
        print(name, f"{secs:.1f} s", flush=True)
        out_path.write_text(json.dumps(out, separators=(",", ":")))


if __name__ == "__main__":
    main()

"""Writes tests/golden/c5_production.json: CPU-oracle decodes of C5
PRODUCTION emissions (V = 1000, beam = 200) over their first T frames, the
large-vocabulary kernel's long parity case.

The oracle is the std::set / std::map restatement of CTCBeamSearch.cpp, and
on these emissions every frame appends a label (the best prefix is ~T labels
long), so its string work grows ~T^1.75: measured here 200 s for T = 100 and
674 s for T = 200 per utterance, ~3 h at T = 1000 and ~10 h at T = 2000.  The
fixture is therefore T = 1000 (half of C5's 2000, 40x the 24-frame prefix
checked before): `--T` sets it.

The emissions are the bench's C5 model (bench.make_weights /
make_features, H = in = 1024, V = 1000, 32 utterances, T = 2000) run through
the library's fp32 dense arithmetic on the GPU: tools/dump_c5_emissions.py
writes utterances 0, 9, 18, 27 ([T][4][V] float32) and their sha256.  This
script decodes them here with oracle/ctc_oracle.cpp (one thread per
utterance; ~3 h at T = 1000) and records the result with the emission digests;
tests/test_full_configs_gpu.py regenerates the emissions on the GPU, checks
the digests (the fixture belongs to those exact bytes) and compares the
wide kernel, whole and in two T-segments, against it.  The emissions
themselves (32 MB) are not committed.

    python tools/dump_c5_emissions.py gpurun_out/c5fix        # on the GPU box
    python tests/golden/make_c5_production_golden.py gpurun_out/c5fix [--T 1000]
"""
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


def labels_digest(beam):
    """sha256 over the ranked final beam's label sequences (ids, in rank order)."""
    m = hashlib.sha256()
    for lab, _ in beam:
        m.update(np.asarray(lab, np.int32).tobytes())
        m.update(b"|")
    return m.hexdigest()


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default="gpurun_out/c5fix")
    ap.add_argument("--T", type=int, default=1000)
    args = ap.parse_args()
    src = Path(args.src)
    meta = json.loads((src / "c5_emis.json").read_text())
    emis = np.load(src / "c5_emis.npy")
    Tfull, V, beam = meta["T"], meta["V"], meta["beam"]
    assert emis.shape == (Tfull, len(meta["utterances"]), V), emis.shape
    for j, d in enumerate(meta["sha256"]):
        assert hashlib.sha256(np.ascontiguousarray(emis[:, j, :]).tobytes()).hexdigest() == d
    T = min(args.T, Tfull)
    emis = np.ascontiguousarray(emis[:T])
    t0 = time.time()
    ref = oracle.decode(emis, beam, 0, is_log=True, nthreads=emis.shape[1], max_hyps=1024)
    secs = time.time() - t0
    out = {
        "source": "tools/dump_c5_emissions.py: bench C5 model, ASR_DENSE_F32, log_softmax emissions",
        "T": T, "T_production": Tfull, "B": meta["B"], "H": meta["H"], "V": V, "beam": beam,
        "utterances": meta["utterances"], "emis_sha256": meta["sha256"],
        "oracle_seconds": round(secs, 1),
        "best_labels": [[int(c) for c in r[0][0]] for r in ref],
        "best_logp": [r[0][1] for r in ref],
        "n_hyps": [len(r) for r in ref],
        "beam_labels_sha256": [labels_digest(r) for r in ref],
        "beam_logp": [[lp for _, lp in r] for r in ref],
    }
    (Path(__file__).resolve().parent / "c5_production.json").write_text(json.dumps(out, separators=(",", ":")))
    print(f"c5_production: {secs:.1f} s, best lengths {[len(r[0][0]) for r in ref]}", flush=True)


if __name__ == "__main__":
    main()

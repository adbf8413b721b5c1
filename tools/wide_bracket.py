"""Parity bracket of the large-vocabulary kernel over V and T (diagnostic)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import asr, oracle  # noqa: E402


def same(got, ref):
    for g, r in zip(got, ref):
        if [list(l) for l, _ in g] != [list(map(int, l)) for l, _ in r]:
            return False
        for (_, x), (_, y) in zip(g, r):
            if abs(x - y) > 1e-9 * max(1.0, abs(y)):
                return False
    return True


asr.set_device(0)
beam = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for V in [1001, 1500, 2048, 2049, 3000, 4000, 4095, 4096]:
    res = []
    for T in [1, 2, 3, 4, 6, 8]:
        emis = oracle.synthetic_emissions(T, 2, V, seed0=3000 + 8 + V + beam)
        ref = oracle.decode(emis, beam, 0, nthreads=16)
        dec = asr.CTCDecoder(V, beam, 0)
        dec.decode(emis)
        got = dec.beams(max_hyps=dec.config()[0])
        dec.close()
        res.append(f"T{T}:{'ok' if same(got, ref) else 'BAD'}")
    print(V, beam, " ".join(res), flush=True)

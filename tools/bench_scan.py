"""Summarise a round's bench lines (gpurun_out/<run>/*.json) into a markdown
table: python tools/bench_scan.py profiles/r05/bench_scan.md run:note ..."""
import glob
import json
import os
import sys


def main():
    out_path = sys.argv[1]
    notes = dict(a.split(":", 1) for a in sys.argv[2:])
    rows = []
    for d in notes:
        for f in sorted(glob.glob(f"gpurun_out/{d}/*.json")):
            try:
                j = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
            except Exception:
                continue
            if "value" not in j:
                continue
            c = j.get("config", {})
            clk = (j.get("clock") or {}).get("gfxclk_mhz", {}).get("mean")
            rows.append((d, os.path.basename(f)[:-5], c.get("workload", "")[:2], c.get("batch_per_gpu"),
                         j["value"] / 1e6, (j.get("parity") or {}).get("match"), c.get("inflight_decodes"),
                         c.get("production_streams"), c.get("segments"), c.get("hw_queues"), clk))
    out = ["# Round bench lines (builder, one MI355X per line, 20 timed steps / 5 warmup unless named)", "",
           "Every line is `bench.py` output of the tree at that point (`gpurun_out/<run>/`, run with "
           "`tools/bench_matrix.sh`).",
           "frames/s is the whole job's, per GPU; N > 1 rows are one GPU running one rank's shard of C4's 2048 "
           "utterances.", "", "| run | what the run tested |", "|---|---|"]
    out += [f"| {k} | {v} |" for k, v in notes.items()]
    out += ["", "| run | line | config | utts/GPU | M frames/s | parity | D | P | segments | queues | gfx MHz |",
            "|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append("| %s | %s | %s | %s | %.1f | %s | %s | %s | %s | %s | %s |" % (
            r[0], r[1], r[2], r[3], r[4], "yes" if r[5] else "", r[6], r[7], r[8], r[9],
            "%.0f" % r[10] if r[10] else ""))
    open(out_path, "w").write("\n".join(out) + "\n")
    print(len(rows), "lines")


if __name__ == "__main__":
    main()

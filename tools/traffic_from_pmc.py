"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into
profiles/<round>/traffic.json: HBM bytes per launch of each kernel variant
(the full template instance, e.g. ctc_beam_kernel<4,8,1,false>), keyed by the
bench workload the passes ran.  bench.py embeds the entry of the workload and
decoder variant it actually ran as roofline.traffic, with its source label.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md:
FETCH_SIZE reads exactly half the bytes of 16-B/lane coalesced streaming
reads; the decoder's emission loads are 4-B/lane global_load_dword, for
which the counter is not halved (checked: 4055 KiB vs 3.71 MB of emission
rows per C2 launch), so no correction is applied to the decoder.

    python tools/traffic_from_pmc.py FETCH.csv WRITE.csv WORKLOAD [source-label] [round]
"""
import csv
import json
import sys
from pathlib import Path


def per_kernel(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("asr::", "").replace(" ", "")
        agg.setdefault(short, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fetch, write = per_kernel(sys.argv[1]), per_kernel(sys.argv[2])
    workload = sys.argv[3]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    rnd = sys.argv[5] if len(sys.argv) > 5 else "r03"
    p = Path(__file__).resolve().parents[1] / "profiles" / rnd / "traffic.json"
    p.parent.mkdir(parents=True, exist_ok=True)
    allw = json.loads(p.read_text()) if p.exists() else {}
    out = {}
    for k in sorted(set(fetch) & set(write)):
        out[k] = {"fetch_kib": round(fetch[k], 1), "write_kib": round(write[k], 1),
                  "hbm_bytes_per_launch": int((fetch[k] + write[k]) * 1024), "source": label}
    allw[workload] = out
    p.write_text(json.dumps(allw, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Summarise a rocprofv3 SQ counter pass over bench.py into
profiles/<round>/issue.json[workload][variant]: the decoder kernel's
instruction-issue roofline per kernel variant (full template instance),
which bench.py embeds as roofline.issue when it ran that workload and
variant.

Counters (one pass, 8 SQ slots): SQ_WAVES, SQ_INSTS_VALU, SQ_INSTS_SALU,
SQ_INSTS_LDS, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
SQ_ACTIVE_INST_ANY.  Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles); WAIT_ANY +
WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES.

Derived, per launch (every wave alive for the whole kernel; --cus: the CUs
the decode ran on, default one workgroup per CU = B CUs — the one-wave
kernel packs 16 utterances per CU, so pass the decode partition):
  kernel_cycles  = 4 * WAVE_CYCLES / WAVES   (a wave's lifetime in cycles)
  per wave-frame = INSTS_x / WAVES / T
  active_frac    = ACTIVE_INST_ANY / WAVE_CYCLES  (cycles a wave issues)
  wait_frac      = WAIT_ANY / WAVE_CYCLES         (parked: s_waitcnt / barrier)
  stall_frac     = WAIT_INST_ANY / WAVE_CYCLES    (issue-stalled)
  salu_util      = SALU per CU / kernel_cycles: against the CU's one scalar
                   unit (one SALU issue per cycle)
  valu_util      = 2 * VALU per SIMD / kernel_cycles: a wave64 VALU op holds
                   a SIMD-32 for >= 2 cycles (fp64 and transcendental ops more)
  lds_util       = 2 * LDS per CU / kernel_cycles: >= 2 LDS-array cycles per
                   wave instruction (MI355X_MICROARCH.md §LDS)

    python tools/issue_from_pmc.py SQ.csv --kernel ctc_beam_kernel --T 500 --B 64 \
        --workload C2 [--source label] [--round r03]
"""
import argparse
import csv
import json
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="ctc_beam_kernel")
    ap.add_argument("--T", type=int, required=True)
    ap.add_argument("--B", type=int, required=True)
    ap.add_argument("--workload", default="C2")
    ap.add_argument("--source", default="")
    ap.add_argument("--round", default="r04")
    ap.add_argument("--cus", type=int, default=0, help="CUs the decode ran on (default: B)")
    args = ap.parse_args()
    per = {}   # dispatch -> counter -> value
    variants = set()
    for r in csv.DictReader(open(args.csv)):
        if args.kernel not in r["Kernel_Name"]:
            continue
        variants.add(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("asr::", "").replace(" ", ""))
        per.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    if len(variants) != 1:
        raise SystemExit(f"expected one variant of {args.kernel}, found {sorted(variants)}")
    variant = variants.pop()
    cus = args.cus or args.B
    if not per:
        raise SystemExit(f"no {args.kernel} dispatches in {args.csv}")
    keys = sorted({k for d in per.values() for k in d})
    avg = {k: sum(d.get(k, 0.0) for d in per.values()) / len(per) for k in keys}
    waves = avg["SQ_WAVES"]
    nw = waves / args.B
    cyc = 4.0 * avg["SQ_WAVE_CYCLES"] / waves
    wf = waves * args.T
    issue = {
        "dispatches": len(per),
        "waves_per_workgroup": round(nw, 2),
        "kernel_cycles": round(cyc),
        "cycles_per_frame": round(cyc / args.T, 1),
        "valu_per_wave_frame": round(avg["SQ_INSTS_VALU"] / wf, 1),
        "salu_per_wave_frame": round(avg["SQ_INSTS_SALU"] / wf, 1),
        "lds_per_wave_frame": round(avg["SQ_INSTS_LDS"] / wf, 1),
        "active_frac": round(avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"], 4),
        "wait_frac": round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 4),
        "stall_frac": round(avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"], 4),
        "cus": cus,
        "salu_util": round(avg["SQ_INSTS_SALU"] / cus / cyc, 4),
        "valu_util": round(2.0 * avg["SQ_INSTS_VALU"] / (4 * cus) / cyc, 4),
        "lds_util": round(2.0 * avg["SQ_INSTS_LDS"] / cus / cyc, 4),
    }
    out = {"T": args.T, "B": args.B,
           "counters_avg_per_launch": {k: round(v) for k, v in avg.items()},
           "issue": issue, "source": args.source}
    p = Path(__file__).resolve().parents[1] / "profiles" / args.round / "issue.json"
    p.parent.mkdir(parents=True, exist_ok=True)
    allw = json.loads(p.read_text()) if p.exists() else {}
    allw.setdefault(args.workload, {}).setdefault(variant, {}).update(out)   # keeps a valu_mix entry
    p.write_text(json.dumps(allw, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Fold the decoder's wait / issue counter passes (tools/profile_bench.sh
passes `wait` and `issue`) into profiles/<round>/issue.json
[workload][variant]["waits"]: where a wave's non-issuing cycles go.

Per wave-frame (counters / WAVES / T; SQ_* cycle counters count
quad-cycles, x4 = shader cycles):
  wave_qc            SQ_WAVE_CYCLES (a wave's lifetime)
  active_qc          SQ_ACTIVE_INST_ANY (sq pass): issuing
  wait_qc            SQ_WAIT_ANY (sq pass): parked on s_waitcnt / barrier
  stall_qc           SQ_WAIT_INST_ANY (sq pass): ready but not issued
  active split       SQ_ACTIVE_INST_{VALU,SCA,LDS,MISC} (issue pass)
  wait_inst_lds_qc   SQ_WAIT_INST_LDS: waiting to issue an LDS instruction
  vmem_rd/wr cycles  SQ_INST_CYCLES_VMEM_{RD,WR}; smem: SQ_INSTS_SMEM,
                     SQ_INST_CYCLES_SMEM; SQ_LDS_BANK_CONFLICT (cycles)
  ifetch             SQ_IFETCH (instruction fetches)

    python tools/wait_from_pmc.py WAIT.csv ISSUE.csv SQ.csv --kernel ctc_wave_kernel --T 500 --B 1024 \
        --workload C4 --source label --round r05
"""
import argparse
import collections
import csv
import json
from pathlib import Path


def load(path, kernel):
    per = collections.defaultdict(dict)
    name = None
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("asr::", "").replace(" ", "")
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    avg = {k: sum(c[k] for c in per.values()) / len(per) for k in next(iter(per.values()))}
    return name, len(per), avg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("wait")
    ap.add_argument("issue")
    ap.add_argument("sq")
    ap.add_argument("--kernel", default="ctc_wave_kernel")
    ap.add_argument("--T", type=int, required=True)
    ap.add_argument("--B", type=int, required=True)
    ap.add_argument("--workload", default="C4")
    ap.add_argument("--source", default="")
    ap.add_argument("--round", default="r05")
    args = ap.parse_args()
    name, n, w = load(args.wait, args.kernel)
    _, _, i = load(args.issue, args.kernel)
    _, _, q = load(args.sq, args.kernel)
    wf = float(args.B * args.T)
    f = lambda x: round(x / wf, 1)  # noqa: E731
    out = {"dispatches": n, "per_wave_frame": {
        "wave_qc": f(w["SQ_WAVE_CYCLES"]), "active_qc": f(q["SQ_ACTIVE_INST_ANY"]),
        "wait_qc": f(q["SQ_WAIT_ANY"]), "stall_qc": f(q["SQ_WAIT_INST_ANY"]),
        "active_valu_qc": f(i["SQ_ACTIVE_INST_VALU"]), "active_salu_qc": f(i["SQ_ACTIVE_INST_SCA"]),
        "active_lds_qc": f(i["SQ_ACTIVE_INST_LDS"]), "active_misc_qc": f(i["SQ_ACTIVE_INST_MISC"]),
        "branches": f(i["SQ_INSTS_BRANCH"]), "lds_insts": f(i["SQ_INSTS_LDS"]),
        "wait_inst_lds_qc": f(w["SQ_WAIT_INST_LDS"]), "vmem_rd_cycles": f(w["SQ_INST_CYCLES_VMEM_RD"]),
        "vmem_wr_cycles": f(w["SQ_INST_CYCLES_VMEM_WR"]), "smem_insts": f(w["SQ_INSTS_SMEM"]),
        "smem_cycles": f(w["SQ_INST_CYCLES_SMEM"]), "lds_bank_conflict_cycles": f(w["SQ_LDS_BANK_CONFLICT"]),
        "ifetch": f(i["SQ_IFETCH"])},
        "reading": "wait_qc is the s_waitcnt / barrier time: with SMEM and VMEM a few cycles per frame and "
                   "LDS-issue waits ~2 %, it is the latency of dependent LDS round trips (the one-wave kernel "
                   "has no barrier); stall_qc is issue arbitration between the CU's waves",
        "source": args.source}
    root = Path(__file__).resolve().parents[1] / "profiles" / args.round
    p = root / "issue.json"
    alli = json.loads(p.read_text()) if p.exists() else {}
    alli.setdefault(args.workload, {}).setdefault(name, {})["waits"] = out
    p.write_text(json.dumps(alli, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

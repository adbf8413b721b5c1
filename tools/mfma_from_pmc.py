"""Summarise rocprofv3 --pmc passes over bench.py (tools/profile_bench.sh
passes `mfma` and `valu`) into profiles/<round>/mfma.json and the decoder's
VALU mix into profiles/<round>/issue.json [workload][variant]["valu_mix"].

mfma pass counters: SQ_VALU_MFMA_BUSY_CYCLES (cycles, 32 per
v_mfma_f32_16x16x4_f32 and 16 per v_mfma_f32_16x16x32_bf16 per SIMD),
SQ_INSTS_VALU_MFMA_{F32,BF16}, SQ_INSTS_VALU_MFMA_MOPS_{F32,BF16} (one MOP =
512 flop), SQ_BUSY_CYCLES, SQ_WAVES, SQ_ACTIVE_INST_ANY,
GRBM_GUI_ACTIVE (summed over the 8 XCDs: / 8 = the dispatch's wall clock
cycles), GRBM_COUNT.  Counter passes serialise dispatches, so each one ran
alone on its stream's CUs.  Per kernel (dispatches grouped by MFMA count, so
the bench's full-size standalone GEMM and its pipeline slices are apart):
  wall_cycles   = GRBM_GUI_ACTIVE / 8
  mfma_busy     = MFMA_BUSY_CYCLES / (4 SIMDs x cus x wall_cycles)
  flop          = 512 x MFMA_MOPS_F32 (one MOP = 512 flop); for the split-bf16
                  kernels (bf16 MFMAs, 6 products per fp32 product) gflop is the
                  fp32-equivalent 512 x MOPS_BF16 / 6, bf16_gflop the matrix-core work
  clock_ghz     = wall_cycles / dispatch duration
valu pass counters (decoder): SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU,
SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, SQ_ACTIVE_INST_SCA, SQ_WAVE_CYCLES.

    python tools/mfma_from_pmc.py --mfma M.csv --valu V.csv --workload C4 \
        --cus gemm_wide_kernel=256 --cus rnn_recur_mfma_kernel=128 --T 1000 --B 2048 \
        --decoder ctc_wave_kernel --decoder-cus 128 --source label --round r04
"""
import argparse
import collections
import csv
import json
from pathlib import Path


def variant(name):
    return name.split("(")[0].replace("void ", "").replace("asr::", "").replace(" ", "")


def load(path):
    per = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (variant(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return per, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mfma", required=True)
    ap.add_argument("--valu", required=True)
    ap.add_argument("--workload", default="C4")
    ap.add_argument("--cus", action="append", default=[], help="kernel=CUs it ran on (its stream's CU mask)")
    ap.add_argument("--slice-cus", type=int, default=0,
                    help="CUs of a kernel's smaller dispatch groups (the pipeline's CU-masked slices of a "
                         "GEMM whose full-size standalone run has the most MFMAs)")
    ap.add_argument("--slice", action="append", default=[],
                    help="kernel=CUs of that kernel's smaller dispatch groups (overrides --slice-cus)")
    ap.add_argument("--wpw", action="append", default=[],
                    help="kernel=waves per workgroup: a dispatch group's busy CUs are then "
                         "min(its mask's CUs, SQ_WAVES / wpw), the kernels running one workgroup per CU "
                         "(default 8 for gemm_x3_kernel / rnn_recur_x3_kernel / rnn_recur_mfma_kernel)")
    ap.add_argument("--T", type=int, required=True)
    ap.add_argument("--B", type=int, required=True)
    ap.add_argument("--decoder", default="ctc_wave_kernel")
    ap.add_argument("--decoder-cus", type=int, required=True)
    ap.add_argument("--source", default="")
    ap.add_argument("--round", default="r04")
    args = ap.parse_args()
    cus = dict(x.split("=") for x in args.cus)
    wpw = {"gemm_x3_kernel": 8, "rnn_recur_x3_kernel": 8, "rnn_recur_mfma_kernel": 8}
    wpw.update({k: int(v) for k, v in (x.split("=") for x in args.wpw)})
    per, meta = load(args.mfma)
    groups = collections.defaultdict(list)
    for d, c in per.items():
        name, secs = meta[d]
        n = c.get("SQ_INSTS_VALU_MFMA_F32", 0) + c.get("SQ_INSTS_VALU_MFMA_BF16", 0)
        if n <= 0:
            continue
        groups[(name, round(n))].append((c, secs))
    out = {}
    biggest = {}
    for (name, nmfma) in groups:
        biggest[name] = max(biggest.get(name, 0), nmfma)
    for (name, nmfma), lst in sorted(groups.items()):
        ncu = next((int(v) for k, v in cus.items() if k in name), 256)
        if nmfma < biggest[name]:
            sl = next((int(v) for k, v in (x.split("=") for x in args.slice) if k in name), args.slice_cus)
            ncu = sl or ncu
        avg = {k: sum(c[k] for c, _ in lst) / len(lst) for k in lst[0][0]}
        secs = sum(s for _, s in lst) / len(lst)
        # one workgroup per CU: the group's own workgroup count bounds its busy CUs
        # (a 1024-utterance recurrence is 64 workgroups on a 128-CU mask)
        cus_src = "CU mask"
        w = next((v for k, v in wpw.items() if k in name), None)
        if w and avg.get("SQ_WAVES"):
            nwg = int(round(avg["SQ_WAVES"] / w))
            if nwg < ncu:
                ncu, cus_src = nwg, f"SQ_WAVES / {w} waves per workgroup"
        wall = avg["GRBM_GUI_ACTIVE"] / 8.0
        bf16 = 512.0 * avg.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) / 1e9
        rec = {"dispatches": len(lst), "cus": ncu, "cus_source": cus_src, "mfma_f32_insts": round(avg["SQ_INSTS_VALU_MFMA_F32"]),
               "mfma_bf16_insts": round(avg.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)),
               "gflop": round(512.0 * avg["SQ_INSTS_VALU_MFMA_MOPS_F32"] / 1e9 + bf16 / 6.0, 2),
               "bf16_gflop": round(bf16, 2),
               "mfma_busy_cycles": round(avg["SQ_VALU_MFMA_BUSY_CYCLES"]),
               "wall_cycles": round(wall), "duration_ms": round(1e3 * secs, 4),
               "clock_ghz": round(wall / secs / 1e9, 3) if secs > 0 else None,
               "mfma_busy": round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (4.0 * ncu * wall), 4),
               "counters_avg": {k: round(v) for k, v in avg.items()}}
        out.setdefault(name, []).append(rec)
    root = Path(__file__).resolve().parents[1] / "profiles" / args.round
    root.mkdir(parents=True, exist_ok=True)
    p = root / "mfma.json"
    allw = json.loads(p.read_text()) if p.exists() else {}
    allw[args.workload] = {"kernels": out, "source": args.source,
                           "note": "rocprofv3 --pmc (dispatches serialised); mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES "
                                   "/ (4 SIMDs x CUs x GRBM_GUI_ACTIVE/8)"}
    p.write_text(json.dumps(allw, indent=1))
    # decoder VALU mix
    vper, vmeta = load(args.valu)
    dec = [(c, vmeta[d][1]) for d, c in vper.items() if args.decoder in vmeta[d][0]]
    vname = next(vmeta[d][0] for d in vper if args.decoder in vmeta[d][0])
    avg = {k: sum(c[k] for c, _ in dec) / len(dec) for k in dec[0][0]}
    wf = args.B * args.T
    f64 = sum(avg[k] for k in avg if k.endswith("_F64"))
    mix = {"dispatches": len(dec), "valu_per_wave_frame": round(avg["SQ_INSTS_VALU"] / wf, 1),
           "f64_valu_per_wave_frame": round(f64 / wf, 1), "f64_share": round(f64 / avg["SQ_INSTS_VALU"], 4),
           "f64_breakdown_per_wave_frame": {k.replace("SQ_INSTS_VALU_", ""): round(avg[k] / wf, 1)
                                            for k in avg if k.endswith("_F64")},
           "active_valu_per_valu": round(avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_INSTS_VALU"], 3),
           "sca_active_per_wave_frame": round(avg["SQ_ACTIVE_INST_SCA"] / wf, 1),
           "counters_avg": {k: round(v) for k, v in avg.items()}, "source": args.source}
    # the mfma pass also holds the decoder's wall clock and SQ busy (its dispatches have no MFMA)
    mdec = [c for d, c in per.items() if args.decoder in meta[d][0]]
    if mdec:
        g = sum(c["GRBM_GUI_ACTIVE"] for c in mdec) / len(mdec) / 8.0
        wc = 4.0 * avg["SQ_WAVE_CYCLES"] / (args.B)   # a wave's average lifetime (cycles)
        mix["wall_cycles"] = round(g)
        mix["wave_lifetime_over_wall"] = round(wc / g, 4)
        mix["sq_busy_over_wall"] = round(sum(c["SQ_BUSY_CYCLES"] for c in mdec) / len(mdec) / 32.0 / g, 4)
        # VALU demand per SIMD per frame against the wall: 2 or 4 cycles per wave64 VALU op
        per_simd = avg["SQ_INSTS_VALU"] / (4.0 * args.decoder_cus)
        mix["valu_busy_at_2cyc"] = round(2 * per_simd / g, 4)
        mix["valu_busy_at_4cyc"] = round(4 * per_simd / g, 4)
    ip = root / "issue.json"
    alli = json.loads(ip.read_text()) if ip.exists() else {}
    alli.setdefault(args.workload, {}).setdefault(vname, {})["valu_mix"] = mix
    ip.write_text(json.dumps(alli, indent=1))
    print(json.dumps({"mfma": out, "valu_mix": mix}, indent=1)[:4000])


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 SQ counter passes of single conv shapes (tools/conv_bench.py --shape)
into per-dispatch averages and the derived figures DESIGN.md §2.9 / §2.13 quote.

    python tools/sq_shapes.py OUT.json NAME=DIR_A,DIR_B [NAME=DIR_A,DIR_B ...]

Each DIR is a rocprofv3 -d directory of one --pmc pass (run_counter_collection.csv); only the
conv kernels' dispatches (conv_pipe16 / conv_split / conv_gemm) are averaged.  Derived:
  kernel cycles        = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
  mfma_busy_frac       = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles * 1024 SIMDs)
  mfma                 = SQ_VALU_MFMA_BUSY_CYCLES / 32 (v_mfma_f32_32x32x16: 32 busy cycles)
  valu_per_mfma        = (SQ_INSTS_VALU - mfma) / mfma   (SQ_INSTS_VALU counts the MFMAs too)
  lds_per_mfma         = SQ_INSTS_LDS / mfma
  waves_per_cu         = 4 * SQ_WAVE_CYCLES / (kernel cycles * 256)   (occupancy)
  *_frac               = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_INST_LDS, SQ_ACTIVE_INST_ANY,
                         SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (all quad-cycles)
"""
import csv
import json
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(dict)
    names = {}
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if not any(k in n for k in ("conv_pipe16", "conv_split", "conv_gemm", "conv_expand16", "conv_big16", "conv_haloc16")):
                continue
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[did] = n.split("(")[0].replace("void ", "")
    return per, names


def summarise(dirs):
    tot = defaultdict(float)
    cnt = defaultdict(int)
    kern = set()
    for d in dirs:
        per, names = load(d)
        for did, cs in per.items():
            kern.add(names[did])
            for k, v in cs.items():
                tot[k] += v
                cnt[k] += 1
    avg = {k: tot[k] / cnt[k] for k in tot}
    cyc = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8
    out = {"counters_per_dispatch": {k: round(v, 1) for k, v in sorted(avg.items())},
           "dispatches": max(cnt.values()) if cnt else 0, "kernels": sorted(kern)}
    if cyc:
        out["kernel_cycles"] = round(cyc)
        mb = avg.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if mb:
            n = mb / 32
            out["mfma_busy_frac"] = round(mb / (cyc * 1024), 4)
            out["mfma"] = round(n)
            if "SQ_INSTS_VALU" in avg:
                out["valu_per_mfma"] = round((avg["SQ_INSTS_VALU"] - n) / n, 2)
            if "SQ_INSTS_LDS" in avg:
                out["lds_per_mfma"] = round(avg["SQ_INSTS_LDS"] / n, 2)
        if "SQ_WAVE_CYCLES" in avg:
            out["waves_per_cu"] = round(4 * avg["SQ_WAVE_CYCLES"] / (cyc * 256), 2)
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if k in avg:
                out[k.lower() + "_frac"] = round(avg[k] / wc, 4)
    return out


def main(out_json, *specs):
    res = {}
    for sp in specs:
        name, dirs = sp.split("=", 1)
        res[name] = summarise(dirs.split(","))
        r = res[name]
        print(f"{name:34s} busy {r.get('mfma_busy_frac', float('nan')):.3f} "
              f"valu/mfma {r.get('valu_per_mfma', float('nan')):6.2f} "
              f"lds/mfma {r.get('lds_per_mfma', float('nan')):5.2f} "
              f"waves/CU {r.get('waves_per_cu', float('nan')):5.2f} "
              f"wait_any {r.get('sq_wait_any_frac', float('nan')):.3f} "
              f"wait_inst_lds {r.get('sq_wait_inst_lds_frac', float('nan')):.3f}")
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into HBM bytes per kernel launch.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d D1 -o run -- python3 bench.py ...
    rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d D2 -o run -- python3 bench.py ...
    python tools/pmc_traffic.py D1 D2 profiles/roundN_conv_traffic.json

FETCH_SIZE and WRITE_SIZE are in KiB (their rocprofv3 expressions end in /1024); on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled
(MI355X_MICROARCH.md, HBM section).  Both counters include Infinity-Cache hits.
"""
import csv
import json
import sys
from collections import defaultdict


def template_args(name):
    """The template arguments of a demangled kernel name: 'void f<1, 256, true, 2>(...)' ->
    ['1', '256', 'true', '2']."""
    head = name.split("(")[0]
    if "<" not in head:
        return []
    return [s.strip() for s in head[head.index("<") + 1:head.rindex(">")].split(",")]


def family(name):
    # conv_big16<DT, BM, BN, XBN, RES>: RES 1 / 2 = conv1 forming the previous block output
    # (the fold, its own family beside the MFMA one; bench.py's roofline 'fold')
    if "conv_big16<" in name and template_args(name)[4:5] in (["1"], ["2"]):
        return "conv_fold16"
    if "conv_gemm_f32" in name or "conv_split_f32" in name:
        return "conv_f32"        # the fp32 conv family: split kernels + stems on conv_gemm_f32
    if any(k in name for k in ("conv_gemm_h16", "conv_pipe16", "conv_halo16", "conv_haloc16",
                               "conv_big16", "conv_expand16")):
        return "conv_h16"        # the 16-bit conv family: pipelined, halo (64 and 128-512
                                 # channels), 256-row, expansion + fallback shapes
    return name.split("(")[0].replace("void ", "")


def load(d, counter):
    out = {}
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def library_sha16():
    import hashlib
    import os
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "multimodal-auv_amd", "mauv", "libmauv_hip.so")
    with open(so, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main(fetch_dir, write_dir, out_json, fam=None):
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    agg = defaultdict(lambda: [0, 0, 0.0, 0.0])
    for _, (n, v) in fe.items():
        a = agg[family(n)]
        a[0] += 1
        a[2] += 2.0 * v * 1024.0
    for _, (n, v) in wr.items():
        a = agg[family(n)]
        a[1] += 1
        a[3] += v * 1024.0
    rows = {k: {"launches": v[0], "read_bytes": v[2], "write_bytes": v[3],
                "bytes_per_launch": (v[2] + v[3]) / max(v[0], 1)} for k, v in agg.items()}
    # the conv family of the profiled step: the one with more launches (a 16-bit step also runs
    # the fusion head's fp32 linears on the split kernel)
    fam = fam or max((k for k in ("conv_f32", "conv_h16") if k in rows),
                     key=lambda k: rows[k]["launches"])
    conv = rows[fam]
    res = {"kernel": {"conv_f32": "conv_f32 (conv_split_f32 + stem conv_gemm_f32)",
                      "conv_h16": "conv_h16 (conv_pipe16 + conv_halo16 + conv_haloc16 + conv_big16 + conv_expand16 + conv_gemm_h16)"}[fam],
           "bytes_per_launch": round(conv["bytes_per_launch"]),
           "launches": conv["launches"], "per_family": rows,
           "method": "2*FETCH_SIZE + WRITE_SIZE (rocprofv3 PMC, separate passes, KiB units)",
           # the library the passes profiled: bench.py reports whether its own matches
           "library_sha16": library_sha16()}
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in sorted(rows.items(), key=lambda kv: -(kv[1]["read_bytes"] + kv[1]["write_bytes"]))[:15]:
        print(f"{k[:50]:50s} {v['launches']:6d} {v['bytes_per_launch'] / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:5])

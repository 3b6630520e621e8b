"""Per-shape HBM traffic of the conv kernels from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) over `tools/conv_bench.py --mark` (each timed pass is preceded by a torch.flip
marker kernel; conv_bench's MARK lines name the pass and its algorithmic bytes).

    python tools/shape_traffic.py BENCH_STDOUT FETCH_DIR WRITE_DIR [OUT_JSON]

FETCH_SIZE is doubled on gfx950 (MI355X_MICROARCH.md, HBM section); both counters are KiB.
"""
import csv
import json
import sys


def counters(d, name):
    rows = []
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == name:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return rows


def split_by_marker(rows):
    """[[conv-kernel KiB values of pass i] ...] in marker order."""
    out, cur = [], None
    for _, k, v in rows:
        if "flip" in k:
            cur = []
            out.append(cur)
        elif cur is not None and ("conv_" in k or "stem" in k):
            cur.append(v)
    return out


def main():
    marks = [ln.split() for ln in open(sys.argv[1]) if ln.startswith("MARK ")]
    fe = split_by_marker(counters(sys.argv[2], "FETCH_SIZE"))
    wr = split_by_marker(counters(sys.argv[3], "WRITE_SIZE"))
    res, tot_alg, tot_hbm = [], 0.0, 0.0
    for m, f, w in zip(marks, fe, wr):
        _, i, trunk, name, kind, key, alg, calls = m
        calls = int(calls)
        hbm = (2.0 * sum(f) + sum(w)) * 1024.0 / calls
        rd, wt = 2.0 * sum(f) * 1024.0 / calls, sum(w) * 1024.0 / calls
        res.append({"trunk": trunk, "layer": name, "pass": kind, "shape": key, "alg_bytes": float(alg),
                    "hbm_bytes": hbm, "read_bytes": rd, "write_bytes": wt,
                    "ratio": hbm / float(alg)})
        tot_alg += float(alg)
        tot_hbm += hbm
    res.sort(key=lambda r: -(r["hbm_bytes"] - r["alg_bytes"]))
    print(f"{'trunk':6s} {'layer':9s} {'pass':6s} {'shape':22s} {'alg MB':>8s} {'read MB':>8s} "
          f"{'write MB':>8s} {'ratio':>6s}")
    for r in res[:40]:
        print(f"{r['trunk']:6s} {r['layer']:9s} {r['pass']:6s} {r['shape']:22s} "
              f"{r['alg_bytes'] / 1e6:8.1f} {r['read_bytes'] / 1e6:8.1f} {r['write_bytes'] / 1e6:8.1f} "
              f"{r['ratio']:6.2f}")
    print(f"TOTAL (unique shapes): algorithmic {tot_alg / 1e9:.2f} GB, HBM {tot_hbm / 1e9:.2f} GB, "
          f"ratio {tot_hbm / max(tot_alg, 1):.2f}")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump({"method": "2*FETCH_SIZE + WRITE_SIZE per conv pass (rocprofv3 PMC, separate "
                                 "passes) over tools/conv_bench.py --mark", "passes": res}, f, indent=1)


if __name__ == "__main__":
    main()

"""Per-kernel statistics of the STEADY training steps of a rocprofv3 kernel trace (VERDICT r5:
the --stats summaries of a short bench run also count the process's setup — FusedAdam's state
fills for 696 tensors, model.to() copies, the first-call kernels).

A step ends with its Adam launch (adam_kernel*, one per step).  The kernels after the first Adam
launch up to and including the last one are K = (number of Adam launches - 1) steady steps
(the first step is the warm-up; everything before it is setup); per kernel name: calls, total,
average and share, divided by K.

    python tools/steady_stats.py <rocprofv3 -d dir> [out.csv]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, out=None):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    if len(ad) < 2:
        raise SystemExit(f"{f}: {len(ad)} Adam launches; need a warm-up step and >= 1 more")
    K = len(ad) - 1
    agg = defaultdict(lambda: [0, 0])
    for r in rows[ad[0] + 1:ad[-1] + 1]:
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    res = sorted(agg.items(), key=lambda kv: -kv[1][1])
    fh = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(fh)
    w.writerow(["Name", "Calls_per_step", "TotalDurationNs_per_step", "AverageNs", "Percentage",
                "steady_steps"])
    for name, (n, ns) in res:
        w.writerow([name, round(n / K, 2), round(ns / K), round(ns / n), round(100 * ns / tot, 3),
                    K])
    if out:
        fh.close()
        print(f"{K} steady steps, {tot / K / 1e6:.2f} ms of kernel time per step, "
              f"{sum(v[0] for v in agg.values()) / K:.0f} launches per step -> {out}")


if __name__ == "__main__":
    main(*sys.argv[1:3])

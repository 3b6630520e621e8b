"""Per-kernel time difference between two rocprofv3 --stats runs of the same command (an A/B of
a switch): the kernels whose total time moved most, and the totals.

    python tools/kstat_diff.py <rocprofv3 -d dir A> <rocprofv3 -d dir B> [top]
"""
import csv
import glob
import os
import sys


def load(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))[0]
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f))}


def main(a, b, top=25):
    A, B = load(a), load(b)
    ta, tb = sum(v[1] for v in A.values()), sum(v[1] for v in B.values())
    print(f"total kernel time A {ta / 1e6:.2f} ms  B {tb / 1e6:.2f} ms  B/A {tb / ta:.4f}")
    rows = []
    for k in set(A) | set(B):
        ca, na = A.get(k, (0, 0.0))
        cb, nb = B.get(k, (0, 0.0))
        rows.append((nb - na, k, ca, na, cb, nb))
    rows.sort(key=lambda r: -abs(r[0]))
    print(f"{'dB-A ms':>9} {'calls A':>8} {'ms A':>9} {'calls B':>8} {'ms B':>9}  kernel")
    for d, k, ca, na, cb, nb in rows[:int(top)]:
        print(f"{d / 1e6:9.3f} {ca:8d} {na / 1e6:9.3f} {cb:8d} {nb / 1e6:9.3f}  {k[:110]}")


if __name__ == "__main__":
    main(*sys.argv[1:4])

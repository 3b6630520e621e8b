"""Per-step GPU occupancy of a rocprofv3 kernel trace taken with the trunks on their concurrent
streams: for each step (adam_kernel to adam_kernel) the wall span, the union of kernel intervals
(time with at least one kernel running), the summed kernel time, and the idle gaps > 20 us —
whether a step is bound by its kernels or by gaps between them.

    python tools/busy_union.py <dir with *kernel_trace.csv>
"""
import csv
import glob
import os
import re
import sys


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    for a, b in zip(ad, ad[1:]):
        seq = rows[a + 1:b + 1]
        t0 = int(rows[a]["End_Timestamp"])
        t1 = int(rows[b]["End_Timestamp"])
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                    for r in seq)
        busy, cur_s, cur_e, gaps = 0, None, None, []
        last_name = ""
        for s, e, n in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    if s - cur_e > 20_000:
                        gaps.append((s - cur_e, re.sub(r"\(.*", "", last_name)[:50],
                                     re.sub(r"\(.*", "", n)[:50]))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            last_name = n if e >= (cur_e or 0) else last_name
        busy += cur_e - cur_s
        ksum = sum(e - s for s, e, _ in iv)
        print(f"step: wall {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms "
              f"({busy / (t1 - t0):.3f}), kernel sum {ksum / 1e6:.2f} ms, launches {len(iv)}, "
              f"gaps>20us {len(gaps)} totalling {sum(g[0] for g in gaps) / 1e6:.2f} ms")
        for g in sorted(gaps, reverse=True)[:6]:
            print(f"   gap {g[0] / 1e3:.0f} us after {g[1]} before {g[2]}")


if __name__ == "__main__":
    main(sys.argv[1])

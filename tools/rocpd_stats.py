"""Per-kernel totals from rocprofv3 SQLite output (run_results.db, the default format when
--output-format is not given): python tools/rocpd_stats.py DIR [DIR2] [--per N] [--top K].
Kernel names are grouped by template head (conv_pipe16<MODE> etc.); with two directories the
columns are side by side (an A/B).  --per divides the totals (e.g. by the traced steps)."""
import argparse
import re
import sqlite3


def load(d, per):
    c = sqlite3.connect(f"{d}/run_results.db")
    agg = {}
    for name, dur in c.execute("select name, duration from kernels"):
        n = re.sub(r"\(.*", "", name).replace("void ", "")
        n = re.sub(r"conv_pipe16<(\d).*", r"conv_pipe16<\1>", n)
        n = re.sub(r"conv_split_f32<(\d).*", r"conv_split_f32<\1>", n)
        agg[n] = agg.get(n, 0.0) + dur / 1e6 / per
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ds = [load(d, a.per) for d in a.dirs]
    print("total ms " + "  ".join(f"{sum(d.values()):9.2f}" for d in ds))
    keys = sorted(set().union(*ds), key=lambda k: -max(d.get(k, 0.0) for d in ds))
    for k in keys[:a.top]:
        print("  ".join(f"{d.get(k, 0.0):9.2f}" for d in ds) + "  " + k[:100])


if __name__ == "__main__":
    main()

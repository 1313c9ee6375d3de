"""Per-kernel duration statistics from a rocprofv3 rocpd database (the
default output of `rocprofv3 --kernel-trace --stats`), grouped by kernel AND
launch grid so that e.g. the 1 M-block C2 launches of bench.py are separated
from the 2 048-block launches of its end-to-end leg.

usage: python tools/rocpd_stats.py <results.db> [--csv out.csv]
"""
import argparse
import csv
import re
import sqlite3
import statistics
import sys


def short(name: str) -> str:
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select name, grid_x, workgroup_x, duration from kernels"))
    groups = {}
    for name, gx, wx, dur in rows:
        groups.setdefault((short(name), gx, wx), []).append(dur / 1e3)  # ns -> us
    out = []
    for (k, gx, wx), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": k, "grid_x": gx, "workgroup_x": wx, "calls": len(d), "total_us": round(sum(d), 1),
                    "avg_us": round(statistics.mean(d), 2), "median_us": round(statistics.median(d), 2),
                    "min_us": round(min(d), 2), "max_us": round(max(d), 2)})
    w = csv.DictWriter(open(a.csv, "w", newline="") if a.csv else sys.stdout, fieldnames=list(out[0]))
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()

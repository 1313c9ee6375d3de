"""Dispatch timeline from a rocprofv3 --kernel-trace results.db: every
dispatch in start order with its duration and the idle gap since the previous
dispatch ended (same device), so the cost of launch boundaries in a pipeline
shows next to the kernels' own time.

    python tools/kernel_timeline.py <rocprofv3 output dir> [--after NAME] [--last N]

--after NAME: start at the first dispatch whose name contains NAME (e.g. the
first k_count_hist of bench.py's c3 leg); --last N: only the last N rows.
A per-name summary (count, mean duration, mean gap before it) ends the output.
"""
import argparse
import collections
import glob
import sqlite3


def rows(path):
    db = glob.glob(path + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    q = (f"select s.display_name, d.start, d.end, d.grid_size_x from {kd} d join {ks} s on d.kernel_id = s.id "
         f"order by d.start")
    out = []
    for name, st, en, grid in c.execute(q):
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        out.append((short, int(st), int(en), grid))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--after", default="")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rs = rows(a.dir)
    if a.after:
        i = next((k for k, r in enumerate(rs) if a.after in r[0]), len(rs))
        rs = rs[i:]
    if a.last:
        rs = rs[-a.last:]
    prev_end = None
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for name, st, en, grid in rs:
        gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"{name[:56]:56s} {(en - st) / 1e3:9.1f} us  gap {gap:8.1f} us  grid {grid}")
        g = agg[name[:56]]
        g[0] += 1
        g[1] += (en - st) / 1e3
        g[2] += gap
        prev_end = en if prev_end is None else max(prev_end, en)
    print("--- summary: name, dispatches, mean us, mean gap before (us)")
    for name, (n, d, g) in agg.items():
        print(f"{name:56s} {n:4d} {d / n:9.1f} {g / n:8.1f}")


if __name__ == "__main__":
    main()

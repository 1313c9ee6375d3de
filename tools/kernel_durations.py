"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace results.db,
in launch order (tools/profile_batches.sh and the replay experiments use it).

    python tools/kernel_durations.py <rocprofv3 output dir> [name substring]
"""
import glob
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    q = f"select s.display_name, d.end - d.start, d.grid_size_x from {kd} d join {ks} s on d.kernel_id = s.id order by d.start"
    for name, dur, grid in c.execute(q):
        if pat in name:
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            print(f"{short:60s} {dur / 1000:10.1f} us  grid {grid}")


if __name__ == "__main__":
    main()

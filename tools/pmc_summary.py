"""Summarise rocprofv3 PMC csv passes: per kernel, mean of each counter.

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json --blocks N --kernel SUBSTR]
       python tools/pmc_summary.py gpurun_out/<dir> --pipeline SHAPE --image-bytes N --json out.json
         (a C3 leg: every dispatch from the first --first-kernel dispatch on, summed and divided
          by the number of --first-kernel dispatches = pipeline calls; bench.py reads the json)
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half of
a wide coalesced streaming read (MI355X_MICROARCH.md, HBM section), so
hbm_read_bytes = 2 * FETCH_SIZE * 1024 for those kernels.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                acc[k]["_dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def load_pipeline(d, first_kernel):
    """Per pipeline call: the sum over every dispatch from the first
    `first_kernel` dispatch on (the image-building kernels run before it),
    divided by the number of `first_kernel` dispatches.  Returns
    (per-call counter sums, calls, per-kernel dispatch counts)."""
    tot = defaultdict(float)
    calls = None
    kernels = defaultdict(int)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        # the first kernel by name prefix (k_count_hist is templated on its workgroup size)
        first = [r for r in rows if short(r["Kernel_Name"]).startswith(first_kernel)]
        start = min((int(r["Dispatch_Id"]) for r in first), default=None)
        if start is None:
            raise SystemExit(f"{f}: no {first_kernel} dispatch")
        n = len({r["Dispatch_Id"] for r in first})
        if calls is not None and n != calls:
            raise SystemExit(f"{f}: {n} pipeline calls, other passes had {calls}")
        calls = n
        seen = set()
        for r in rows:
            if int(r["Dispatch_Id"]) < start:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen and r["Counter_Name"] in ("FETCH_SIZE",):
                seen.add(r["Dispatch_Id"])
                kernels[short(r["Kernel_Name"])] += 1
    return {c: v / calls for c, v in tot.items()}, calls, {k: v / calls for k, v in kernels.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--kernel", default="k_full_blocks4<1024, false>")
    ap.add_argument("--library", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                       "revel_amd", "librevel_wal.so"),
                    help="the librevel_wal.so the PMC pass ran (its SHA-256 goes into the json)")
    ap.add_argument("--pipeline", default=None, help="C3 leg shape (zipf | small): per-call pipeline totals")
    ap.add_argument("--first-kernel", default="k_count_hist")
    ap.add_argument("--image-bytes", type=int, default=None)
    a = ap.parse_args()
    if a.pipeline:
        import hashlib
        cs, calls, kernels = load_pipeline(a.dir, a.first_kernel)
        with open(a.library, "rb") as fh:
            sha = hashlib.sha256(fh.read()).hexdigest()
        fetch, write = cs.get("FETCH_SIZE"), cs.get("WRITE_SIZE")
        out = {"leg": "c3" if a.pipeline == "zipf" else "c3_small", "shape": a.pipeline,
               "image_bytes": a.image_bytes, "library_sha256": sha, "calls": calls,
               "dispatches_per_call": kernels, "fetch_size_kib_per_call": fetch, "write_size_kib_per_call": write,
               "hbm_read_bytes_per_call": None if fetch is None else 2 * fetch * 1024,
               "hbm_write_bytes_per_call": None if write is None else write * 1024,
               "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM); WRITE_SIZE x1; summed over every "
                             "dispatch of one count -> scan -> verify call"}
        if fetch is not None and write is not None:
            out["hbm_bytes_per_call"] = out["hbm_read_bytes_per_call"] + out["hbm_write_bytes_per_call"]
            if a.image_bytes:
                out["read_over_image"] = round(out["hbm_read_bytes_per_call"] / a.image_bytes, 3)
        print(json.dumps(out, indent=1))
        if a.json:
            with open(a.json, "w") as f:
                json.dump(out, f, indent=1)
        return
    res = load(a.dir)
    for k, cs in res.items():
        print(f"== {k}")
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {v:16.1f}")
        if "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"]:
            w = cs["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if c in cs:
                    print(f"   share {c:26s} {cs[c] / w:8.3f}")
        if "GRBM_GUI_ACTIVE" in cs:
            print(f"   eff clock GHz ~ {cs['GRBM_GUI_ACTIVE'] / 8 / cs['_dur_ns']:.3f}")
    if a.json:
        cs = res.get(a.kernel)
        if cs is None:
            raise SystemExit(f"kernel {a.kernel} not found; have {list(res)}")
        fetch = cs.get("FETCH_SIZE")
        write = cs.get("WRITE_SIZE")
        import hashlib
        with open(a.library, "rb") as fh:
            sha = hashlib.sha256(fh.read()).hexdigest()
        out = {"kernel": a.kernel, "blocks": a.blocks, "library_sha256": sha,
               "fetch_size_kib": fetch, "write_size_kib": write,
               "hbm_read_bytes_per_launch": None if fetch is None else 2 * fetch * 1024,
               "hbm_write_bytes_per_launch": None if write is None else write * 1024,
               "correction": "gfx950: FETCH_SIZE x2 for wide coalesced reads (MI355X_MICROARCH.md HBM); "
                             "WRITE_SIZE x1",
               "counters": cs}
        if fetch is not None and write is not None:
            out["hbm_bytes_per_launch"] = out["hbm_read_bytes_per_launch"] + out["hbm_write_bytes_per_launch"]
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes per kernel (mean per dispatch).

  python tools/pmc_summary.py gpurun_out/pmc_dir [kernel-substring ...] [--out file.json]
With --out, the first matching kernel's corrected HBM bytes per launch are
written as {"kernel", "hbm_bytes_per_launch", "fetch_bytes", "write_bytes",
"counters"} (what bench.py reads as roofline.traffic).
FETCH_SIZE / WRITE_SIZE are reported raw (KB, as rocprofv3 gives them) and
as bytes with the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
counts half of a 16-B/lane streaming read: x2)."""
import collections
import csv
import glob
import json
import sys


def main():
    argv = sys.argv[1:]
    out_path = None
    if "--out" in argv:
        i = argv.index("--out")
        out_path = argv[i + 1]
        del argv[i:i + 2]
    d = argv[0]
    keys = argv[1:] or [""]
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            short = name.replace("(anonymous namespace)::", "").split("(")[0][-90:]
            rows[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for kname, cnt in rows.items():
        m = {c: sum(v) / len(v) for c, v in cnt.items()}
        if "FETCH_SIZE" in m:
            m["fetch_bytes_corrected"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            m["write_bytes"] = m["WRITE_SIZE"] * 1024
        out[kname] = m
    print(json.dumps(out, indent=1))
    if out_path and out:
        kname, m = next(iter(out.items()))
        rec = {"kernel": kname, "fetch_bytes": m.get("fetch_bytes_corrected"), "write_bytes": m.get("write_bytes"),
               "hbm_bytes_per_launch": (m.get("fetch_bytes_corrected") or 0) + (m.get("write_bytes") or 0),
               "correction": "FETCH_SIZE x 1024 x 2 (gfx950 16-B/lane streaming reads), WRITE_SIZE x 1024",
               "counters": m}
        with open(out_path, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-launch means of rocprofv3 PMC counters for kernels matching a pattern.

usage: tools/pmc_summary.py <prof_dir> [kernel_substring] [--prefix P] [--json out.json]
Sums each counter over its per-XCD/SE rows per dispatch, then averages over
dispatches of the matching kernel (warm-up launch included)."""
import collections
import csv
import glob
import json
import os
import sys


def summarize(prof_dir, pat="decode", prefix=""):
    out = {}
    for f in sorted(glob.glob(os.path.join(prof_dir, prefix + "*", "run_counter_collection.csv"))):
        byd = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                byd[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, d in byd.items():
            out[c] = sum(d.values()) / len(d)
    return out


if __name__ == "__main__":
    argv = sys.argv[1:]
    prefix = ""
    if "--prefix" in argv:
        i = argv.index("--prefix")
        prefix = argv[i + 1]
        del argv[i:i + 2]
    if "--json" in argv:
        i = argv.index("--json")
        jpath = argv[i + 1]
        del argv[i:i + 2]
    else:
        jpath = None
    args = argv
    res = summarize(args[0], args[1] if len(args) > 1 else "decode", prefix)
    for k in sorted(res):
        print(f"{k:32s} {res[k]:.6g}")
    if jpath:
        json.dump(res, open(jpath, "w"), indent=1)

#!/usr/bin/env python3
"""Per-dispatch means of every PMC pass directory under gpurun_out/<tag> (rocprofv3
--pmc ... --output-format csv), plus per-wave-iteration instruction counts for a 2^24-auction
headline launch. Diagnostic.    python tools/summarize_pmc.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import os
import sys


def pmc(path):
    fs = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return None, 0
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for d in per.values() for c in d})
    return {c: sum(d[c] for d in per.values()) / len(per) for c in names}, len(per)


def main():
    root = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
    out = {}
    for d in sorted(os.listdir(root)):
        p = os.path.join(root, d)
        if os.path.isdir(p):
            v, n = pmc(p)
            if v:
                out[d] = {"dispatches": n, "per_dispatch_mean": v}
    wi = batch / 64
    flat = {k: v for part in out.values() for k, v in part["per_dispatch_mean"].items()}
    per_wi = {k: flat[k] / wi for k in flat if k.startswith("SQ_INSTS")}
    out["per_wave_iteration"] = per_wi
    if "FETCH_SIZE" in flat and "WRITE_SIZE" in flat:
        out["hbm_bytes_per_launch"] = flat["FETCH_SIZE"] * 1024 * 2 + flat["WRITE_SIZE"] * 1024
        out["hbm_over_algorithmic"] = out["hbm_bytes_per_launch"] / (141 * batch)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

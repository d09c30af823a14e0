#!/usr/bin/env python3
"""Per-dispatch means of every PMC pass directory under gpurun_out/<tag> (rocprofv3 --pmc ...
--output-format csv), grouped per workload, with per-wave-tile instruction counts, cycle
fractions and HBM traffic against each workload's OWN algorithmic bytes. Diagnostic.

    python tools/summarize_pmc.py gpurun_out/prof_<tag> [bench_driver.log]

Pass directories are named <workload>_<pass> (c1_sqA, c4_fetch, ...; a name without a
c<n>_ prefix is the headline). Batch and algorithmic bytes per auction of each workload come
from the bench JSON line (the headline's `config` / configs_<n>), given or found as
<dir>/bench_driver.log. The first dispatch of every pass is dropped (the populations'
iteration-0 launch runs uninitialised learners; the first launch of a process is cold)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def pmc(path, skip_first=True):
    fs = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return None, 0
    per = collections.OrderedDict()
    for r in csv.DictReader(open(fs[0])):
        d = per.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    keys = sorted(per)
    if skip_first and len(keys) > 2:
        keys = keys[1:]
    names = sorted({c for k in keys for c in per[k]})
    return {c: sum(per[k][c] for k in keys) / len(keys) for c in names}, len(keys)


def bench_line(path):
    if not path or not os.path.exists(path):
        return None
    line = None
    for ln in open(path):
        if ln.startswith("{"):
            line = json.loads(ln)
    return line


def workload_shape(bench, wl):
    """(batch, algorithmic bytes per auction) of a workload from the bench line."""
    if bench is None:
        return None, None
    if wl == "headline":
        return bench["config"]["auctions_per_gpu_per_step"], bench["roofline"]["algorithmic_bytes_per_auction"]
    b = bench.get(f"configs_{wl[1:]}")
    if b is None:
        return None, None
    return b["auctions_per_gpu_per_step"], b["algorithmic_bytes_per_auction"]


def derive(v, batch, bpa):
    out = {}
    if batch:
        tiles = batch / 64
        out["per_wave_tile"] = {k: v[k] / tiles for k in v if k.startswith("SQ_INSTS")}
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
            if k in v:
                out.setdefault("frac_of_wave_cycles", {})[k] = v[k] / wc
    if "SQ_WAVES" in v and wc:
        out["wave_cycles_per_wave"] = wc / v["SQ_WAVES"]
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        t = v["FETCH_SIZE"] * 1024 * 2 + v["WRITE_SIZE"] * 1024  # gfx950 corrections
        out["hbm_bytes_per_launch"] = t
        if batch and bpa:
            out["algorithmic_bytes_per_launch"] = batch * bpa
            out["hbm_over_algorithmic"] = t / (batch * bpa)
    return out


def main():
    root = sys.argv[1]
    bench = bench_line(sys.argv[2] if len(sys.argv) > 2 else os.path.join(root, "bench_driver.log"))
    groups = collections.defaultdict(dict)
    for d in sorted(os.listdir(root)):
        p = os.path.join(root, d)
        if not os.path.isdir(p):
            continue
        v, n = pmc(p)
        if not v:
            continue
        m = re.match(r"(c\d)_(.+)", d)
        wl, pas = (m.group(1), m.group(2)) if m else ("headline", d)
        groups[wl][pas] = {"dispatches": n, "per_dispatch_mean": v}
    out = {}
    for wl, passes in groups.items():
        batch, bpa = workload_shape(bench, wl)
        flat = {k: x for p in passes.values() for k, x in p["per_dispatch_mean"].items()}
        out[wl] = {"batch": batch, "algorithmic_bytes_per_auction": bpa, "passes": passes,
                   **derive(flat, batch, bpa)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

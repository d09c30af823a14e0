#!/usr/bin/env python3
"""Per-kernel, per-dispatch means of every PMC pass directory under gpurun_out/prof_<tag>
(rocprofv3 --pmc ... --output-format csv), keyed by workload AND kernel name (the kernel
name carries its template arguments, so P = 2 and P = 8 builds never mix), with per-wave-tile
instruction counts, cycle fractions and HBM traffic against the workload's OWN algorithmic
bytes. Diagnostic; its output is the tracked profiles/<tag>_pmc_summary.json from which
tools/make_pmc_traffic.py derives profiles/pmc_traffic.json.

    python tools/summarize_pmc.py gpurun_out/prof_<tag> [bench_driver.log]

Pass directories are named <workload>_<pass>: workloads `hd` (the headline), c1, c2, c3, c4,
c1p8, c4p8 (bench.py's configs_1 ... configs_4_p8 lines), c1g (configs_1's generate mode); passes fetch, write (FETCH_SIZE /
WRITE_SIZE: separate runs), sqA, sqB. Batch and algorithmic bytes per auction come from the
bench JSON line (given, or <dir>/bench_driver.log). The first dispatch of every kernel in a
pass is dropped (the populations' iteration-0 launch runs uninitialised learners; the first
launch of a process is cold)."""
import collections
import csv
import glob
import json
import os
import re
import sys

WORKLOADS = {"hd": "headline", "c1": "configs_1", "c2": "configs_2", "c3": "configs_3", "c4": "configs_4",
             "c1p8": "configs_1_p8", "c4p8": "configs_4_p8", "c1g": "configs_1.generate_mode"}


def pmc_by_kernel(path, skip_first=True):
    """{kernel name: (per-dispatch mean {counter: value}, dispatches)} of one pass directory."""
    fs = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return {}
    per = collections.defaultdict(lambda: collections.OrderedDict())
    for r in csv.DictReader(open(fs[0])):
        d = per[r["Kernel_Name"]].setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, disp in per.items():
        ids = sorted(disp)
        if skip_first and len(ids) > 2:
            ids = ids[1:]
        names = sorted({c for i in ids for c in disp[i]})
        out[k] = ({c: sum(disp[i][c] for i in ids) / len(ids) for c in names}, len(ids))
    return out


def pmc(path, skip_first=True):
    """The per-dispatch mean of a pass holding ONE kernel (kept for the older tools)."""
    by = pmc_by_kernel(path, skip_first)
    if len(by) != 1:
        return None, 0
    return next(iter(by.values()))


def bench_line(path):
    if not path or not os.path.exists(path):
        return None
    line = None
    for ln in open(path):
        if ln.startswith("{"):
            line = json.loads(ln)
    return line


def workload_shape(bench, key):
    """(batch, algorithmic bytes per auction) of a bench line entry."""
    if bench is None:
        return None, None
    if key == "headline":
        return bench["config"]["auctions_per_gpu_per_step"], bench["roofline"]["algorithmic_bytes_per_auction"]
    parent, _, sub = key.partition(".")
    b = bench.get(parent)
    if b is None:
        return None, None
    if sub:  # a generate-mode line: the parent line's batch, its own (write) bytes
        return b["auctions_per_gpu_per_step"], b.get(sub, {}).get("algorithmic_bytes_per_auction")
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
        if "SQ_WAVES" in v:
            out["wave_cycles_per_wave"] = wc / v["SQ_WAVES"]
    if "SQ_LDS_BANK_CONFLICT" in v and "SQ_ACTIVE_INST_LDS" in v and v["SQ_ACTIVE_INST_LDS"]:
        out["lds_bank_conflict_cycles_per_lds_active"] = v["SQ_LDS_BANK_CONFLICT"] / v["SQ_ACTIVE_INST_LDS"]
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        t = v["FETCH_SIZE"] * 1024 * 2 + v["WRITE_SIZE"] * 1024  # KiB units; FETCH_SIZE x 2 on gfx950
        out["hbm_bytes_per_launch"] = t
        out["hbm_bytes_formula"] = "FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 (per-dispatch means)"
        if batch and bpa:
            out["algorithmic_bytes_per_launch"] = batch * bpa
            out["hbm_over_algorithmic"] = t / (batch * bpa)
    return out


def summarize(root, bench):
    groups = collections.defaultdict(lambda: collections.defaultdict(dict))  # wl -> kernel -> pass
    for d in sorted(os.listdir(root)):
        p = os.path.join(root, d)
        m = re.match(r"(hd|c\dp8|c\dg|c\d)_(.+)$", d)
        if not os.path.isdir(p) or not m:
            continue
        for k, (v, n) in pmc_by_kernel(p).items():
            groups[m.group(1)][k][m.group(2)] = {"dispatches": n, "per_dispatch_mean": v}
    out = {}
    for wl, kernels in groups.items():
        key = WORKLOADS[wl]
        batch, bpa = workload_shape(bench, key)
        ent = {"bench_key": key, "batch": batch, "algorithmic_bytes_per_auction": bpa, "kernels": {}}
        for k, passes in kernels.items():
            flat = {c: x for p in passes.values() for c, x in p["per_dispatch_mean"].items()}
            ent["kernels"][k] = {"passes": passes, **derive(flat, batch, bpa)}
        out[wl] = ent
    return out


def main():
    root = sys.argv[1]
    bench = bench_line(sys.argv[2] if len(sys.argv) > 2 else os.path.join(root, "bench_driver.log"))
    print(json.dumps(summarize(root, bench), indent=1))


if __name__ == "__main__":
    main()

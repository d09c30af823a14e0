#!/usr/bin/env python3
"""One row per (bench line, simulate kernel) from the per-workload kernel traces of
tools/prof_round.sh (gpurun_out/prof_<tag>/tr_<workload>/, each its own rocprofv3 run of one
bench line), beside the HIP-event kernel_ms the same run's bench JSON line reports -- so every
BENCH line's kernel_ms is matched to a trace row of its own workload (two lines whose kernels
share a name, configs_2 and configs_3, no longer fold into one row).

    python tools/summarize_traces.py gpurun_out/prof_<tag> > profiles/<tag>_kernel_stats_by_workload.csv

The trace average covers every launch of the kernel in the run (warm-up included); the bench's
kernel_ms is the mean over the timed steps of ag_simulate on its stream (the kernel plus the
~5 us k_reduce_counters). Columns: workload, bench line, kernel, calls, trace average / min /
max (us), bench kernel_ms (us), trace average / bench.
"""
import csv
import glob
import json
import os
import re
import sys

LINES = {  # trace directory -> bench line keys whose kernels it ran
    "hd": ["headline", "generate_mode"],
    "c1": ["configs_1", "configs_1.generate_mode"],
    "c1p8": ["configs_1_p8", "configs_1_p8.generate_mode"],
    "c2": ["configs_2", "configs_2.generate_mode"],
    "c3": ["configs_3", "configs_3.generate_mode"],
    "c4": ["configs_4", "configs_4.generate_mode"],
    "c4p8": ["configs_4_p8", "configs_4_p8.generate_mode"],
}


def bench_line(log):
    js = [ln for ln in open(log) if ln.startswith("{")]
    return json.loads(js[-1]) if js else {}


def line_ms(res, key):
    if key == "headline":
        return res.get("roofline", {}).get("kernel_ms")
    obj = res
    for part in key.split("."):
        obj = obj.get(part, {}) if isinstance(obj, dict) else {}
    return obj.get("kernel_ms") if isinstance(obj, dict) else None


def kernel_of(name, key):
    """Is trace kernel `name` the simulate kernel of bench line `key`?"""
    gen = key.endswith("generate_mode")
    name = name[len("void "):] if name.startswith("void ") else name
    if key in ("headline", "generate_mode"):
        return name.startswith("ag::k_oracle<2, 6, " + ("true" if gen else "false") + ">")
    if not name.startswith("ag::k_simulate<"):
        return False
    args = name[len("ag::k_simulate<"):name.index(">")].split(", ")
    p8 = "_p8" in key
    is_gen = len(args) >= 8 and args[7] == "true"
    return args[0] == ("8" if p8 else "2") and is_gen == gen


def main():
    src = sys.argv[1]
    w = csv.writer(sys.stdout)
    w.writerow(["workload_trace", "bench_line", "kernel", "calls", "trace_avg_us", "trace_min_us", "trace_max_us",
                "bench_kernel_us", "trace_avg_over_bench"])
    for wl, keys in LINES.items():
        d = os.path.join(src, f"tr_{wl}")
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not stats or not os.path.exists(d + ".log"):
            continue
        res = bench_line(d + ".log")
        rows = list(csv.DictReader(open(stats[0])))
        for key in keys:
            ms = line_ms(res, key)
            for r in rows:
                name = r["Name"]
                if kernel_of(name, key):
                    avg = float(r["AverageNs"]) / 1e3
                    w.writerow([wl, key, re.sub(r"\(.*", "", name).replace("void ", ""), r["Calls"], f"{avg:.2f}",
                                f"{float(r['MinNs']) / 1e3:.2f}", f"{float(r['MaxNs']) / 1e3:.2f}",
                                "" if ms is None else f"{ms * 1e3:.2f}",
                                "" if ms is None else f"{avg / (ms * 1e3):.3f}"])


if __name__ == "__main__":
    main()

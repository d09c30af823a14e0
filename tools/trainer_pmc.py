#!/usr/bin/env python3
"""Trainer PMC summary: merges rocprofv3 --pmc passes (T1: instruction mix, T2: cycles / waits,
T3: integer / branch mix) of k_bidder_train<0/1> and k_lrts_train into per-kernel figures --
VALU instructions per BCE row (win-rate fit), fraction of wave cycles issuing VALU / waiting,
effective clock, and the VALU-issue roofline fraction: wave-level VALU instructions x 4 cycles
(a wave64 VALU op occupies a 16-lane SIMD for 4 cycles; FP64 FMA at full rate on CDNA4) over
1024 SIMDs at the measured clock, divided by the dispatch's duration.

    python tools/trainer_pmc.py out.json pass_dir [pass_dir ...]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for x in csv.DictReader(open(path)):
            m = re.search(r"(k_\w+<[^>]*>)", x["Kernel_Name"])
            k = m.group(1) if m else x["Kernel_Name"][:40]
            agg[k][x["Counter_Name"]] += float(x["Counter_Value"])
            dur[k] = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    return agg, dur


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    merged = collections.defaultdict(dict)
    durs = collections.defaultdict(list)
    for d in dirs:
        agg, dur = load(d)
        for k, v in agg.items():
            merged[k].update(v)
            durs[k].append(dur[k])
    res = {}
    for k, v in merged.items():
        ms = sum(durs[k]) / len(durs[k])
        r = {"ms_mean_over_passes": ms, "counters": v}
        if "SQ_WAVE_CYCLES" in v and "GRBM_GUI_ACTIVE" in v:
            wc = v["SQ_WAVE_CYCLES"]
            clk = v["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3)
            r.update(clock_ghz=clk / 1e9, valu_active_frac=v["SQ_ACTIVE_INST_VALU"] / wc,
                     wait_any_frac=v["SQ_WAIT_ANY"] / wc, wait_inst_any_frac=v["SQ_WAIT_INST_ANY"] / wc)
            if "SQ_INSTS_VALU" in v:
                t = v["SQ_INSTS_VALU"] * 4 / (1024 * clk)
                r.update(valu_issue_ms=t * 1e3, valu_roofline_frac=t / (ms * 1e-3))
        res[k] = r
        print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in r.items() if a != "counters"})
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

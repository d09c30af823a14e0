#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a tools/prof_r04.sh run: HBM bytes per launch =
FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024 (gfx950 corrections, MI355X_MICROARCH.md), mean over
the dispatches, for the headline kernel and the general kernel of every population line,
with the ratio to the bench line's algorithmic bytes (bench_driver.log of the same run).
    python tools/make_pmc_traffic.py gpurun_out/prof_<tag> <tag>"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import pmc  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d, tag = sys.argv[1], sys.argv[2]
    bench = None
    for ln in open(os.path.join(d, "bench_driver.log")):
        if ln.startswith("{"):
            bench = json.loads(ln)
    out = {}

    def traffic(fetch, write):
        f, nf = pmc(os.path.join(d, fetch))
        w, nw = pmc(os.path.join(d, write))
        if not f or not w:
            return None, 0
        return f["FETCH_SIZE"] * 2 * 1024 + w["WRITE_SIZE"] * 1024, min(nf, nw)

    def step_counter(path, name, P):
        """(mean per step of the counter summed over the step's kernels -- those of P
        participants: a pass's command may run other lines too --, steps, kernel names)"""
        fs = glob.glob(os.path.join(d, path, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            return None, 0, []
        per, kern = collections.OrderedDict(), {}
        for r in csv.DictReader(open(fs[0])):
            if r["Counter_Name"] == name and re.search(rf"<{P}, ", r["Kernel_Name"]):
                i = int(r["Dispatch_Id"])
                per[i] = per.get(i, 0.0) + float(r["Counter_Value"])
                kern[i] = r["Kernel_Name"]
        names = sorted(set(kern.values()))
        ids = sorted(per)[len(names):]  # the first step dropped
        steps = len(ids) / len(names)
        return sum(per[i] for i in ids) / steps, int(steps), names

    def step_traffic(fetch, write, P):
        f, nf, names = step_counter(fetch, "FETCH_SIZE", P)
        w, nw, _ = step_counter(write, "WRITE_SIZE", P)
        if f is None or w is None:
            return None, 0, []
        return f * 2 * 1024 + w * 1024, min(nf, nw), [n.split("(")[0] for n in names]

    head_dir = os.environ.get("HEAD_DIR")  # the headline passes of another run (same build)
    if head_dir:
        d_pop, d = d, head_dir
    t, n = traffic("fetch", "write")
    if head_dir:
        d = d_pop
    B = bench["config"]["auctions_per_gpu_per_step"]
    if t is None:  # no headline pass in this run (k_oracle unchanged): keep the committed one
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            prev = json.load(f)
        out.update({k: prev[k] for k in ("batch", "hbm_bytes_per_launch", "source", "over_algorithmic")})
    else:
        out.update({"batch": B, "hbm_bytes_per_launch": t,
                    "source": f"profiles/{tag}_pmc_summary.json (k_oracle<2,6,false>, FETCH_SIZE*2*1024 + "
                              f"WRITE_SIZE*1024, mean over {n} dispatches of {B} auctions)",
                    "over_algorithmic": t / (bench["roofline"]["algorithmic_bytes_per_auction"] * B)})
    for c in ("1", "2", "3", "4", "1p8", "4p8"):
        key = f"configs_{c[0]}" + ("_p8" if c.endswith("p8") else "")
        t, n, names = step_traffic(f"c{c}_fetch", f"c{c}_write", 8 if c.endswith("p8") else 2)
        if t is None or key not in bench:
            continue
        b = bench[key]["auctions_per_gpu_per_step"]
        out[key] = {"batch": b, "hbm_bytes_per_launch": t,
                    "source": f"profiles/{tag}_pmc_summary.json (FETCH_SIZE*2*1024 + WRITE_SIZE*1024 summed over "
                              f"the step's kernels {names}; mean over {n} steps, the first dropped)",
                    "over_algorithmic": t / (bench[key]["algorithmic_bytes_per_auction"] * b)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a tracked PMC summary (tools/summarize_pmc.py output): per
bench line, the HBM bytes per launch of its simulate kernel (FETCH_SIZE x 2 x 1024 +
WRITE_SIZE x 1024, per-dispatch means) and the ratio to the line's algorithmic bytes. Every
figure is read from the summary it names (workload -> kernel), so it can be recomputed from it.

    python tools/make_pmc_traffic.py profiles/<tag>_pmc_summary.json > profiles/pmc_traffic.json
"""
import json
import sys


def main():
    path = sys.argv[1]
    with open(path) as f:
        summ = json.load(f)
    out = {}
    for wl, ent in summ.items():
        # the workload's simulate kernel: k_oracle for the headline, k_simulate for the populations
        ks = [k for k, v in ent["kernels"].items() if "hbm_bytes_per_launch" in v and
              ("k_oracle" in k or "k_simulate" in k)]
        if len(ks) != 1:
            continue
        k = ks[0]
        v = ent["kernels"][k]
        rec = {"batch": ent["batch"], "hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
               "algorithmic_bytes_per_launch": v.get("algorithmic_bytes_per_launch"),
               "over_algorithmic": v.get("hbm_over_algorithmic"),
               "kernel": k.split("(")[0],
               "source": f"{path}: [{wl!r}]['kernels'][{k.split('(')[0]!r}...]['hbm_bytes_per_launch'] "
                         f"({v['hbm_bytes_formula']}; fetch pass {v['passes']['fetch']['dispatches']} dispatches, "
                         f"write pass {v['passes']['write']['dispatches']})"}
        if ent["bench_key"] == "headline":
            out.update(rec)
        else:
            out[ent["bench_key"]] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

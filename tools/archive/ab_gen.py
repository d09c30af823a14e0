#!/usr/bin/env python3
"""Generate mode (ag_simulate_generated, the headline workload with its inputs drawn on the chip)
at 4 / 5 / 6 workgroups per CU of the Oracle kernel's persistent grid, in one process; outputs
checked equal. Diagnostic only.   python tools/archive/ab_gen.py [B]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import HEADLINE_FIELDS, AuctionEngine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 27
    items, values = bench.catalogue()
    eng = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    out = eng.alloc_outputs(B, HEADLINE_FIELDS)
    ref = eng.alloc_outputs(B, HEADLINE_FIELDS)
    cnt = eng.new_counters()
    eng.simulate_generated(0, 0, ref, cnt)
    st = torch.cuda.current_stream()
    t = {}
    for _ in range(3):
        for bpc in (4, 5, 6, 8):
            eng.set_blocks_per_cu(bpc)
            for _ in range(3):
                eng.simulate_generated(0, 0, out, cnt)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(10):
                cnt.zero_()
                eng.simulate_generated(0, 0, out, cnt)
            b.record(st)
            torch.cuda.synchronize()
            t.setdefault(bpc, []).append(a.elapsed_time(b) / 10)
            assert all(torch.equal(out[k], ref[k]) for k in out), bpc
    for bpc, v in t.items():
        ms = float(np.median(v))
        print(f"generate mode, {bpc} workgroups/CU: {ms:.4f} ms  {84 * B / ms / 1e6:.0f} GB/s written = "
              f"{84 * B / ms / 1e6 / 8000:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()

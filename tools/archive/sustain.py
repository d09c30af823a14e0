"""Per-launch k_simulate durations over a long back-to-back run (clock / power drift check)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine  # noqa: E402

B = 1 << 24
items, values = bench.catalogue()
e = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
e.load_catalog(items, values)
inp = e.alloc_inputs(B)
e.generate(0, 0, inp)
out = e.alloc_outputs(B, ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev"))
cnt = e.new_counters()
st = torch.cuda.current_stream()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record(st)
for i in range(n):
    ev[i][0].record(st)
    e.simulate(inp, out)  # no counters: k_simulate only
    ev[i][1].record(st)
t1.record(st)
torch.cuda.synchronize()
d = np.array([a.elapsed_time(b) for a, b in ev])
print("total ms/launch incl. gaps", t0.elapsed_time(t1) / n)
for j in range(0, n, n // 10):
    print(f"launches {j:4d}-{j + n // 10 - 1:4d}: mean {d[j:j + n // 10].mean():.4f} ms  min {d[j:j + n // 10].min():.4f}")
# with idle gaps of 2 ms between launches
g = []
for i in range(30):
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e6))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    e.simulate(inp, out)
    b.record(st)
    torch.cuda.synchronize()
    g.append(a.elapsed_time(b))
print("with idle gaps: mean", np.mean(g[3:]), "min", np.min(g))

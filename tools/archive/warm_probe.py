"""Why are the first ~40 k_simulate launches of a fresh process slower? Per-launch durations
of the headline step (ag_simulate with counters) under three conditions:
  A. fresh process, buffers just written by ag_generate (the bench's situation);
  B. after a 1 s idle gap (clock / power-state ramp shows up again here);
  C. on freshly allocated output buffers, GPU already warm (first-touch / TLB shows up here);
  D. after 60 ms of an unrelated streaming kernel (torch copy) -- clocks warm, our buffers cold.
Also prints the measured copy bandwidth (read + write bytes / time) of a 4 GiB torch copy."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
FIELDS = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
items, values = bench.catalogue()
e = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
e.load_catalog(items, values)
inp = e.alloc_inputs(B)
e.generate(0, 0, inp)
out = e.alloc_outputs(B, FIELDS)
cnt = e.new_counters()
st = torch.cuda.current_stream()
torch.cuda.synchronize()


def run(n, o=None):
    o = o or out
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        cnt.zero_()
        ev[i][0].record(st)
        e.simulate(inp, o, cnt)
        ev[i][1].record(st)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in ev])


def show(tag, d):
    blocks = [d[j:j + 10] for j in range(0, len(d), 10)]
    print(f"{tag}: " + " ".join(f"{b.mean():.3f}" for b in blocks), flush=True)


show("A fresh process (per 10 launches)", run(120))
time.sleep(1.0)
show("B after 1 s idle", run(60))
out2 = e.alloc_outputs(B, FIELDS)
show("C fresh outputs, warm GPU", run(60, out2))
del out2
time.sleep(1.0)
x = torch.empty(1 << 29, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
x.fill_(1.0)
torch.cuda.synchronize()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.06:
    y.copy_(x)
torch.cuda.synchronize()
show("D after 60 ms of torch copy", run(60))
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    y.copy_(x)
a.record(st)
for _ in range(20):
    y.copy_(x)
b.record(st)
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 20
print(f"copy 4 GiB -> 4 GiB: {ms:.3f} ms, {2 * x.numel() * 8 / ms / 1e6:.0f} GB/s (read + write)")

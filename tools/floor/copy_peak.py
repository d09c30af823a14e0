"""Copy-kernel variants for the measured HBM peak (diagnostic): 4 GiB -> 4 GiB, 16 B per lane."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
from auctiongym_amd.engine import stream_copy  # noqa: E402

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfloor.so"))
L.copy_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
n = 1 << 32
src = torch.ones(n // 8, dtype=torch.float64, device="cuda")
dst = torch.empty_like(src)
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)
cus = torch.cuda.get_device_properties(0).multi_processor_count
runs = {"ag_stream_copy": lambda: stream_copy(src, dst), "torch copy_": lambda: dst.copy_(src)}
for g in (4, 8, 16):
    runs[f"persistent plain {g}/CU"] = lambda g=g: L.copy_run(0, cus * g, src.data_ptr(), dst.data_ptr(), n, sp)
    runs[f"persistent nt {g}/CU"] = lambda g=g: L.copy_run(1, cus * g, src.data_ptr(), dst.data_ptr(), n, sp)
runs["tiles plain"] = lambda: L.copy_run(2, 0, src.data_ptr(), dst.data_ptr(), n, sp)
runs["tiles nt"] = lambda: L.copy_run(3, 0, src.data_ptr(), dst.data_ptr(), n, sp)
for _ in range(5):
    for f in runs.values():
        f()
torch.cuda.synchronize()
res = {k: [] for k in runs}
for r in range(5):
    for k, f in runs.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(10):
            f()
        b.record(st)
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) / 10)
for k, t in res.items():
    ms = float(np.median(t))
    print(f"{k:28s} {ms:.3f} ms  {2 * n / ms / 1e6:.0f} GB/s")

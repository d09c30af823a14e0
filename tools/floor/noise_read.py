"""Noise-read floor (tools/floor/noise_read.hip): the SP_Truthful_TS batch's Thompson noise
(2^20 auctions x 2 slots x 60 floats = 503 MB) read in the tile layout (dword rows) vs quad
tiles (16-B loads), grids of 4 / 8 / 16 workgroups per CU. Diagnostic only.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/floor/libnoise.so tools/floor/noise_read.hip"""
import ctypes
import os

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnoise.so"))
L.noise_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
tiles = 2 * (1 << 20) // 64
nz = torch.randn(tiles * 60 * 64, device="cuda")
out = torch.empty(tiles * 64, device="cuda")
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)
cus = torch.cuda.get_device_properties(0).multi_processor_count
names = {0: "rows, 20 loads per group", 1: "rows, 60 loads at once", 4: "rows, 4 loads per group",
         2: "quads, 5 x 16-B per group", 3: "quads, 15 x 16-B at once", 5: "quads, one 16-B at a time"}
runs = {f"{names[v]}, {g}/CU": (v, g) for v in (4, 0, 1, 5, 2, 3) for g in (4, 8, 16)}
for _ in range(20):
    for v, g in runs.values():
        L.noise_run(v, cus * g, nz.data_ptr(), tiles, out.data_ptr(), sp)
torch.cuda.synchronize()
t = {k: [] for k in runs}
for r in range(10):
    for k, (v, g) in runs.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(10):
            L.noise_run(v, cus * g, nz.data_ptr(), tiles, out.data_ptr(), sp)
        b.record(st)
        torch.cuda.synchronize()
        t[k].append(a.elapsed_time(b) / 10)
nbytes = nz.numel() * 4
for k in runs:
    ms = float(np.median(t[k]))
    print(f"{k:40s} {ms:.4f} ms  {nbytes / ms / 1e9:.2f} TB/s", flush=True)

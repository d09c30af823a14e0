"""Streaming floor of the SP_Oracle byte pattern (tools/floor/stream_floor.hip) next to
ag_simulate on the same buffers: HIP events on the launch stream, isolated and back to back.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/floor/libfloor.so tools/floor/stream_floor.hip"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine  # noqa: E402


class Ptrs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("ctx", "part", "u", "winner", "item", "price", "bid", "est",
                                              "tru", "bev", "outcome")]


def main():
    L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfloor.so"))
    L.floor_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Ptrs), ctypes.c_int64, ctypes.c_void_p]
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 27
    items, values = bench.catalogue()
    eng = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    full = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    out = eng.alloc_outputs(B, full)
    cnt = eng.new_counters()
    from auctiongym_amd.engine import HEADLINE_FIELDS
    outw = eng.alloc_outputs(B, HEADLINE_FIELDS)
    P = lambda t: t.data_ptr()  # noqa: E731
    p = Ptrs(P(inp["ctx"]), P(inp["part"]), P(inp["u"]), P(out["winner"]), P(out["item"]), P(out["price"]),
             P(out["bid"]), P(out["est_ctr"]), P(out["true_ctr"]), P(out["best_ev"]), P(out["outcome"]))
    pw = Ptrs(P(inp["ctx"]), P(inp["part"]), P(inp["u"]), P(outw["winner_outcome"]), P(outw["item"]),
              P(outw["price"]), P(outw["bid"]), P(outw["est_ctr"]), P(outw["true_ctr"]), P(outw["best_ev"]), None)
    L.floor_queue.argtypes = [ctypes.c_int, ctypes.POINTER(Ptrs), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    L.floor_chunk.argtypes = [ctypes.c_int, ctypes.POINTER(Ptrs), ctypes.c_int64, ctypes.c_void_p]
    qbuf = torch.zeros(8 * 32, dtype=torch.int32, device="cuda")
    qc = ctypes.c_void_p(qbuf.data_ptr())
    tin = torch.zeros(7 * B, dtype=torch.float64, device="cuda")      # 56 B per auction, tiled
    tout = torch.empty(84 * B // 8, dtype=torch.float64, device="cuda")  # 84 B per auction, tiled
    p2 = Ptrs(P(tin), P(inp["part"]), P(inp["u"]), P(out["winner"]), P(out["item"]), P(tout),
              P(out["bid"]), P(out["est_ctr"]), P(out["true_ctr"]), P(out["best_ev"]), P(out["outcome"]))
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    runs = {
        "floor persistent 8 blocks/CU": lambda: L.floor_run(1, cus * 8, ctypes.byref(p), B, sp),
        "floor persistent 4 blocks/CU": lambda: L.floor_run(1, cus * 4, ctypes.byref(p), B, sp),
        "floor persistent nt 8 blocks/CU": lambda: L.floor_run(2, cus * 8, ctypes.byref(p), B, sp),
        "floor w2 nt 8 blocks/CU": lambda: L.floor_run(3, cus * 8, ctypes.byref(p), B, sp),
        "floor w2 nt 4 blocks/CU": lambda: L.floor_run(3, cus * 4, ctypes.byref(p), B, sp),
        "floor one tile per block": lambda: L.floor_run(0, 0, ctypes.byref(p), B, sp),
        "floor nt 4/CU, winner|outcome word": lambda: L.floor_run(4, cus * 4, ctypes.byref(p), B, sp),
        "floor nt 8/CU, winner|outcome word": lambda: L.floor_run(4, cus * 8, ctypes.byref(p), B, sp),
        "floor nt 4/CU, tiled inputs": lambda: L.floor_run(5, cus * 4, ctypes.byref(p2), B, sp),
        "floor nt 4/CU, tiled outputs": lambda: L.floor_run(6, cus * 4, ctypes.byref(p2), B, sp),
        "floor nt 4/CU, tiled in + out": lambda: L.floor_run(7, cus * 4, ctypes.byref(p2), B, sp),
        "floor nt 8/CU, tiled in + out": lambda: L.floor_run(7, cus * 8, ctypes.byref(p2), B, sp),
        "floor nt 4/CU, 16-B tiles in + out": lambda: L.floor_run(8, cus * 4, ctypes.byref(p2), B, sp),
        "floor nt 8/CU, 16-B tiles in + out": lambda: L.floor_run(8, cus * 8, ctypes.byref(p2), B, sp),
        "floor nt one tile per block, word": lambda: L.floor_run(9, 0, ctypes.byref(pw), B, sp),
        "floor nt 4/CU work queue, word": lambda: L.floor_queue(cus * 4, ctypes.byref(pw), B, qc, sp),
        "floor nt 2 tiles per block, word": lambda: L.floor_chunk(2, ctypes.byref(pw), B, sp),
        "floor nt 4 tiles per block, word": lambda: L.floor_chunk(4, ctypes.byref(pw), B, sp),
        "floor nt 8 tiles per block, word": lambda: L.floor_chunk(8, ctypes.byref(pw), B, sp),
        "floor nt 16 tiles per block, word": lambda: L.floor_chunk(16, ctypes.byref(pw), B, sp),
        "floor nt 64 tiles per block, word": lambda: L.floor_chunk(64, ctypes.byref(pw), B, sp),
        "floor nt 8/CU work queue, word": lambda: L.floor_queue(cus * 8, ctypes.byref(pw), B, qc, sp),
        "ag_simulate (r04 fields)": lambda: eng.simulate(inp, out, cnt),
        "ag_simulate (bench: winner|outcome)": lambda: eng.simulate(inp, outw, cnt),
        "ag_simulate, no counters": lambda: eng.simulate(inp, out, None),
        "torch copy+fill of the same bytes": None,
    }
    src = torch.empty(56 * B // 8, dtype=torch.float64, device="cuda")
    dst = torch.empty(56 * B // 8, dtype=torch.float64, device="cuda")
    fill = torch.empty(29 * B // 8, dtype=torch.float64, device="cuda")
    runs["torch copy+fill of the same bytes"] = lambda: (dst.copy_(src), fill.fill_(1.0))
    from auctiongym_amd.engine import stream_copy
    big = torch.empty(141 * B // 16, dtype=torch.float64, device="cuda")  # 141 B per auction moved
    big2 = torch.empty_like(big)
    runs["ag_stream_copy of 141 B/auction (read+write)"] = lambda: stream_copy(big, big2)
    for _ in range(max(5, (200 << 24) // B)):
        for f in runs.values():
            f()
    torch.cuda.synchronize()
    iso = {k: [] for k in runs}
    sus = {k: [] for k in runs}
    for r in range(12 if B <= 1 << 24 else 4):
        for k, f in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            f()
            b.record(st)
            torch.cuda.synchronize()
            iso[k].append(a.elapsed_time(b))
            a.record(st)
            for _ in range(10):
                f()
            b.record(st)
            torch.cuda.synchronize()
            sus[k].append(a.elapsed_time(b) / 10)
    for k in runs:
        mi, ms = float(np.median(iso[k])), float(np.median(sus[k]))
        print(f"{k:36s} isolated {mi:7.4f} ms ({141 * B / (mi * 1e-3) / 1e12:7.2f} TB/s)   back-to-back {ms:7.4f} ms "
              f"({141 * B / (ms * 1e-3) / 1e12:7.2f} TB/s)")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""How the reference's third-party CPU arithmetic sums on THIS host, against the orders the
oracle pins (measured on the host that ran the reference for tests/golden/): numpy's
`items @ ctx` (OpenBLAS dgemv) vs ora_dot, torch's F.linear(x[5], W[K][5]) (MKL sgemv) vs
ora_ts_logit, torch.sigmoid on K < 32 elements vs ora_ts_sigmoid, and the win-rate model's
Linear(3, 1) vs the search bid's restated z. Prints one JSON line of agreement fractions.
Diagnostic (CPU only).    python tools/host_order_probe.py"""
import json
import os
import platform
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    L = O.lib()
    g = np.random.default_rng(0)
    res = {"cpu": platform.processor() or "", "torch_cpu_capability": torch.backends.cpu.get_cpu_capability()}
    try:
        res["cpu"] = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except (OSError, IndexError):
        pass
    # numpy dgemv (the Oracle CTR's dot), K = 12, D = 6
    ok = n = 0
    for _ in range(2000):
        items = g.normal(0, 1, (12, 6))
        x = np.concatenate([g.normal(0, 1, 5), [1.0]])
        ref = items @ x
        for k in range(12):
            ok += L.ora_dot(np.ascontiguousarray(items[k]).ctypes.data, x.ctypes.data, 6) == ref[k]
            n += 1
    res["numpy_dot_vs_ora_dot"] = ok / n
    # torch F.linear + sigmoid (the LR-TS forward), K = 12, Do = 5
    okz = okc = n = 0
    for _ in range(2000):
        W = g.normal(0, 1, (12, 5)).astype(np.float32)
        x = np.concatenate([g.normal(0, 1, 4), [1.0]]).astype(np.float32)
        z = F.linear(torch.from_numpy(x), torch.from_numpy(W))
        c = torch.sigmoid(z).numpy()
        z = z.numpy()
        for k in range(12):
            okz += np.float32(L.ora_ts_logit(W[k].ctypes.data, x.ctypes.data, 5, k, 12)) == z[k]
            okc += np.float32(L.ora_ts_sigmoid(float(z[k]), k, 12)) == c[k]
            n += 1
    res["torch_linear_vs_ora_ts_logit"] = okz / n
    res["torch_sigmoid_vs_ora_ts_sigmoid"] = okc / n
    # Linear(3, 1) on [128, 3] rows (the search bid's win-rate model)
    lin = torch.nn.Linear(3, 1)
    ok = n = 0
    for _ in range(200):
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(g.normal(0, 1, (1, 3)).astype(np.float32)))
            lin.bias.copy_(torch.from_numpy(g.normal(0, 1, 1).astype(np.float32)))
        X = g.uniform(0, 1, (128, 3)).astype(np.float32)
        with torch.no_grad():
            z = lin(torch.from_numpy(X)).numpy()[:, 0]
        w = lin.weight.detach().numpy()[0]
        b = lin.bias.detach().numpy()[0]
        c, v, gg = X[:, 0], X[:, 1], X[:, 2]
        cv = (v.astype(np.float64) * w[1] + (c * w[0]).astype(np.float32)).astype(np.float32)  # fma(v, w1, c w0)
        zz = ((cv + gg * w[2]).astype(np.float32) + b).astype(np.float32)
        ok += int(np.sum(zz == z))
        n += 128
    res["torch_linear3_vs_search_z"] = ok / n
    print(json.dumps(res))


if __name__ == "__main__":
    main()

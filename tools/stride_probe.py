"""Does the spacing of the Krylov basis vectors change MAXPY/MDot bandwidth?
Basis = one allocation, vectors `stride` doubles apart (stride = N + pad)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Vec

N = 256 ** 3
ctx = Context(0)
out = {}
for pad in [0, 512, 2048, 4096 + 512, 16384 + 256, 65536 + 1024, 3 * 65536 + 512]:
    stride = N + pad
    T = torch.empty(31 * stride + 1024, dtype=torch.float64, device="cuda")
    T.uniform_(-1, 1)
    base = T.data_ptr()
    V = [Vec(ctx, N, device_ptr=base + j * stride * 8) for j in range(30)]
    w = Vec(ctx, N, device_ptr=base + 30 * stride * 8)
    torch.cuda.synchronize()
    res = {}
    for k in (8, 30):
        for name, fn in (("maxpy", lambda: w.maxpy(np.full(k, 1e-300), V[:k])), ("mdot", lambda: w.mdot(V[:k]))):
            fn()
            ctx.reset_kernel_stats(); ctx.set_timing(True)
            for _ in range(10):
                fn()
            ctx.set_timing(False)
            s = ctx.kernel_stats()[name]
            res[f"{name}{k}"] = round(s["bytes"] / (s["ms"] * 1e-3) / 1e9)
    out[pad] = res
    del V, w, T
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))

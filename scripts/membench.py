#!/usr/bin/env python3
"""Reference HBM rates on this box for the config-3 buffer sizes (torch kernels):
fill of the 126 MB coefficient buffer, and copy of it."""
import json, torch
B, M = 65536, 10
n = B * M * 24
a = torch.empty(n, dtype=torch.float64, device="cuda"); b = torch.empty_like(a)
def t(fn, K=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K * 1e3
fill_us = t(lambda: a.fill_(1.0)); copy_us = t(lambda: b.copy_(a))
big = torch.empty(8 * n, dtype=torch.float64, device="cuda")
fill_big_us = t(lambda: big.fill_(1.0), 10)
print(json.dumps({"fill_126MB_us": fill_us, "fill_GBs": n * 8 / fill_us / 1e3, "copy_126MB_us": copy_us,
                  "copy_GBs": 2 * n * 8 / copy_us / 1e3, "fill_1GB_GBs": 8 * n * 8 / fill_big_us / 1e3}))

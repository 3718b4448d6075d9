"""Diagnostic: achievable HBM write / copy rates on this box for the decoder's
output size (10.19 GB): torch fill_ (a pure write stream) and a device copy."""
import json
import time

import torch

N = 10_188_726_152
x = torch.empty(N, dtype=torch.uint8, device="cuda")
y = torch.empty(N, dtype=torch.uint8, device="cuda")
res = {}
for name, fn in [("fill", lambda: x.fill_(7)), ("zero", lambda: x.zero_()), ("copy", lambda: y.copy_(x))]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    bytes_moved = N * (2 if name == "copy" else 1)
    res[name] = {"ms": round(ms, 4), "GB/s": round(bytes_moved / ms / 1e6, 1)}
print(json.dumps(res))

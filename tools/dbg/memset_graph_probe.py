"""Does a HIP graph replay a captured hipMemsetAsync?  (Diagnostic for the
round-3 graph-replay hang, ADVICE r3: k_encode_reset replaced the encoder's
two memsets on the assumption that replays skip them.)

Captures, on torch's capture stream: hipMemsetAsync(x, 0, 8) then a torch
kernel x += 1; replays the graph 3 times and prints x[0] after each.  x
starts at 5 (capture runs nothing): a replayed memset gives 1, 1, 1, a
skipped one 6, 7, 8.  Also memsets of 4 and 24 bytes (the sizes the line
index and the decoder use; a 4-byte memset zeroes only half of x[0], which
still reads 1 when replayed).  Run under `timeout`."""
import ctypes
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so.7")   # the soname torch already loaded: one HIP runtime
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int

for nbytes in (8, 4, 24):
    x = torch.full((4,), 5, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        rc = hip.hipMemsetAsync(x.data_ptr(), 0, nbytes, s)
        x.add_(1)
    torch.cuda.synchronize()
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(x.cpu().tolist())
    print("memset %2d bytes (rc %d): after replays %s -> %s" % (
        nbytes, rc, seen, "memset replayed" if all(v[0] == 1 for v in seen) else "memset NOT replayed"), flush=True)
sys.exit(0)

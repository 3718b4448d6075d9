"""Debug: decode_records_device on law-2 rows (GPU), print the error word."""
import os
import sys
import numpy as np
import torch
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "vcf-compression_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import vcfc
import workload
from test_gpu_encode import _device_encode

dev = torch.device("cuda:0")
for n, seed in [(12, 33), (3000, 33), (3000, 7), (20000, 33)]:
    rows = workload.DeviceRows(torch, vcfc, n, 2504, 2, seed=seed, device="cuda:0")
    out, rec, err = _device_encode(torch, vcfc, rows)
    rec_t = torch.from_numpy(rec.astype(np.int64)).to(dev)
    dws_bytes = vcfc.decode_workspace_size(n)
    dws = torch.empty(dws_bytes, dtype=torch.uint8, device=dev)
    cap = rows.total_bytes + 64
    lines = torch.empty(cap, dtype=torch.uint8, device=dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    derr = torch.empty(1, dtype=torch.int64, device=dev)
    for exact in (False, True):
        vcfc.decode_records_device(out.data_ptr(), int(rec[n]), rec_t.data_ptr(), n, 2504, lines.data_ptr(), cap,
                                   loff.data_ptr(), dws.data_ptr(), dws_bytes, derr.data_ptr(),
                                   torch.cuda.current_stream(dev).cuda_stream, exact=exact)
        torch.cuda.synchronize()
        e = int(derr.cpu().numpy().view(np.uint64)[0])
        k = e >> 8
        ok = e == vcfc.NO_ERROR and bool(torch.equal(lines[:rows.total_bytes], rows.buf[:rows.total_bytes]))
        print(n, seed, "exact" if exact else "light", hex(e), "ok" if ok else "BAD", flush=True)
        if e != vcfc.NO_ERROR and k < n:
            ln = rows.host_lines([k])[0]
            print("  record", k, "line len", len(ln), repr(ln[:120]), ln.count(b"\t"), "rec bytes", int(rec[k + 1] - rec[k]))
            print("  rec head", out[int(rec[k]):int(rec[k]) + 64].cpu().numpy().tobytes())
            print("  loff", loff[:4].cpu().tolist(), "dec head", lines[:120].cpu().numpy().tobytes())

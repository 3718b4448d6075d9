"""Diagnostic: per-row start/end wall clock of k_encode_fast (a library built
with the tools/diag/row_times.h hooks, picked by VCFC_LIB), and what a decoupled look-back
over row sizes would have to wait for: row i's output offset is known once
every row < i has finished, i.e. at max(end[0..i]).

  VCFC_LIB=build_rt/libvcfc.so python tools/row_times.py [--law 1] [--rows 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "vcf-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--law", type=int, default=1)
    ap.add_argument("--rows", type=int, default=1000000)
    ap.add_argument("--samples", type=int, default=2504)
    ap.add_argument("--out", default=os.path.join(R, "gpurun_out", "row_times.json"))
    a = ap.parse_args()
    import torch
    import vcfc
    import workload
    dev = "cuda:0"
    n = a.rows
    rows = workload.DeviceRows(torch, vcfc, n, a.samples, a.law, seed=1000, device=dev)
    ws_bytes = vcfc.workspace_size(n, rows.line_bytes)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
    recs = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    res = {}
    for it in range(4):
        vcfc.encode_rows_device(rows.buf.data_ptr(), rows.line_off.data_ptr(), rows.line_len.data_ptr(), n,
                                rows.line_bytes, recs.data_ptr(), cap, rec.data_ptr(), ws.data_ptr(), ws_bytes,
                                err.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    t = ws[ws_bytes - 16 * n:].view(torch.int64).cpu().numpy().reshape(n, 2).astype(np.float64)
    t -= t[:, 0].min()
    t *= 0.01   # 100 MHz -> us
    st, en = t[:, 0], t[:, 1]
    dur = en - st
    ready = np.maximum.accumulate(en)
    wait = ready - en
    rs = np.diff(rec.cpu().numpy())
    q = [50, 90, 99, 99.9]
    res["kernel_us"] = float(en.max())
    res["row_us_pct"] = {str(p): float(np.percentile(dur, p)) for p in q}
    res["row_us_mean"] = float(dur.mean())
    res["wait_us_pct"] = {str(p): float(np.percentile(wait, p)) for p in [25, 50, 75, 90, 99]}
    res["wait_us_mean"] = float(wait.mean())
    res["wait_over_row"] = float(wait.sum() / dur.sum())
    res["start_inversions"] = float(np.mean(np.diff(st) < 0))
    res["frac_ready_within_us"] = {str(b): float(np.mean(wait <= b)) for b in [0, 0.5, 1, 2, 4, 8]}
    res["record_bytes_pct"] = {str(p): float(np.percentile(rs, p)) for p in [50, 90, 99, 99.9, 100]}
    res["frac_records_le"] = {str(b): float(np.mean(rs <= b)) for b in [1024, 2048, 3072, 4096]}
    print(json.dumps(res))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()

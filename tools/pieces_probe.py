"""Diagnostic: does splitting the headline batch into P sequential pieces
(encode -> size scan -> compaction per piece, one stream) keep a piece's
staging in the MALL for its compaction?  Per-stage HIP-event times summed
over the pieces of a step (vcfc_encode_rows_device_timed), P = 1 .. 32.
Each piece writes its records to its own region of `out` (not a product
layout; the time is the question).

  python tools/pieces_probe.py [--law 1] [--steps 10]
"""
import argparse
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "vcf-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--law", type=int, default=1)
    ap.add_argument("--rows", type=int, default=1000000)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    import vcfc
    import workload
    dev = torch.device("cuda:0")
    n = a.rows
    rows = workload.DeviceRows(torch, vcfc, n, 2504, a.law, seed=1000, device=dev)
    lens = rows.line_len_host.astype(np.int64)
    cap = vcfc.encode_bound(n, rows.line_bytes)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    rec = torch.empty(n + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for P in (1, 2, 4, 8, 16, 32):
        cuts = [n * k // P for k in range(P + 1)]
        pbytes = [int(lens[cuts[k]:cuts[k + 1]].sum()) for k in range(P)]
        ws_bytes = max(vcfc.workspace_size(cuts[k + 1] - cuts[k], pbytes[k]) for k in range(P))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        obase = [0]
        for k in range(P):
            obase.append(obase[-1] + vcfc.encode_bound(cuts[k + 1] - cuts[k], pbytes[k]))
        assert obase[-1] <= cap + 64 * P
        timer = vcfc.StageTimer()

        def step(f):
            for k in range(P):
                r0, m = cuts[k], cuts[k + 1] - cuts[k]
                f(rows.buf.data_ptr(), rows.line_off.data_ptr() + 8 * r0, rows.line_len.data_ptr() + 4 * r0, m,
                  pbytes[k], out.data_ptr() + obase[k], obase[k + 1] - obase[k], rec.data_ptr() + 8 * r0,
                  ws.data_ptr(), ws_bytes, err.data_ptr(), stream)

        for _ in range(3):
            step(vcfc.encode_rows_device)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step(timer.encode)
        e1.record()
        torch.cuda.synchronize()
        st, calls = timer.read()
        assert int(err.item()) == -1
        res[P] = {"step_ms": round(e0.elapsed_time(e1) / a.steps, 4),
                  "stages_ms_per_step": {k: round(v * P / max(calls, 1), 4) for k, v in st.items()}}
        print(P, json.dumps(res[P]), flush=True)
        del ws
    os.makedirs(os.path.join(R, "gpurun_out"), exist_ok=True)
    with open(os.path.join(R, "gpurun_out", "pieces_law%d.json" % a.law), "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()

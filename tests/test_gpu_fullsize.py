"""Full-size GPU parity (BASELINE configs[1]/[2] and [4]: 2504 samples x 1M
variants): EVERY record of the batch against the oracle, for both synthetic
laws (law 0 = the reference generator's random_vcf law,
other/random_vcf.py:66-70; law 1 = chr22-shaped; law 2 = general shapes,
SURVEY §8(d) D3: haploid, GT:DP:GQ, missing), plus the decode round trip
of the same batch (reference compress_data_line src/compress.cpp:5-203 and
decompress2_data_line :741-986).

The records stay in HBM: the GPU digests each record in place
(vcfc_record_hash_device) and the oracle digests its own encode of the same
rows on the host's cores (vcfo_encode_rows_hash, threaded), so 8 bytes per
row are compared instead of ~1 GB of records.  Sizes are compared exactly."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu
REPO = G.REPO


@pytest.fixture(scope="module")
def torch():
    import torch as T   # before libvcfc: one HIP runtime in the process
    assert T.cuda.is_available(), "GPU tests need a GPU"
    return T


@pytest.fixture(scope="module")
def vcfc(torch):
    import sys
    sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))
    import vcfc as V
    return V


def threads():
    return int(os.environ.get("OMP_NUM_THREADS", "16") or 16)


@pytest.mark.parametrize("law", [1, 0, 2])
def test_full_batch_every_record_and_round_trip(torch, vcfc, law):
    import workload
    from test_gpu_encode import _device_encode
    n, S = 1_000_000, 2504
    dev = torch.device("cuda:0")
    rows = workload.DeviceRows(torch, vcfc, n, S, law, seed=31 + law, device="cuda:0")
    out, rec, err = _device_encode(torch, vcfc, rows)
    assert err == vcfc.NO_ERROR
    rec_t = torch.from_numpy(rec.astype(np.int64)).to(dev)
    h = torch.empty(n, dtype=torch.int64, device=dev)
    vcfc.record_hash_device(out.data_ptr(), rec_t.data_ptr(), n, h.data_ptr(),
                            torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    got_h = h.cpu().numpy().view(np.uint64)
    # the oracle's encode of every row, on the host
    buf = rows.buf[:rows.total_bytes].cpu().numpy()
    st, size, want_h = G.oracle_encode_rows_hash(buf, rows.line_off.cpu().numpy(), rows.line_len.cpu().numpy(),
                                                 threads=threads())
    assert (st == 0).all()
    sizes = np.diff(rec)
    bad = np.nonzero((size.astype(np.uint64) != sizes) | (want_h != got_h))[0]
    assert bad.size == 0, "rows differ from the oracle: %s" % bad[:10].tolist()
    # decode round trip of the same batch, on the GPU
    del buf
    dws_bytes = vcfc.decode_workspace_size(n)
    dws = torch.empty(dws_bytes, dtype=torch.uint8, device=dev)
    cap = rows.total_bytes + 64
    lines = torch.empty(cap, dtype=torch.uint8, device=dev)
    loff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    derr = torch.empty(1, dtype=torch.int64, device=dev)
    for exact in (False, True):   # the light plan assumes 3-byte tokens; code 4 = plan again exactly
        vcfc.decode_records_device(out.data_ptr(), int(rec[n]), rec_t.data_ptr(), n, S, lines.data_ptr(), cap,
                                   loff.data_ptr(), dws.data_ptr(), dws_bytes, derr.data_ptr(),
                                   torch.cuda.current_stream(dev).cuda_stream, exact=exact)
        torch.cuda.synchronize(dev)
        e = int(derr.cpu().numpy().view(np.uint64)[0])
        if e == vcfc.NO_ERROR or (e & 0xFF) != 4:
            break
    assert e == vcfc.NO_ERROR, hex(e)
    assert int(loff[n].item()) == rows.total_bytes
    assert bool(torch.equal(lines[:rows.total_bytes], rows.buf[:rows.total_bytes]))

"""k_sparse_plan (csrc/vcfc_sparse.hip) on the CPU emulator: the planned
offsets/prefixes, applied with the reference's write order, reproduce the
reference's sparse file (hole-aware digest)."""
import os
import struct
import tempfile

import numpy as np
import pytest

import emu_io as E
import golden_io as G
import sparse_digest


def header_end(v):
    p = 0
    while v[p:p + 1] == b"#":
        p = v.index(b"\n", p) + 1
    return p


def rec_index(body):
    ro, p = [], 0
    while len(body) - p >= 8:
        L = ((body[p] & 0x3F) << 24) | (body[p + 1] << 16) | (body[p + 2] << 8) | body[p + 3]
        ro.append(p)
        p += 8 + L - 4
    ro.append(p)
    return ro


def materialise(v, path):
    h = header_end(v)
    body = v[h:]
    ro = rec_index(body)
    data_start = h + 8
    fo, pf, st = E.emu_sparse_plan(body, ro, data_start)
    assert st[0] == (1 << 64) - 1
    replay = bool(st[1] != 0)
    n = len(ro) - 1
    fd = os.open(path, os.O_CREAT | os.O_TRUNC | os.O_RDWR, 0o600)
    os.pwrite(fd, v[:h] + b"\0" * 8, 0)
    for i in range(n):
        pre = bytearray(pf[16 * i:16 * i + 16])
        if i == 0:
            os.pwrite(fd, struct.pack("<Q", (int(fo[0]) - data_start) & (2**64 - 1)), data_start - 8)
        elif replay:
            os.pwrite(fd, struct.pack(">Q", (int(fo[i]) - int(fo[i - 1])) & (2**64 - 1)), int(fo[i - 1]) + 8)
        if replay:
            pre[8:16] = b"\0" * 8
        os.pwrite(fd, bytes(pre) + body[ro[i]:ro[i + 1]], int(fo[i]))
    os.close(fd)
    return replay


def test_plan_random_100x10000():
    v = G.gz("random_100x10000.vcfc.gz")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "o.sparse")
        assert materialise(v, p) is False
        assert sparse_digest.digest(p) == G.manifest()["sparse_100x10000"]


def test_plan_edge_overlap_replay():
    v = G.gz("sparse_edge.vcfc.gz")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "o.sparse")
        assert materialise(v, p) is True
        assert sparse_digest.digest(p) == G.manifest()["sparse_edge"]


def test_sparse_query_driver_matches_oracle_and_reference():
    """vcfc_dec::sparse_query (product driver + decode kernels, emulated) on
    every golden sparse-query case: byte-identical to the oracle restatement
    (including every line before a throw) and consistent with the reference
    CLI's recorded stdout / exit status."""
    d = G.sparse_query_cases()
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        built = set()
        for c in d["cases"]:
            path = os.path.join(wd, c["file"] + ".sparse")
            if c["file"] not in built:
                G.build_sparse_file(d, c["file"], path, G.oracle_sparsify)
                built.add(c["file"])
            q = c["query"].encode()
            want = G.oracle_sparse_query(path, q)
            ref, hr, a, b = G.oracle_parse_query(q)
            got = E.emu_sparse_query(path, ref, hr, a, b)
            assert got == want, (c, got[0], want[0], len(got[1]), len(want[1]))
            assert G.check_sparse_case(c, *got), c


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_sparse_query_driver_on_mutated_files(seed):
    """Random byte patches in the distance prefixes, record headers and
    bodies of a sparse file (walk errors, off-hop parses, bad POS fields):
    the product driver against the oracle restatement."""
    import random
    rnd = random.Random(seed)
    d = G.sparse_query_cases()
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        path = os.path.join(wd, "m.sparse")
        G.build_sparse_file(d, "random_100x10000", path, G.oracle_sparsify)
        v = G.gz("random_100x10000.vcfc.gz")
        ds = header_end(v) + 8
        with open(path, "r+b") as f:
            for _ in range(6):
                k = rnd.randrange(0, 60)
                slot = ds + (300000000 + 10000 + 2 * k) * 16384
                off = slot + rnd.choice([rnd.randrange(0, 16), rnd.randrange(16, 24), rnd.randrange(24, 400)])
                f.seek(off)
                f.write(bytes([rnd.randrange(256)]))
        for q in [b"1:10000-10200", b"1:10010-10050", b"1:10040-10040", b"1:10001-10090", b"1:10100-10100"]:
            want = G.oracle_sparse_query(path, q)
            ref, hr, a, b = G.oracle_parse_query(q)
            got = E.emu_sparse_query(path, ref, hr, a, b)
            assert got == want, (seed, q, got[0], want[0], len(got[1]), len(want[1]))

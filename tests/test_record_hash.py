"""The batch checker's record digest (include/vcfc.h vcfc_record_hash_device,
csrc/vcfc_check.hip) on the CPU: the kernel on the fiber emulator and the
oracle's vcfo_hash64 against a plain-Python statement of the digest, and the
oracle's threaded row encode against its one-line encode.  These digests are
what the full-size GPU parity tests (tests/test_gpu_fullsize.py) compare."""
import random

import numpy as np

import decode_cases as D
import emu_io as E
import golden_io as G

M64 = (1 << 64) - 1


def mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def py_hash64(rec):
    h = (len(rec) * 0x9E3779B97F4A7C15) & M64
    for k in range(0, (len(rec) + 7) // 8):
        w = int.from_bytes(rec[8 * k:8 * k + 8].ljust(8, b"\0"), "little")
        h = (h + mix64(w ^ ((k * 0xD1B54A32D192ED03 + 0x8CB92BA72F3D8DD7) & M64))) & M64
    return mix64(h)


def test_oracle_digest_matches_statement():
    rnd = random.Random(1)
    for n in list(range(0, 40)) + [511, 512, 513, 4096, 10007]:
        rec = bytes(rnd.randrange(256) for _ in range(n))
        assert G.oracle_hash64(rec) == py_hash64(rec), n


def test_emulated_kernel_digest_every_alignment():
    """Records of 0..1100 bytes at every byte alignment, packed back to back
    (lengths past 512 words per lane-pass included)."""
    rnd = random.Random(2)
    lens = [0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 63, 64, 65, 511, 512, 513, 520, 1100] + \
           [rnd.randrange(0, 300) for _ in range(40)]
    recs = [bytes(rnd.randrange(256) for _ in range(n)) for n in lens]
    for lead in range(4):
        blob = b"\xAB" * lead + b"".join(recs)
        off = np.zeros(len(recs) + 1, dtype=np.uint64)
        np.cumsum([len(r) for r in recs], out=off[1:])
        off += lead
        got = E.emu_record_hash(blob, off)
        want = [G.oracle_hash64(r) for r in recs]
        assert [int(x) for x in got] == want, lead


def test_threaded_oracle_rows_match_line_encode():
    vcf = G.gz("fuzz_encode.vcf.gz")
    buf, off, ln = E.data_lines(vcf)
    st, size, h = G.oracle_encode_rows_hash(buf, off, ln, threads=5)
    for i in range(len(off)):
        s1, rec = G.oracle_encode_line(buf[int(off[i]):int(off[i]) + int(ln[i])])
        assert st[i] == s1, i
        if s1 == 0:
            assert size[i] == len(rec) and int(h[i]) == G.oracle_hash64(rec), i
    rnd = random.Random(3)
    rows = D.rows(rnd, 50, 300, escapes=0.05, odd=0.02)
    blob = b"\n".join(rows) + b"\n"
    b2, off2, ln2 = E.data_lines(blob)
    st2, size2, h2 = G.oracle_encode_rows_hash(b2, off2, ln2, threads=3)
    assert (st2 == 0).all()
    assert [int(x) for x in h2] == [G.oracle_hash64(G.oracle_encode_line(r)[1]) for r in rows]

"""Pipelined ingest on the CPU: the product pipeline
(csrc/vcfc_ingest_driver.h: reader threads -> line index + encode -> writer)
and its kernels (csrc/vcfc_ingest.hip, csrc/vcfc_encode.hip) compiled against
the fiber SIMT emulator, with chunks of a few KiB so that lines straddle
chunk boundaries.  Checked byte-exact against the reference's own compress
outputs (tests/golden) and against the oracle (statuses, error lines, the
output written before an error)."""
import random

import pytest

import decode_cases as D
import emu_io as E
import golden_io as G

OK, E_LT8COLS, E_8COLS, E_HEADER, E_ARG = 0, 1, 2, 3, 5


def check(vcf, chunk, name=""):
    st_o, want, el_o = G.oracle_compress(vcf)
    st, got, el = E.emu_compress(vcf, chunk=chunk)
    assert st == st_o, (name, chunk, st, st_o)
    assert got == want, (name, chunk, len(got), len(want))
    if st_o != OK:
        assert el == el_o, (name, chunk, el, el_o)


@pytest.mark.parametrize("chunk,lines", [(4096, 900), (65536, 3000), (1 << 20, None)])
def test_reference_config1(chunk, lines):
    """configs[0] through the pipelined driver; with small chunks on a prefix
    of the file (every line straddling chunks), whole with 1 MiB chunks."""
    vcf = G.gz("random_100x10000.vcf.gz")
    if lines is None:   # (three reader threads)
        st, out, _ = E.emu_compress(vcf, chunk=chunk, read_threads=3)
        assert st == OK and out == G.gz("random_100x10000.vcfc.gz")
        return
    cut = 0
    while vcf[cut:cut + 1] == b"#":   # header lines
        cut = vcf.index(b"\n", cut) + 1
    for _ in range(lines):
        cut = vcf.index(b"\n", cut) + 1
    check(vcf[:cut], chunk, "config1 prefix")


def test_reference_edge_file_and_bad_header():
    ec = G.edge_cases()
    st, out, _ = E.emu_compress(bytes.fromhex(ec["file"]["input"]), chunk=4096)
    assert st == OK and out.hex() == ec["file"]["output"]
    check(bytes.fromhex(ec["bad_header_file"]["input"]), 4096, "bad_header_file")


def mixed_file(rnd, n_rows, samples):
    """Header, data rows, and the lines compress() treats specially: empty
    lines, '##'/'#' lines between data rows, a final line without '\\n'."""
    lines = [D.header(samples).rstrip(b"\n").split(b"\n")[0], D.header(samples).rstrip(b"\n").split(b"\n")[1]]
    for r in D.rows(rnd, n_rows, samples, escapes=0.03):
        lines.append(r)
        x = rnd.random()
        if x < 0.05:
            lines.append(b"")
        elif x < 0.08:
            lines.append(b"##note=%d" % rnd.randrange(1000))
        elif x < 0.10:
            lines.append(b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS0")
    return b"\n".join(lines) + (b"\n" if rnd.random() < 0.5 else b"")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mixed_files_match_oracle(seed):
    rnd = random.Random(seed)
    for samples in (1, 40, 300):
        vcf = mixed_file(rnd, 60, samples)
        for chunk in (1 << 12, 1 << 14, 1 << 20):
            check(vcf, chunk, "mixed S=%d" % samples)


@pytest.mark.parametrize("seed", [4, 5])
def test_errors_match_oracle(seed):
    """A failing line (data line with < 8 or exactly 8 columns, a '#' header
    line with < 8 terms) in various chunks: output up to that line, its
    status and line number."""
    rnd = random.Random(seed)
    base = mixed_file(rnd, 80, 50).split(b"\n")
    bad = [b"1\t2\t3", b"1\t2\t3\t4\t5\t6\t7\t8", b"#CHROM\tPOS", b"#", b"1\t2\t3\t4\t5\t6\t7\t8\t9"]
    for b in bad:
        for at in (2, 5, 40, len(base) - 1):
            lines = list(base)
            lines.insert(at, b)
            vcf = b"\n".join(lines)
            for chunk in (1 << 12, 1 << 16):
                check(vcf, chunk, "bad %r at %d" % (b, at))
        # two failures: the first one wins
        lines = list(base)
        lines.insert(30, b"#CHROM")
        lines.insert(10, b)
        check(b"\n".join(lines), 1 << 12, "two failures")


def test_empty_and_tiny_inputs():
    for vcf in (b"", b"\n", b"\n\n\n", b"##x", b"##x\n", b"#", b"1\t2\t3\t4\t5\t6\t7\t8\t9",
                b"1\t2\t3\t4\t5\t6\t7\t8\t9\t0|0\n\n", b"\r\n"):
        for chunk in (4096, 1 << 16):
            check(vcf, chunk, repr(vcf))


def long_line_file(rnd, n_short, long_samples, samples=40):
    """Short rows with a few rows of `long_samples` tokens mixed in (at the
    start, the middle, and as an unterminated last line)."""
    lines = D.header(samples).rstrip(b"\n").split(b"\n")
    rows = D.rows(rnd, n_short, samples, escapes=0.03)
    big = [b"\t".join([b"1", b"%d" % (10 + k), b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] +
                       [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(n)])
           for k, n in enumerate(long_samples)]
    body = [big[0]] + rows[:n_short // 2] + big[1:-1] + rows[n_short // 2:] + [big[-1]]
    return b"\n".join(lines + body)


@pytest.mark.parametrize("chunk", [4096, 8192])
def test_line_longer_than_chunk(chunk):
    """A line longer than the chunk grows that chunk (doubling, its bytes
    kept) until the line fits: one pass, output identical to the reference's
    (compress() reads line by line, src/compress.cpp:218)."""
    rnd = random.Random(chunk)
    vcf = long_line_file(rnd, 50, [2000, 5000, 1100, 9000])   # lines of 4.4 KB .. 36 KB
    check(vcf, chunk, "long lines")
    st, out, _ = E.emu_compress(vcf, chunk=chunk)
    assert st == OK
    # a single line longer than every chunk, no header
    vcf = b"\t".join([b"1", b"2", b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + [b"0|1"] * 3000)
    check(vcf, chunk, "one long line")


def test_line_longer_than_max_chunk():
    """Growth stops at cfg.max_chunk: E_ARG, and the lines before the long one
    are written (the C ABI's limit is 3 GiB; a record's LEN is < 2^30)."""
    rnd = random.Random(9)
    lines = D.header(40).rstrip(b"\n").split(b"\n") + D.rows(rnd, 20, 40)
    head = b"\n".join(lines) + b"\n"
    vcf = head + b"\t".join([b"1", b"2", b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + [b"0|1"] * 5000) + b"\n"
    st, out, _ = E.emu_compress(vcf, chunk=4096, max_chunk=16384)
    assert st == E_ARG
    st_o, want, _ = G.oracle_compress(head)
    assert st_o == OK and want.startswith(out) and len(out) > 0


def test_short_lines_overflow_the_segment_slot():
    """More than 256 lines in a 16 KiB segment of the line index (short '##'
    lines, runs of empty lines): those segments are scanned again."""
    rnd = random.Random(11)
    head = b"".join(b"##k%d=%d\n" % (i, rnd.randrange(10)) for i in range(4000))
    rows = D.rows(rnd, 30, 20)
    body = b"\n".join(rows[:10]) + b"\n" + b"\n" * 6000 + b"\n".join(rows[10:]) + b"\n"
    vcf = head + D.header(20) + body
    for chunk in (1 << 14, 1 << 20):
        check(vcf, chunk, "short lines")


@pytest.mark.parametrize("mem_bound,piece", [(0, 1000), (12_345, 777), (10 ** 9, 4096), (65_536, 65_536)])
def test_held_output_places_every_byte(mem_bound, piece):
    """vcfc_ing::Held (dist_compress's rank output held until its offset is
    known): bytes in memory up to mem_bound, the rest in an unlinked spill
    file; place() writes them all at the offset, in order, once."""
    import ctypes
    import os
    import tempfile
    data = os.urandom(300_001)
    L = E.lib()
    u64, vp = ctypes.c_uint64, ctypes.c_void_p
    L.emu_held.argtypes = [ctypes.c_char_p, u64, u64, u64, ctypes.c_char_p, ctypes.c_int, u64,
                           ctypes.POINTER(u64), ctypes.POINTER(u64)]
    with tempfile.TemporaryDirectory() as d:
        op = os.path.join(d, "out")
        with open(op, "wb") as f:
            f.write(b"x" * 17)
        fd = os.open(op, os.O_WRONLY)
        m, s = ctypes.c_uint64(0), ctypes.c_uint64(0)
        try:
            st = L.emu_held(data, len(data), piece, mem_bound, d.encode(), fd, 17, ctypes.byref(m), ctypes.byref(s))
        finally:
            os.close(fd)
        assert st == 0
        assert m.value == min(mem_bound, len(data)) and m.value + s.value == len(data)
        assert open(op, "rb").read() == b"x" * 17 + data
        assert os.listdir(d) == ["out"]   # the spill file was unlinked at once

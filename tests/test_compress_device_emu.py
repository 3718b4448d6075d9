"""Device-resident compress() (vcfc_compress_device, csrc/vcfc_ingest_driver.h
compress_device: line index + encoder over file bytes already in device
memory, output left there) on the CPU emulator, with chunks of a few KiB so
chunk ends fall between lines everywhere, '#' lines interleave with records
and long lines grow their chunk.  Checked against the reference's own
compress outputs (tests/golden) and the oracle: bytes, statuses, error lines
(reference src/compress.cpp:205-257)."""
import random

import pytest

import emu_io as E
import golden_io as G
import test_ingest_emu as T

OK, E_ARG = 0, 5


def nl(vcf):
    """The device entry takes whole lines: getline returns an unterminated
    last line as if it ended with '\\n'."""
    return vcf if not vcf or vcf.endswith(b"\n") else vcf + b"\n"


def check(vcf, chunk, name=""):
    vcf = nl(vcf)
    st_o, want, el_o = G.oracle_compress(vcf)
    st, got, el = E.emu_compress_device(vcf, chunk=chunk)
    assert st == st_o, (name, chunk, st, st_o)
    assert got == want, (name, chunk, len(got), len(want))
    if st_o != OK:
        assert el == el_o, (name, chunk, el, el_o)


def test_reference_config1():
    """A 1 500-line prefix of configs[0] in 4 KiB and 64 KiB chunks (the whole
    file runs through the device path on the GPU, tests/test_gpu_ingest.py)."""
    vcf = G.gz("random_100x10000.vcf.gz")
    cut = 0
    while vcf[cut:cut + 1] == b"#":
        cut = vcf.index(b"\n", cut) + 1
    for _ in range(1500):
        cut = vcf.index(b"\n", cut) + 1
    check(vcf[:cut], 4096, "config1 prefix, 4 KiB chunks")
    check(vcf[:cut], 1 << 16, "config1 prefix, 64 KiB chunks")


def test_reference_edge_file_and_bad_header():
    ec = G.edge_cases()
    st, out, _ = E.emu_compress_device(nl(bytes.fromhex(ec["file"]["input"])), chunk=4096)
    assert st == OK and out.hex() == ec["file"]["output"]
    check(bytes.fromhex(ec["bad_header_file"]["input"]), 4096, "bad_header_file")


@pytest.mark.parametrize("seed", [1, 2])
def test_mixed_files_match_oracle(seed):
    """'#' lines between data rows (the scratch-buffer placement), empty lines."""
    rnd = random.Random(seed)
    for samples in (1, 40, 300):
        vcf = T.mixed_file(rnd, 60, samples)
        for chunk in (1 << 12, 1 << 20):
            check(vcf, chunk, "mixed S=%d" % samples)


def test_errors_match_oracle():
    rnd = random.Random(4)
    base = T.mixed_file(rnd, 80, 50).split(b"\n")
    for b in (b"1\t2\t3", b"1\t2\t3\t4\t5\t6\t7\t8", b"#CHROM\tPOS", b"#"):
        for at in (2, 40, len(base) - 1):
            lines = list(base)
            lines.insert(at, b)
            for chunk in (1 << 12, 1 << 16):
                check(b"\n".join(lines), chunk, "bad %r at %d" % (b, at))


def test_tiny_inputs_and_unterminated():
    for vcf in (b"", b"\n", b"\n\n\n", b"##x\n", b"#\n", b"1\t2\t3\t4\t5\t6\t7\t8\t9\n", b"\r\n"):
        check(vcf, 4096, repr(vcf))
    st, out, _ = E.emu_compress_device(b"##x", chunk=4096)   # last byte not '\n'
    assert st == E_ARG and out == b""


@pytest.mark.parametrize("chunk", [4096, 8192])
def test_line_longer_than_chunk(chunk):
    rnd = random.Random(chunk)
    check(T.long_line_file(rnd, 50, [2000, 5000, 1100, 9000]), chunk, "long lines")


def test_line_longer_than_max_chunk():
    rnd = random.Random(9)
    lines = T.D.header(40).rstrip(b"\n").split(b"\n") + T.D.rows(rnd, 20, 40)
    head = b"\n".join(lines) + b"\n"
    vcf = head + b"\t".join([b"1", b"2", b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + [b"0|1"] * 5000) + b"\n"
    st, out, _ = E.emu_compress_device(vcf, chunk=4096, max_chunk=16384)
    assert st == E_ARG
    st_o, want, _ = G.oracle_compress(head)
    assert st_o == OK and out == want


def test_short_lines_overflow_the_segment_slot():
    """More than 256 lines in a 16 KiB segment (short '##' lines, runs of
    empty lines): k_nl_place scans those segments again."""
    rnd = random.Random(11)
    head = b"".join(b"##k%d=%d\n" % (i, rnd.randrange(10)) for i in range(4000))
    rows = T.D.rows(rnd, 30, 20)
    body = b"\n".join(rows[:10]) + b"\n" + b"\n" * 6000 + b"\n".join(rows[10:]) + b"\n"
    vcf = head + T.D.header(20) + body
    for chunk in (1 << 14, 1 << 20):
        check(vcf, chunk, "short lines")


PREFIX = b"1\t%d\trs\tA\tC\t50\tPASS\tAC=1\tGT\t"


def hop_trap_file(kind, rnd, S_A=300, S_B=45):
    """Lines on which the hop line index (vcfc_line_index with the header's
    sample count S) guesses a data line's end wrongly: row A (longer than the
    index's 1 KiB first window, which finds shorter lines exactly) has fewer
    samples than the header, and the byte where A would end with S 3-byte
    tokens is the '\\n' of a later line B with TABs at the 31 places 4, 8, ...
    before it.  The hop index then counts A..B as one line; the encoder must
    see the '\\n' inside it and the chunk is indexed again from every byte.
      tab:    A ends in a full token: its '\\n' sits where a TAB would
      escape: A ends in "0|" and B starts with TAB and 3-byte fields, so the
              merged row is 3-byte tokens throughout, one of them "0|\\n"
              (the fast kernel's escape path must refuse it)
      var:    A mixes 1-byte tokens (the variable-token kernel's scan)
      lines:  '#' and empty lines between A and B"""
    toks = lambda k: [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(k)]
    pre = PREFIX % 7
    if kind == "escape":
        a = pre + b"\t".join(toks(S_A - 1) + [b"0|"])
        b = b"\t" + b"\t".join([b"abc"] * 8) + b"\t" + b"\t".join(toks(S_B))
        S = S_A + 8 + S_B                     # |B| = 4 (S - S_A)
        mid = []
    else:
        if kind == "var":
            at = toks(S_A)
            for i in rnd.sample(range(S_A), 6):
                at[i] = b"1"
            at[0] = b"0"; at[1] = b"1|0"      # 6 x 1-byte: 12 bytes shorter
        else:
            at = toks(S_A)
        a = pre + b"\t".join(at)
        mid = [b"##between", b""] if kind == "lines" else []
        # B ends where A's guess does: len(A) + 1 + sum(mid + 1) + len(B) = len(pre) + 4 S - 1
        gap = sum(len(m) + 1 for m in mid)
        S = S_A + 60
        blen = len(pre) + 4 * S - 1 - len(a) - 1 - gap
        pb = PREFIX % 8
        nb = (blen - len(pb) + 1) // 4
        pad = blen - (len(pb) + 4 * nb - 1)
        pb = pb.replace(b"rs", b"rs" + b"x" * pad)
        b = pb + b"\t".join(toks(nb))
        assert len(b) == blen and nb >= 32
    hdr = T.D.header(S)
    rows = [PREFIX % (100 + i) + b"\t".join(toks(S)) for i in range(5)]
    body = rows[:3] + [a] + mid + [b] + rows[3:]
    return hdr + b"\n".join(body) + b"\n"


@pytest.mark.parametrize("kind", ["tab", "escape", "var", "lines"])
def test_hop_index_wrong_guess_is_caught(kind):
    rnd = random.Random(kind)
    vcf = hop_trap_file(kind, rnd)
    for chunk in (4096, 1 << 16):
        check(vcf, chunk, "hop trap " + kind)
    redo = []
    st, out, _ = E.emu_compress_device(vcf, chunk=1 << 16, redo=redo)
    st2, out2, _ = E.emu_compress_device(vcf, chunk=1 << 16, hop=False, redo=redo)
    assert st == st2 == OK and out == out2
    assert redo == [1, 0]   # the guess went wrong once, and was caught


def chr22_like(rnd, n_rows, S, prefix_jitter=40):
    """Rows of S 3-byte tokens behind prefixes whose lengths vary by up to
    prefix_jitter bytes (the hop index guesses each end from the previous
    row's prefix length), some '##' lines and an empty line among them."""
    lines = T.D.header(S).rstrip(b"\n").split(b"\n")
    for i in range(n_rows):
        info = b"AC=%d;AF=0.%d;NS=%s" % (rnd.randrange(100), rnd.randrange(10 ** 6), b"9" * rnd.randrange(prefix_jitter))
        toks = [rnd.choice([b"0|0", b"0|0", b"0|1", b"1|0", b"1|1", b"0|2"]) for _ in range(S)]
        lines.append(b"\t".join([b"22", b"%d" % (16050000 + 37 * i), b"rs%d" % rnd.randrange(10 ** 8), b"A", b"G",
                                 b"100", b"PASS", info, b"GT"] + toks))
        if i % 17 == 5:
            lines.append(b"##mid=%d" % i)
        if i == 11:
            lines.append(b"")
    return b"\n".join(lines) + b"\n"


@pytest.mark.parametrize("S,jitter", [(300, 40), (700, 300), (64, 5)])
def test_hop_index_equals_scan_index(S, jitter):
    """Where no guess goes wrong the hop index gives the scan index's tables
    exactly: guess windows that hit, miss (prefix lengths jumping by up to
    300 bytes: the VERIFY round) and lines shorter than the first KiB."""
    rnd = random.Random(S)
    vcf = chr22_like(rnd, 150, S, jitter)
    assert E.emu_line_index(vcf, S) == E.emu_line_index(vcf, 0)
    for chunk in (1 << 15, 1 << 20):
        check(vcf, chunk, "chr22-like S=%d" % S)


@pytest.mark.parametrize("kind", ["tab", "escape", "var", "lines"])
def test_hop_index_trap_counts_fewer_lines(kind):
    """On the trap files the hop index misses the '\\n' of row A (so the
    encoder's check is what makes test_hop_index_wrong_guess_is_caught pass)."""
    vcf = hop_trap_file(kind, random.Random(kind))
    S = vcf.split(b"\n")[1].count(b"\t") - 8
    hop, scan = E.emu_line_index(vcf, S), E.emu_line_index(vcf, 0)
    # A..B counted as one data line ('#' and empty lines between them swallowed)
    assert hop[0][0] < scan[0][0] and hop[0][1] == scan[0][1] - 1

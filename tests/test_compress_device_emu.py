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
from hop_cases import chr22_like, hop_trap_dense_segment, hop_trap_file, law2_like

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


@pytest.mark.parametrize("S,jitter", [(300, 40), (700, 300), (64, 5)])
def test_hop_index_equals_scan_index(S, jitter):
    """Where no guess goes wrong the hop index gives the scan index's tables
    exactly: guess windows that hit, miss (prefix lengths jumping by up to
    300 bytes: the VERIFY round) and lines shorter than the first KiB."""
    rnd = random.Random(S)
    vcf = chr22_like(rnd, 150, S, jitter)
    scan = E.emu_line_index(vcf, 0)
    assert E.emu_line_index(vcf, S) == scan
    # the walkers compress_device takes for such files (no learned
    # candidates: GUESS rounds), with the product's walker count and with
    # one wave of walkers (~40 lines each)
    assert E.emu_line_index(vcf, S, learn=False) == scan
    assert E.emu_line_index(vcf, S, hop_walkers=4, learn=False) == scan
    for chunk in (1 << 15, 1 << 20):
        check(vcf, chunk, "chr22-like S=%d" % S)


@pytest.mark.parametrize("S,jitter,walkers", [(2504, 40, 2), (2504, 40, 8), (700, 40, 2), (700, 300, 2)])
def test_hop_guess_rounds(S, jitter, walkers):
    """Round 6: GUESS rounds (k_nl_hop without learned candidates) guess the
    next 4 / 8 line ends from the mean line length and read one 256-byte
    window per line.  On chr22-like rows without '#' lines among them the
    walkers read ~0.3 KB per 10 KB line (LINE rounds alone: ~0.55 KB); the
    index is the scan's exactly, with prefixes jumping by up to 300 bytes
    too (windows that miss: the line by LINE)."""
    vcf = chr22_like(random.Random(S * 3 + jitter), 400, S, jitter)
    keep = [ln for ln in vcf.split(b"\n") if ln and not ln.startswith(b"##mid")]
    vcf = b"\n".join(keep) + b"\n"
    scan = E.emu_line_index(vcf, 0)
    E.emu_hop_read()
    assert E.emu_line_index(vcf, S, hop_walkers=walkers, learn=False) == scan
    guess = E.emu_hop_read()
    assert E.emu_line_index(vcf, S, hop_walkers=walkers, learn=True) == scan
    line = E.emu_hop_read()
    if S == 2504 and jitter == 40:
        assert guess < 0.04 * len(vcf) and guess < 0.7 * line, (guess, line, len(vcf))
    # every walker's first lines guessed from the first data line's length
    # (compress_device's len_hint) instead of found by LINE
    first = next(ln for ln in vcf.split(b"\n") if ln and not ln.startswith(b"#"))
    assert E.emu_line_index(vcf, S, hop_walkers=walkers, learn=False, len_hint=len(first) + 1) == scan
    hinted = E.emu_hop_read()
    if S == 2504 and jitter == 40:
        assert hinted < guess, (hinted, guess)
    assert E.emu_line_index(vcf, S, hop_walkers=walkers, learn=False, len_hint=700) == scan   # a wrong hint
    check(vcf, 1 << 22, "guess S=%d" % S)


@pytest.mark.parametrize("kind", ["tab", "escape", "var", "lines"])
def test_hop_index_trap_counts_fewer_lines(kind):
    """On the trap files the hop index misses the '\\n' of row A (so the
    encoder's check is what makes test_hop_index_wrong_guess_is_caught pass)."""
    vcf = hop_trap_file(kind, random.Random(kind))
    S = vcf.split(b"\n")[1].count(b"\t") - 8
    hop, scan = E.emu_line_index(vcf, S), E.emu_line_index(vcf, 0)
    # A..B counted as one data line ('#' and empty lines between them swallowed)
    assert hop[0][0] < scan[0][0] and hop[0][1] == scan[0][1] - 1


def test_hop_index_wrong_guess_in_dense_segment():
    """A wrong guess inside a segment of more than 128 line ends whose last
    line is a '#' line (hop_trap_dense_segment): k_nl_place's rescan finds
    more ends than the hop counted, flags the index, and the chunk is indexed
    again from every byte -- the output is the reference's."""
    vcf = hop_trap_dense_segment(random.Random(5))
    S = vcf.split(b"#CHROM", 1)[1].split(b"\n", 1)[0].count(b"\t") - 8
    hop, scan = E.emu_line_index(vcf, S), E.emu_line_index(vcf, 0)
    assert hop[0][3] == 2 and scan[0][3] == 0          # counts[3]: the rescan found the hop's count wrong
    redo = []
    st, out, _ = E.emu_compress_device(vcf, chunk=1 << 16, redo=redo)
    st_o, want, _ = G.oracle_compress(vcf)
    assert st == st_o == OK and out == want
    assert redo == [1]


def test_hop_index_long_header():
    """A header longer than the first 64 KiB read (the sample count comes
    from a second, 1 MiB read) and one with an empty line before #CHROM: the
    hop index is still used (the trap is hit and caught: one re-index)."""
    rnd = random.Random(77)
    trap = hop_trap_file("tab", rnd)
    meta = b"".join(b"##contig=<ID=chr%d,length=%d>\n" % (i, 10 ** 8 + i) for i in range(3000))
    assert len(meta) > 64 << 10
    for vcf in (meta + trap, b"##fileformat=VCFv4.2\n\n" + trap.split(b"\n", 1)[1]):
        redo = []
        st, out, _ = E.emu_compress_device(vcf, chunk=1 << 20, redo=redo)
        st_o, want, _ = G.oracle_compress(vcf)
        assert st == st_o == OK and out == want
        assert redo == [1]


@pytest.mark.parametrize("S,dp_width", [(2504, 2), (700, 2), (300, 0)])
def test_hop_index_law2_rows(S, dp_width):
    """Law-2-shaped files (hop_cases.law2_like: haploid, GT:DP:GQ, '.', '#'
    lines): the hop index's learned candidates (TRY / LEARN) give exactly the
    scan index's tables, and the walkers read far less than the file when the
    genotype-region lengths repeat per row kind (dp_width 2); with DP/GQ of
    random widths (dp_width 0) the GT:DP:GQ rows are found by FIND and
    nothing breaks."""
    rnd = random.Random(S + dp_width)
    vcf = law2_like(rnd, 120 if S > 1000 else 240, S, dp_width=dp_width)
    scan = E.emu_line_index(vcf, 0)
    assert E.emu_line_index(vcf, S) == scan              # the product's walker count (~20 lines each)
    E.emu_hop_read()
    assert E.emu_line_index(vcf, S, hop_walkers=4) == scan   # one wave, ~60 lines per walker
    read = E.emu_hop_read()
    if S > 1000 and dp_width:
        # 2504 samples (~13 KB lines), ~30 lines per walker, 120 per wave --
        # as the 13 GB config-size file: the three learned kinds are read
        # once per wave, every other line for ~1.3 KB of windows
        assert read < 0.3 * len(vcf), (read, len(vcf))
    for chunk in (1 << 16, 1 << 22):
        check(vcf, chunk, "law2-like S=%d" % S)
    st_o, want, _ = G.oracle_compress(vcf)
    for hop in ("learn", "nolearn"):   # (compress_device chooses by the first data lines; both are exact)
        st, got, _ = E.emu_compress_device(vcf, chunk=1 << 22, hop=hop)
        assert st == st_o == OK and got == want, hop


def test_hop_seeded_candidates_law2():
    """Round 6: compress_device seeds the learning walkers with the region
    lengths and TAB signatures of the irregular data lines in its header
    window (vcfc_ingest_driver.h learn_candidates): the output is the
    oracle's, and on a 120-row law-2 file the walkers read well under half
    of it (they no longer FIND and LEARN each row kind first)."""
    vcf = law2_like(random.Random(2506), 120, 2504, dp_width=2)
    st_o, want, _ = G.oracle_compress(vcf)
    E.emu_hop_read()
    st, got, _ = E.emu_compress_device(vcf, chunk=1 << 24)
    read = E.emu_hop_read()
    assert st == st_o == OK and got == want
    assert read < 0.4 * len(vcf), (read, len(vcf))


def test_law2_rows_deferred_records(monkeypatch):
    """compress_device with deferred records on (vcfc_ctx_set_deferred_records):
    law-2-shaped files whose GT:DP:GQ rows are sized first and written straight
    into the output after the size scan, with the hop index's '\n' checks
    on -- the oracle's output."""
    monkeypatch.setenv("EMU_DEFER", "1")
    for S, dp in ((700, 2), (300, 0)):
        rnd = random.Random(S * 7 + dp)
        vcf = law2_like(rnd, 120, S, dp_width=dp)
        st_o, want, _ = G.oracle_compress(vcf)
        for chunk in (1 << 16, 1 << 22):
            st, got, _ = E.emu_compress_device(vcf, chunk=chunk)
            assert st == st_o == OK and got == want, (S, dp, chunk)


def test_hop_learn_choice():
    """compress_device turns the learned candidates on when the first data
    lines are not all S 3-byte tokens (vcfc_ingest_driver.h
    data_lines_irregular), off for chr22-shaped files."""
    import ctypes
    lib = E.lib()
    S = 300
    chr22 = chr22_like(random.Random(1), 20, S)
    law2 = law2_like(random.Random(2), 20, S, kinds=(0, 1))
    # (the helper itself, through the emulator build's host code)
    lib.emu_data_lines_irregular.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32]
    assert lib.emu_data_lines_irregular(chr22, len(chr22), S) == 0
    assert lib.emu_data_lines_irregular(law2, len(law2), S) == 1


@pytest.mark.parametrize("n_hdr", [1023, 1024, 1500])
def test_many_header_lines(n_hdr):
    """Round 6: the host reads the index counts and the first 1 024 '#' line
    entries in one D2H (k_index_summary), and copies a header that precedes
    every data line ahead of the encode.  Headers of 1 023 / 1 024 / 1 500
    lines (the last past the summary: its tables come in a second D2H), one
    chunk and 4 KiB chunks, a bad header line past entry 1 024."""
    rnd = random.Random(n_hdr)
    hdr = b"".join(b"##meta%d=%s\n" % (i, b"x" * rnd.randint(0, 30)) for i in range(n_hdr))
    S = 40
    hdr += b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + b"\t".join(b"s%d" % i for i in range(S)) + b"\n"
    rows = b"".join(b"1\t%d\t.\tA\tC\t50\tPASS\t.\tGT\t" % (100 + i) +
                    b"\t".join(rnd.choice([b"0|0", b"0|1", b"1|1"]) for _ in range(S)) + b"\n" for i in range(60))
    check(hdr + rows, 1 << 20, "one chunk")
    check(hdr + rows, 4096, "4 KiB chunks")
    bad = hdr.split(b"\n")
    bad[min(n_hdr - 2, 1200)] = b"#bad\theader"
    check(b"\n".join(bad) + rows, 1 << 20, "bad header line")

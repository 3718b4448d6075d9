"""Kernel logic on the CPU: the product kernel source (csrc/vcfc_encode.hip)
compiled against the fiber SIMT emulator (tests/simt_emu) and checked
byte-exact against the oracle / the reference's golden vectors.  The GPU
parity tests (test_gpu_encode.py) repeat these through the real HIP path."""
import random

import numpy as np
import pytest

import emu_io as E
import golden_io as G


def run(lines, lead=0):
    """Place lines in a buffer starting at `lead` (alignment sweep) and encode."""
    buf = bytearray(b"#" * lead)
    offs, lens = [], []
    for ln in lines:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    return E.emu_encode(bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32))


def test_edge_cases_all_alignments():
    ec = G.edge_cases()
    good = [c for c in ec["cases"] if "record" in c]
    lines = [bytes.fromhex(c["line"]) for c in good]
    want = b"".join(bytes.fromhex(c["record"]) for c in good)
    for lead in range(16):
        st, out, ro, err = run(lines, lead)
        assert err == E.NO_ERROR if hasattr(E, "NO_ERROR") else err == (1 << 64) - 1
        assert out == want, lead


def test_error_rows_report_first_failing_row():
    ec = {c["name"]: c for c in G.edge_cases()["cases"]}
    ok = bytes.fromhex(ec["run300_00"]["line"])
    eight = bytes.fromhex(ec["eight_cols"]["line"])
    seven = bytes.fromhex(ec["seven_cols"]["line"])
    st, out, ro, err = run([ok, ok, eight, ok, seven])
    assert err == (2 << 8) | 2
    assert out[:int(ro[2])] == bytes.fromhex(ec["run300_00"]["record"]) * 2
    st, out, ro, err = run([ok, seven, eight])
    assert err == (1 << 8) | 1


def test_fuzz_corpus_byte_exact():
    """The first 1 200 lines of the reference's fuzz corpus (the GPU test runs
    all 3 100): records == the reference output's bytes for them."""
    vcf = G.gz("fuzz_encode.vcf.gz")
    buf, lo, ll = E.data_lines(vcf)
    k = 1200
    st, out, ro, err = E.emu_encode(buf, lo[:k], ll[:k])
    assert err == (1 << 64) - 1
    want = G.gz("fuzz_encode.vcfc.gz")
    hdr_end = int(lo[0])
    assert want[:hdr_end + len(out)] == vcf[:hdr_end] + out


def test_random_vcf_rows_byte_exact():
    vcf = G.gz("random_100x10000.vcf.gz")
    want = G.gz("random_100x10000.vcfc.gz")
    buf, lo, ll = E.data_lines(vcf)
    k = 2000
    st, out, ro, err = E.emu_encode(buf, lo[:k], ll[:k])
    assert err == (1 << 64) - 1
    hdr = int(lo[0])
    assert want[hdr:hdr + len(out)] == out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wide_rows_multi_chunk(seed):
    """Rows spanning many 1 KiB chunks, clean and with escapes/empty fields."""
    rnd = random.Random(seed)
    pfx = b"22\t16050075\trs1\tA\tG\t100\tPASS\t" + b"AF=0.1;" * rnd.randint(1, 300) + b"\tGT\t"
    toks = []
    for _ in range(rnd.randint(2000, 5000)):
        r = rnd.random()
        toks.append(b"0|0" if r < 0.85 else b"0|1" if r < 0.9 else b"1|1" if r < 0.95 else b"1|0" if r < 0.99 else b"2|1")
    clean = pfx + b"\t".join(toks)
    dirty = pfx + b"\t".join(toks[:100]) + b"\t\t" + b"\t".join(toks[100:])
    runs = pfx + b"\t".join([b"0|0"] * 4000 + [b"1|1"] * 100)
    lines = [clean, dirty, runs]
    st, out, ro, err = run(lines, lead=seed)
    want = b"".join(G.oracle_encode_line(x)[1] for x in lines)
    assert err == (1 << 64) - 1 and out == want


def _chr22_like_rows(n, samples, seed):
    rnd = random.Random(seed)
    rows = []
    for i in range(n):
        af = rnd.choice([0.0, 0.0005, 0.002, 0.01, 0.05, 0.3, 0.9])
        multi = rnd.random() < 0.1
        toks = []
        for _ in range(samples):
            a = [1 if rnd.random() < af else 0 for _ in range(2)]
            if multi and rnd.random() < 0.01:
                a[rnd.randint(0, 1)] = 2
            toks.append(b"%d|%d" % (a[0], a[1]))
        pfx = b"22\t%d\trs%d\tA\tG\t100\tPASS\tAC=1;AF=%.4f;NS=2504\tGT\t" % (16050075 + 32 * i, i, af)
        rows.append(pfx + b"\t".join(toks))
    return rows


@pytest.mark.parametrize("seed", [11, 12])
def test_chr22_like_rows_skip_path(seed):
    """Long 0|0 runs exercise the whole-chunk skip, 127-chunk boundaries that
    straddle chunks, and run transitions at chunk starts."""
    lines = _chr22_like_rows(40, 2504, seed)
    st, out, ro, err = run(lines, lead=seed % 16)
    assert err == (1 << 64) - 1
    assert E.LAST_RETRIES[0] == 0   # escapes stay on the fast kernel's general step
    for i, ln in enumerate(lines):
        assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(ln)[1], i


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_short_rows_and_cap_boundaries(seed):
    """Rows whose first and last genotype chunk coincide (< 256 samples), and
    runs whose lengths sit on and around the caps (31, 127) and the 256-slot
    chunk, at every class: the first/last-chunk masking and the in-lane
    full/pending byte rules."""
    rnd = random.Random(seed)
    classes = [b"0|0", b"0|1", b"1|0", b"1|1"]
    lens = [1, 2, 3, 4, 5, 29, 30, 31, 32, 33, 61, 62, 63, 125, 126, 127, 128, 129, 253, 254, 255, 256, 257]
    lines = []
    for i in range(48):
        toks = []
        target = rnd.choice([1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 700, 1500])
        while len(toks) < target:
            c = rnd.choice(classes)
            toks += [c] * rnd.choice(lens)
        toks = toks[:target]
        pfx = b"22\t%d\trs%d\tA\tG\t100\tPASS\t%s\tGT\t" % (100 + i, i, b"X" * rnd.randint(1, 40))
        lines.append(pfx + b"\t".join(toks))
    for lead in (0, 1, 2, 3, 7, 13):
        st, out, ro, err = run(lines, lead=lead)
        assert err == (1 << 64) - 1
        assert E.LAST_RETRIES[0] == 0   # every row stayed on the fast kernel
        for i, ln in enumerate(lines):
            assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(ln)[1], (lead, i)


@pytest.mark.parametrize("seed", [31, 32])
def test_dense_rows_wrap_the_ring(seed):
    """Rows whose records are many times the 4 KiB LDS ring (a start at most
    tokens): run groups straddling the ring end, bursts every chunk."""
    rnd = random.Random(seed)
    classes = [b"0|0", b"0|1", b"1|0", b"1|1"]
    lines = []
    for i in range(6):
        n = rnd.choice([9000, 17000, 24001])
        p = rnd.choice([0.5, 0.9, 1.0])
        toks, c = [], 0
        for _ in range(n):
            if rnd.random() < p:
                c = rnd.randrange(4)
            toks.append(classes[c])
        pfx = b"22\t%d\trs%d\tA\tG\t100\tPASS\tAF=0.5\tGT\t" % (100 + i, i)
        lines.append(pfx + b"\t".join(toks))
    for lead in (0, 5, 10):
        st, out, ro, err = run(lines, lead=lead)
        assert err == (1 << 64) - 1
        assert E.LAST_RETRIES[0] == 0
        for i, ln in enumerate(lines):
            assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(ln)[1], (lead, i)


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_escape_rows_on_the_three_byte_path(seed):
    """3-byte escape tokens (multi-allelic, missing, unphased, raw high bytes)
    at every density, at token 0, at chunk edges (512-token chunks), at the
    row end, in runs of escapes, and right after runs that end on the caps:
    the escape path of the fast kernel (esc8), with and without an escape as
    the incoming class of a chunk."""
    rnd = random.Random(seed)
    plain = [b"0|0", b"0|1", b"1|0", b"1|1"]
    escs = [b"0|2", b"2|0", b"./.", b".|.", b"0/1", b"1/1", b"2|2", b"\xff|\x80", b"0|\r", b"3|1"]
    lens = [1, 2, 30, 31, 32, 126, 127, 128, 511, 512, 513]
    lines = []
    for i in range(24):
        target = rnd.choice([1, 2, 511, 512, 513, 1024, 1025, 2504, 5000])
        dens = rnd.choice([0.0005, 0.01, 0.04, 0.3, 1.0])
        toks = []
        while len(toks) < target:
            if rnd.random() < dens:
                toks += [rnd.choice(escs)] * rnd.choice([1, 1, 1, 2, 5])
            else:
                toks += [rnd.choice(plain)] * rnd.choice(lens)
        toks = toks[:target]
        for p in rnd.sample([0, 510, 511, 512, 1023, 1024, target - 1], 3):
            if 0 <= p < target:
                toks[p] = rnd.choice(escs)
        pfx = b"22\t%d\trs%d\tA\tG,T\t100\tPASS\t%s\tGT\t" % (100 + i, i, b"Y" * rnd.randint(1, 60))
        lines.append(pfx + b"\t".join(toks))
    for lead in (0, 3, 9):
        st, out, ro, err = run(lines, lead=lead)
        assert err == (1 << 64) - 1
        assert E.LAST_RETRIES[0] == 0   # escapes stay on the fast kernel
        for i, ln in enumerate(lines):
            assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(ln)[1], (lead, i)


def test_wide_compaction_shape(monkeypatch):
    """The 64-lanes-per-row compaction (chosen on the GPU for rows longer
    than 64 KiB on average) on the edge cases at every alignment and on
    multi-KiB records."""
    monkeypatch.setenv("EMU_WIDE_COMPACT", "1")
    ec = G.edge_cases()
    good = [c for c in ec["cases"] if "record" in c]
    lines = [bytes.fromhex(c["line"]) for c in good]
    want = b"".join(bytes.fromhex(c["record"]) for c in good)
    for lead in (0, 1, 7, 15):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1 and out == want, lead
    rnd = random.Random(5)
    classes = [b"0|0", b"0|1", b"1|0", b"1|1", b"0|2"]
    rows = []
    for i in range(5):
        toks = [classes[rnd.randrange(5)] for _ in range(rnd.choice([3000, 9000]))]
        rows.append(b"22\t%d\trs%d\tA\tG\t100\tPASS\t.\tGT\t" % (100 + i, i) + b"\t".join(toks))
    st, out, ro, err = run(rows, 3)
    assert err == (1 << 64) - 1
    assert out == b"".join(G.oracle_encode_line(x)[1] for x in rows)


def test_many_rows_scan_tiles_and_compaction_tiles():
    """More rows than two 4096-row scan tiles (the size and slot scans'
    look-back across tiles) and records of all sizes between 26 B and a few
    KiB (compaction tiles meeting many records, records crossing the
    primary/overflow split), with failing rows (empty records) between them:
    every record and offset equals the oracle's."""
    rnd = random.Random(77)
    lines, want = [], []
    for i in range(9000):
        k = rnd.choice([1, 1, 1, 2, 40, 300])
        toks = [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2", b"./."]) for _ in range(k)]
        ln = b"\t".join([b"1", b"%d" % i, b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + toks)
        lines.append(ln)
    st, out, ro, err = run(lines)
    assert err == (1 << 64) - 1
    for i in rnd.sample(range(len(lines)), 300) + [0, 4095, 4096, 8191, 8192, 8999]:
        assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(lines[i])[1], i
    assert int(ro[-1]) == sum(len(G.oracle_encode_line(x)[1]) for x in lines)
    # a failing row (7 columns: no record) every 1000 rows: the records
    # before the first one are intact, its error is reported
    bad = list(lines[:1600])
    for i in range(500, 1600, 300):
        bad[i] = b"1\t2\t3\t4\t5\t6\t7"
    st, out2, ro2, err2 = run(bad)
    assert err2 == (500 << 8) | 1
    assert out2[:int(ro2[500])] == out[:int(ro[500])]


def test_output_capacity_short():
    """out_cap below the records' total: the first row whose record ends past
    it is reported (VCFC_E_NOSPACE, row << 8 | 4), the records before it are
    intact, nothing is written past out_cap."""
    rnd = random.Random(5)
    lines = []
    for i in range(300):
        toks = [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(rnd.choice([3, 60, 400]))]
        lines.append(b"\t".join([b"1", b"%d" % i, b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] + toks))
    st, out, ro, err = run(lines)
    assert err == (1 << 64) - 1
    for cut_row in (0, 37, 211):
        cap = int(ro[cut_row]) + int(ro[cut_row + 1] - ro[cut_row]) // 2
        buf = bytearray()
        offs, lens = [], []
        for ln in lines:
            offs.append(len(buf))
            lens.append(len(ln))
            buf += ln + b"\n"
        st2, out2, ro2, err2 = E.emu_encode(bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32), cap=cap)
        assert err2 == (cut_row << 8) | 4, (cut_row, hex(err2))
        assert out2[:int(ro[cut_row])] == out[:int(ro[cut_row])]


PFX_V = b"X\t100\trs1\tA\tG\t50\tPASS\tAC=1\tGT\t"


def _var_rows(rnd, n, kinds):
    """Rows of odd-length tokens (the variable-token kernel's shape)."""
    rows = []
    for i in range(n):
        kind = kinds[i % len(kinds)]
        S = rnd.choice([1, 2, 3, 17, 63, 64, 65, 200, 511, 512, 513, 1023, 1024, 1025, 1500, 2600])
        toks = []
        p00 = rnd.choice([0.0, 0.5, 0.9, 0.99, 1.0])
        for j in range(S):
            if kind == "hap":       # haploid beside diploid
                toks.append(rnd.choice([b"0", b"1"]) if (j * 7 + i) % 3 == 0 else
                            (b"0|0" if rnd.random() < p00 else rnd.choice([b"0|1", b"1|0", b"1|1", b"0|0"])))
            elif kind == "dot":     # "." for missing
                toks.append(b"." if rnd.random() < 0.2 else (b"0|0" if rnd.random() < p00 else
                                                                  rnd.choice([b"0|1", b"1|1", b"2|1"])))
            elif kind == "long":    # GT:DP:GQ and other odd lengths
                toks.append(rnd.choice([b"0|0:35:99", b"0|1:17:12", b"1|1:123:9", b"0|0", b"1", b"./.",
                                        b"0|0:1", b"0" * 41]))
            elif kind == "gdg":     # escapes of 1, 5, 9 and 41 bytes only (the escape-chunk step)
                toks.append(rnd.choice([b"0|0:35:99", b"0|1:17:12", b"1|1:123:9", b"0|0:1", b"1", b"0" * 41]))
            elif kind == "ones":    # every token one byte
                toks.append(rnd.choice([b"0", b"1", b"."]))
            else:                   # plain runs with long 1-byte stretches
                toks.append(b"0|0" if (j // 200) % 2 == 0 else b"1")
        rows.append(PFX_V + b"\t".join(toks))
    return rows


@pytest.mark.parametrize("seed", [51, 52, 53])
def test_variable_token_rows(seed):
    """k_encode_var: rows whose tokens all have odd length (1, 3, 5, 9, 41
    bytes) -- haploid beside diploid, '.', GT:DP:GQ, all-1-byte rows, long
    0|0 runs broken by 1-byte escapes -- byte-exact against the oracle at
    every alignment of the buffer; only rows mixing tokens longer than 3
    bytes with 3-byte ones may be left to the general path."""
    rnd = random.Random(seed)
    lines = _var_rows(rnd, 72, ["hap", "dot", "long", "ones", "runs", "gdg"])
    want = [G.oracle_encode_line(x) for x in lines]
    assert all(w[0] == 0 for w in want)
    for lead in (0, 1, 2, 3, 7, 13):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1
        for i, (_, rec) in enumerate(want):
            assert out[int(ro[i]):int(ro[i + 1])] == rec, (seed, lead, i)
        # only rows with a token longer than 3 bytes may go on to
        # the general path (those mixing them with 3-byte tokens)
        longer = sum(1 for x in lines if max(len(t) for t in x[len(PFX_V):].split(b"\t")) > 3)
        assert E.LAST_RETRIES[0] <= longer, (E.LAST_RETRIES[0], longer)


def test_variable_token_rows_fall_back():
    """Rows the variable-token kernel must hand on (even-length tokens, empty
    fields, a trailing TAB, CR) are encoded by the general path, and the
    others of the batch stay exact."""
    rnd = random.Random(77)
    good = _var_rows(rnd, 8, ["hap", "long"])
    bad = [PFX_V + b"0\t1|1\t10\t0|0", PFX_V + b"0\t\t1|1\t0", PFX_V + b"1\t0|0\t", PFX_V + b"0|0\t1\t0\r",
           PFX_V + b"0\t" * 600 + b"00",
           PFX_V + b"\t".join([b"0"] * 2000 + [b"10", b"11", b"1"])]   # fails in its third chunk
    lines = [x for pair in zip(good, bad + bad[:2]) for x in pair]
    st, out, ro, err = run(lines)
    assert err == (1 << 64) - 1
    for i, x in enumerate(lines):
        assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(x)[1], i
    longer = sum(1 for x in good if max(len(t) for t in x[len(PFX_V):].split(b"\t")) > 3)
    assert 8 <= E.LAST_RETRIES[0] <= 8 + longer


def test_law2_synthetic_rows():
    """The synthetic law-2 rows (bench.py --law 2; kinds haploid, GT:DP:GQ,
    missing, unphased, '.'): byte-exact, and none of them reaches
    the general path (GT:DP:GQ rows take the variable-token kernel's escape
    chunks)."""
    rows = E.emu_synth_rows(40, 700, 2, seed=9)
    buf, lo, ll = rows
    st, out, ro, err = E.emu_encode(buf, lo, ll)
    assert err == (1 << 64) - 1
    gdg = 0
    for i in range(len(lo)):
        line = bytes(buf[int(lo[i]):int(lo[i]) + int(ll[i])])
        gdg += b"GT:DP:GQ" in line
        assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(line)[1], i
    assert gdg > 0 and E.LAST_RETRIES[0] == 0


def test_deferred_records(monkeypatch):
    """With deferred records on (VcfcEncodeArgs::defer_records), rows whose first genotype chunk is all escapes (GT:DP:GQ, all-1-byte,
    a row that turns mixed after its first chunk, another whose later chunk
    sends it to the general path) are deferred: k_encode_var only sizes
    them, the compaction skips their bytes, k_encode_defer writes each record
    straight into out after the size scan.  Byte-exact against the oracle
    beside staged neighbours (records meeting inside 16-byte blocks) at
    several alignments, and with out_cap cutting a deferred record."""
    rnd = random.Random(123)
    lines, expect_defer = [], 0
    for i in range(56):
        kind = i % 7
        if kind == 0:     # GT:DP:GQ, 300..1200 samples (> one 2 KiB chunk)
            S = rnd.choice([300, 301, 777, 1200])
            ln = PFX_V + b"\t".join(b"%d|%d:%d:%d" % (rnd.randint(0, 1), rnd.randint(0, 1), rnd.randint(10, 99),
                                                   rnd.randint(10, 99)) for _ in range(S))
            expect_defer += 1
        elif kind == 1:   # 1-byte tokens, then plain diploid ones (chunk 1 mixed)
            ln = PFX_V + b"\t".join([rnd.choice([b"0", b"1", b"."]) for _ in range(1100)] +
                                    [rnd.choice([b"0|0", b"0|1", b"1|1"]) for _ in range(rnd.randint(1, 700))])
            expect_defer += 1
        elif kind == 2:   # escapes first, an even-length token later: the general path (not deferred)
            ln = PFX_V + b"\t".join([b"0"] * 1500 + [b"10"] + [b"1"] * 3)
        elif kind == 3:   # one chunk only: staged
            ln = PFX_V + b"\t".join(rnd.choice([b"0", b"0|1:5:9"]) for _ in range(rnd.randint(1, 150)))
        elif kind == 4:   # 3-byte tokens: the fast kernel
            ln = b"\t".join([b"1", b"%d" % i, b"a", b"b", b"c", b"d", b"e", b"f", b"GT"] +
                            [rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(rnd.randint(1, 900))])
        elif kind == 5:   # 3-byte escapes beside 1-byte ones over > 1 chunk: k_encode_var's escape chunks
            # (no plain token), deferred; mixed 0|1 tokens later on in half of them
            S = rnd.choice([700, 900, 1300])
            toks = [rnd.choice([b"0/0", b"0/1", b"1/1", b"./.", b"0", b"."]) for _ in range(S)]
            if i % 2:
                toks[800:] = [rnd.choice([b"0|0", b"0|1"]) for _ in toks[800:]]
            ln = PFX_V + b"\t".join(toks)
            expect_defer += 1
        else:             # the same within one chunk (<= 512 tokens): staged by the fast kernel
            ln = PFX_V + b"\t".join(rnd.choice([b"0/0", b"0/1", b"./."]) for _ in range(rnd.randint(1, 512)))
        lines.append(ln)
    want = [G.oracle_encode_line(x)[1] for x in lines]
    monkeypatch.setenv("EMU_DEFER", "0")
    st, out, ro, err = run(lines)   # (off: nothing deferred, the same records)
    assert err == (1 << 64) - 1 and E.last_deferred() == 0 and out == b"".join(want)
    monkeypatch.delenv("EMU_DEFER")   # (the default since round 5: on)
    st, out, ro, err = run(lines)
    assert err == (1 << 64) - 1 and E.last_deferred() == expect_defer and out == b"".join(want)
    monkeypatch.setenv("EMU_DEFER", "1")
    for lead in (0, 3, 9):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1
        assert E.last_deferred() == expect_defer
        for i, w in enumerate(want):
            assert out[int(ro[i]):int(ro[i + 1])] == w, (lead, i)
    buf = bytearray()
    offs, lens = [], []
    for ln in lines:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    cut = 14   # a GT:DP:GQ row: out_cap ends inside its record
    cap = int(ro[cut]) + 100
    st2, out2, ro2, err2 = E.emu_encode(bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32), cap=cap)
    assert err2 == (cut << 8) | 4
    assert out2[:int(ro[cut])] == out[:int(ro[cut])]


def test_deferred_runs_share_tiles(monkeypatch):
    """Output tiles (4 KiB) whose bytes all belong to deferred records are
    skipped by the compaction, including a tile a deferred record ends in
    when the next records up to the tile end are deferred too, or the batch
    ends there; a tile that reaches a staged record is compacted.  Runs of
    GT:DP:GQ rows (records of 2.5-11 KiB, so a tile meets up to three of
    them) beside short staged rows and at the batch end, byte-exact."""
    monkeypatch.setenv("EMU_DEFER", "1")
    rnd = random.Random(77)

    def gdg(S):
        return PFX_V + b"\t".join(b"%d|%d:%d:%d" % (rnd.randint(0, 1), rnd.randint(0, 1), rnd.randint(10, 99),
                                                 rnd.randint(10, 99)) for _ in range(S))
    lines, expect_defer = [], 0
    for run_len in (5, 1, 3, 7):
        for _ in range(run_len):
            lines.append(gdg(rnd.choice([260, 300, 333, 410, 700, 1100])))
            expect_defer += 1
        lines.append(PFX_V + b"\t".join(rnd.choice([b"0|0", b"0|1"]) for _ in range(rnd.randint(1, 40))))
    for _ in range(4):   # the batch ends inside a deferred run
        lines.append(gdg(rnd.choice([260, 500, 900])))
        expect_defer += 1
    want = [G.oracle_encode_line(x)[1] for x in lines]
    for lead in (0, 7):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1 and E.last_deferred() == expect_defer
        assert out == b"".join(want), lead


def _gdg(rnd, S):
    return PFX_V + b"\t".join(b"%d|%d:%d:%d" % (rnd.randint(0, 1), rnd.randint(0, 1), rnd.randint(10, 99),
                                             rnd.randint(10, 99)) for _ in range(S))


def _encode_both(lines, monkeypatch, cap=None):
    """(deferral off, deferral on) results of the emulated encode."""
    buf = bytearray()
    offs, lens = [], []
    for ln in lines:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    args = (bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32))
    monkeypatch.setenv("EMU_DEFER", "0")
    off = E.emu_encode(*args, cap=cap)
    monkeypatch.setenv("EMU_DEFER", "1")
    on = E.emu_encode(*args, cap=cap)
    return off, on


def test_predicted_deferred_records(monkeypatch):
    """Once two rows of a wave agree on their token count, k_encode_var
    sizes a later row deferred on its first chunk without reading the rest
    (all escapes predicted: len + 9 + tokens); k_encode_defer's first pass
    encodes it in full and checks.  Correct predictions: no second layout
    pass.  Byte-exact either way against the oracle and against the encode
    without deferral."""
    rnd = random.Random(5)
    lines = [_gdg(rnd, 700) for _ in range(40)]
    want = b"".join(G.oracle_encode_line(x)[1] for x in lines)
    (st0, out0, ro0, err0), (st1, out1, ro1, err1) = _encode_both(lines, monkeypatch)
    assert err0 == err1 == (1 << 64) - 1
    assert out0 == out1 == want and list(ro0) == list(ro1)
    assert E.last_deferred() == 40 and E.last_mispredict() == 0


@pytest.mark.parametrize("where", ["interior", "last"])
def test_escape_step_refuses_other_shapes(where):
    """esc8 tests the 3-byte shape itself (round 5: on its gathered bytes, for
    interior chunks and the row's last chunk): a 1-byte and a 5-byte token in
    place of two 3-byte ones (the line length, and so the slot count, stays
    that of 3-byte tokens), a token holding 0x0B or 0x08, a TAB inside a
    token -- in a chunk that follows an escape chunk (the escape shape is
    tested alone there) or not -- go to the general step: byte-exact."""
    rnd = random.Random(77 if where == "interior" else 78)
    S = 1100   # chunks of 512 tokens: 0, 1 interior, 2 the last (76 tokens)
    pos = 700 if where == "interior" else 1060
    lines = []
    for defect in ("len15", "vt", "bs", "tab"):
        for esc_before in (False, True):
            toks = [rnd.choice([b"0|0", b"0|1", b"1|1"]) for _ in range(S)]
            if esc_before:   # escapes in the chunk before the defect's
                for k in range(pos - 300, pos - 280):
                    toks[k] = b"0|2"
            if defect == "len15":
                toks[pos], toks[pos + 3] = b"1", b"0|1:5"
            elif defect == "vt":
                toks[pos] = b"0\x0b1"
            elif defect == "bs":
                toks[pos] = b"\x08|1"
            else:
                toks[pos] = b"0\t1"
            lines.append(PFX_V + b"\t".join(toks))
    want = [G.oracle_encode_line(x) for x in lines]
    for lead in (0, 3):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1
        for i, (s0, w) in enumerate(want):
            assert s0 == 0 and out[int(ro[i]):int(ro[i + 1])] == w, (lead, i)


@pytest.mark.parametrize("lead", [0, 5])
def test_unphased_rows_handed_on_and_predicted(lead, monkeypatch):
    """Rows whose first 2 KiB genotype chunk holds 3-byte escapes only
    (unphased "0/1", missing "./."): k_encode_fast hands them to
    k_encode_var with VCFCD_GT0_LONG, which predicts their records without
    reading them; among them rows that turn plain after the first chunk, a
    row with one sample more, a single-chunk row (not handed on) and
    chr22-like rows whose first chunk has a plain token (kept by the fast
    kernel).  Byte-exact against the oracle and the encode without
    deferral."""
    rnd = random.Random(31 + lead)
    unph = [b"0/0", b"0/1", b"1/1", b"./."]
    S = 900

    def row(toks):
        return PFX_V + b"\t".join(toks)
    lines = [row([rnd.choice(unph) for _ in range(S)]) for _ in range(20)]
    lines[7] = row([rnd.choice(unph) for _ in range(600)] + [rnd.choice([b"0|0", b"0|1"]) for _ in range(S - 600)])
    lines[11] = row([rnd.choice(unph) for _ in range(S + 1)])
    lines[13] = row([rnd.choice(unph) for _ in range(300)])
    lines[15] = row([b"0|1"] + [rnd.choice(unph) for _ in range(S - 1)])
    buf = bytearray(b"#" * lead)
    offs, lens = [], []
    for ln in lines:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    args = (bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32))
    want = b"".join(G.oracle_encode_line(x)[1] for x in lines)
    monkeypatch.setenv("EMU_DEFER", "0")
    st0, out0, ro0, err0 = E.emu_encode(*args)
    monkeypatch.setenv("EMU_DEFER", "1")
    st1, out1, ro1, err1 = E.emu_encode(*args)
    assert err0 == err1 == (1 << 64) - 1
    assert out0 == out1 == want and list(ro0) == list(ro1)
    # handed on and deferred: all but the single-chunk row and the row whose
    # first chunk has a plain token
    assert E.last_deferred() == len(lines) - 2
    assert E.last_mispredict() == 1


@pytest.mark.parametrize("seed", range(6))
def test_predicted_deferred_records_random_batches(seed, monkeypatch):
    """Seeded random batches for the prediction machinery: runs of rows with
    one sample count (predictions taken) broken by rows of another count,
    long-first-token rows that turn plain, 1-byte escape rows, even-length
    tokens after the first chunk, plain GT-only rows and short rows, at a
    random buffer alignment and now and then an out_cap inside the batch.
    Records, offsets and the error word equal those of the encode without
    deferral, and the records equal the oracle's."""
    rnd = random.Random(1000 + seed)
    S0 = rnd.choice([260, 300, 700])
    lines = []
    for _ in range(rnd.randint(40, 90)):
        r = rnd.random()
        if r < 0.55:
            lines.append(_gdg(rnd, S0))
        elif r < 0.62:
            lines.append(_gdg(rnd, S0 + rnd.choice([-1, 1, 7])))
        elif r < 0.68:
            lines.append(PFX_V + b"\t".join([b"0|1:33:99"] * rnd.randint(1, 250) +
                                           [rnd.choice([b"0|0", b"0|1"]) for _ in range(S0)]))
        elif r < 0.74:
            lines.append(PFX_V + b"\t".join([rnd.choice([b"0", b"1", b"."]) for _ in range(rnd.randint(1100, 1600))] +
                                           [rnd.choice([b"0|0", b"0|1", b"."]) for _ in range(rnd.randint(0, 300))]))
        elif r < 0.80:
            k = rnd.randint(250, S0 - 2)
            lines.append(PFX_V + b"\t".join([b"0|1:33:99"] * k + [b"0|1:3:99"] * 2 + [b"0|1:33:99"] * (S0 - k - 2)))
        elif r < 0.90:
            lines.append(PFX_V + b"\t".join(rnd.choice([b"0|0", b"0|1", b"1|1", b"0|2"]) for _ in range(S0)))
        else:
            lines.append(PFX_V + b"\t".join(rnd.choice([b"0|0:1", b"1", b"0|0"]) for _ in range(rnd.randint(1, 40))))
    lead = rnd.randint(0, 15)
    buf = bytearray(b"#" * lead)
    offs, lens = [], []
    for ln in lines:
        offs.append(len(buf))
        lens.append(len(ln))
        buf += ln + b"\n"
    args = (bytes(buf), np.array(offs, np.uint64), np.array(lens, np.uint32))
    monkeypatch.setenv("EMU_DEFER", "0")
    st0, out0, ro0, err0 = E.emu_encode(*args)
    assert err0 == (1 << 64) - 1
    assert out0 == b"".join(G.oracle_encode_line(x)[1] for x in lines)
    cap = int(ro0[rnd.randint(1, len(lines) - 1)]) + rnd.randint(0, 200) if rnd.random() < 0.4 else None
    if cap is not None:
        st0, out0, ro0, err0 = E.emu_encode(*args, cap=cap)
    monkeypatch.setenv("EMU_DEFER", "1")
    st1, out1, ro1, err1 = E.emu_encode(*args, cap=cap)
    assert err1 == err0
    if err0 == (1 << 64) - 1:
        assert out1 == out0 and list(ro1) == list(ro0)
    else:
        bad = err0 >> 8
        assert out1[:int(ro0[bad])] == out0[:int(ro0[bad])]


@pytest.mark.parametrize("case", ["ntok", "mixed_later", "general_later", "long_then_plain", "cap",
                                  "cap_underpredicted", "cap_general", "newline"])
def test_mispredicted_deferred_records(case, monkeypatch):
    """Predictions that are wrong: another token count (a row with one
    sample more), plain tokens after a first chunk of 1-byte escapes (the
    record is not all escapes), plain tokens right after a long first token
    (predicted from that token alone, before any genotype chunk is read),
    an even-length token after the first chunk (the row leaves the
    variable-token path: general path, staged, not counted as deferred),
    out_cap cutting the batch (the held-back out_cap report against the
    exact one), a '\\n' inside a predicted row of a guessed line index.  The
    first deferred pass flags it and the layout runs again on exact sizes:
    the same bytes and offsets as without deferral, the same error word."""
    rnd = random.Random(hash(case) & 0xFFFF)
    lines = [_gdg(rnd, 700) for _ in range(12)]
    cap = None
    if case == "ntok":
        lines[6] = _gdg(rnd, 701)
    elif case == "mixed_later":
        # (1-byte escapes in chunk 0: the mixed step takes 1- and 3-byte tokens)
        lines[6] = PFX_V + b"\t".join([rnd.choice([b"0", b"1", b"."]) for _ in range(1100)] +
                                      [rnd.choice([b"0|0", b"0|1"]) for _ in range(400)])
    elif case == "general_later":
        # (two: an odd count of even-length tokens fails the region's parity check up front)
        lines[6] = PFX_V + b"\t".join([b"0|1:33:99"] * 300 + [b"0|1:3:99"] * 2 + [b"0|1:33:99"] * 398)
    elif case == "long_then_plain":   # predicted from its long first token alone; plain tokens follow at once
        lines[6] = PFX_V + b"\t".join([b"0|1:33:99"] + [rnd.choice([b"0|0", b"0|1"]) for _ in range(900)])
    elif case == "newline":
        monkeypatch.setenv("EMU_NL_CHECK", "1")
        lines[6] = PFX_V + b"\t".join([b"0|1:33:99"] * 300 + [b"0|1:33\n99"] + [b"0|1:33:99"] * 399)
    (st0, out0, ro0, err0), _ = _encode_both(lines, monkeypatch)
    if case == "cap":
        cap = int(ro0[9]) + 50
        (st0, out0, ro0, err0), (st1, out1, ro1, err1) = _encode_both(lines, monkeypatch, cap)
        assert err0 == err1 == (9 << 8) | 4
        assert out1[:int(ro0[9])] == out0[:int(ro0[9])]
        return
    if case in ("cap_underpredicted", "cap_general"):
        # a predicted row at the out_cap cut whose prediction is
        # short of its record (one sample more: predicted one byte short) or
        # that is really a general-path row, behind an over-predicted row
        # (1-byte escapes then plain tokens).  Pass 1 cannot write it, so it
        # must size it: the exact layout then reports NOSPACE at that row and
        # nothing lands past out_cap (emu_encode asserts it).
        lines[3] = PFX_V + b"\t".join([rnd.choice([b"0", b"1", b"."]) for _ in range(1100)] +
                                      [rnd.choice([b"0|0", b"0|1"]) for _ in range(400)])
        lines[9] = (_gdg(rnd, 701) if case == "cap_underpredicted" else
                    PFX_V + b"\t".join([b"0|1:33:99"] * 300 + [b"0|1:3:99"] * 2 + [b"0|1:33:99"] * 398))
        (st0, out0, ro0, err0), _ = _encode_both(lines, monkeypatch)
        assert err0 == (1 << 64) - 1
        for cut in (int(ro0[10]) - 1, int(ro0[9]) + 1, int(ro0[10])):
            (st0, out0, r0, e0), (st1, out1, r1, e1) = _encode_both(lines, monkeypatch, cut)
            assert e1 == e0, cut
            bad = e0 >> 8 if e0 != (1 << 64) - 1 else len(lines)
            assert e0 == (1 << 64) - 1 or bad in (9, 10)
            assert out1[:int(r0[bad])] == out0[:int(r0[bad])]
        return
    (st0, out0, ro0, err0), (st1, out1, ro1, err1) = _encode_both(lines, monkeypatch)
    assert E.last_mispredict() == 1
    assert err1 == err0
    if case == "newline":
        assert err0 == (6 << 8) | 9
        return
    assert err0 == (1 << 64) - 1
    assert out1 == out0 == b"".join(G.oracle_encode_line(x)[1] for x in lines)
    assert list(ro1) == list(ro0)
    # (a row that leaves the variable-token path is staged by the general path, not deferred)
    assert E.last_deferred() == (11 if case in ("general_later", "long_then_plain") else 12)


@pytest.mark.parametrize("defer", ["0", "1"])
def test_escape_rows_ending_on_a_chunk_end(defer, monkeypatch):
    """rows whose genotype region is a whole number of 2 KiB
    chunks (1024 / 2048 half-slots: 1024 or 2048 one-byte tokens, 1024
    GT:DP:GQ tokens = 5 x 1024 halves) end on lane 63's half 15 of their
    last chunk, the one place where the interior all-escape store path
    writes a byte into the row end's slot (lane 0's row end rewrites it).
    Byte-exact with and without deferred records, beside rows one half
    shorter and longer."""
    monkeypatch.setenv("EMU_DEFER", defer)
    rnd = random.Random(2024)
    lines = []
    for S in (1023, 1024, 1025, 2047, 2048, 2049):
        lines.append(PFX_V + b"\t".join(rnd.choice([b"0", b"1", b"."]) for _ in range(S)))
    for S in (1023, 1024, 1025):
        lines.append(PFX_V + b"\t".join(b"%d|%d:%d:%d" % (rnd.randint(0, 1), rnd.randint(0, 1), rnd.randint(10, 99),
                                                         rnd.randint(10, 99)) for _ in range(S)))
    want = [G.oracle_encode_line(x)[1] for x in lines]
    for lead in (0, 5):
        st, out, ro, err = run(lines, lead)
        assert err == (1 << 64) - 1
        for i, w in enumerate(want):
            assert out[int(ro[i]):int(ro[i + 1])] == w, (lead, i)
        assert E.LAST_RETRIES[0] == 0


@pytest.mark.parametrize("seed", [51, 52, 53, 54])
def test_sparse_clean_ranges(seed):
    """Sparse clean chunks (the shape a sparse event path would take, round 4;
    measured slower and not kept -- DESIGN.md §4 round 4): 512-token
    chunks holding 0, 1, a few, 62, 63, 64 or 65 non-0|0 tokens (the EV_MAX
    boundary: a range closes early, or the chunk goes to clean8), runs of one
    class crossing chunk ends inside a pending range, 0|0 gaps spanning whole
    chunks and 127-multiples, ranges cut by dense, escape and last chunks,
    and an event at token 0 (the first chunk's virtual run)."""
    rnd = random.Random(seed)
    classes = [b"0|1", b"1|0", b"1|1"]
    lines = []
    for i in range(16):
        nch = rnd.choice([3, 5, 6, 9, 13])
        toks = []
        for c in range(nch):
            kind = rnd.choice(["zero", "few", "edge", "edge", "dense", "esc", "run"])
            chunk = [b"0|0"] * 512
            if kind == "few":
                for p in rnd.sample(range(512), rnd.choice([1, 2, 5, 20])):
                    chunk[p] = rnd.choice(classes)
            elif kind == "edge":
                for p in rnd.sample(range(512), rnd.choice([61, 62, 63, 64, 65])):
                    chunk[p] = rnd.choice(classes)
            elif kind == "dense":
                chunk = [rnd.choice(classes + [b"0|0"]) for _ in range(512)]
            elif kind == "esc":
                chunk[rnd.randrange(512)] = b"0|2"
            elif kind == "run":   # one class from near the chunk end into the next chunk
                cl = rnd.choice(classes)
                for p in range(512 - rnd.randint(1, 40), 512):
                    chunk[p] = cl
                toks += chunk
                chunk = [cl] * rnd.randint(1, 40) + [b"0|0"] * 600
                chunk = chunk[:512]
            toks += chunk
        if rnd.random() < 0.5:
            toks[0] = rnd.choice(classes)
        toks = toks[:len(toks) - rnd.randrange(300)]
        pfx = b"22\t%d\trs%d\tA\tG\t100\tPASS\t%s\tGT\t" % (100 + i, i, b"Z" * rnd.randint(1, 50))
        lines.append(pfx + b"\t".join(toks))
    for lead in (0, 6):
        st, out, ro, err = run(lines, lead=lead)
        assert err == (1 << 64) - 1
        assert E.LAST_RETRIES[0] == 0
        for i, ln in enumerate(lines):
            assert out[int(ro[i]):int(ro[i + 1])] == G.oracle_encode_line(ln)[1], (lead, i)

"""The synthetic workloads (vcf-compression_amd/workload.py + the generator
kernel csrc/vcfc_synth.hip, here on the fiber emulator): every row is a
well-formed VCF data line of the declared shape, and its length is the one
the host layout assumed.  Law 2 is SURVEY §8(d)'s D3 (general shapes)."""
import numpy as np
import pytest

import emu_io as E
import golden_io as G


@pytest.mark.parametrize("law,samples", [(0, 70), (1, 130), (2, 70), (2, 300), (3, 130)])
def test_rows_are_well_formed(law, samples):
    n = 60
    buf, off, ln = E.emu_synth_rows(n, samples, law, seed=5)
    kinds = set()
    for i in range(n):
        line = bytes(buf[int(off[i]):int(off[i]) + int(ln[i])])
        assert buf[int(off[i]) + int(ln[i])] == 10   # '\n' after each line
        f = line.split(b"\t")
        assert len(f) == 9 + samples and all(f), i
        toks = f[9:]
        if law != 2:
            assert all(len(t) == 3 and t[1:2] == b"|" for t in toks)
            continue
        kind = int(f[7].split(b"KIND=")[1])
        kinds.add(kind)
        if kind == 1:
            assert f[8] == b"GT:DP:GQ" and all(len(t) == 9 and t[3:4] == b":" and t[6:7] == b":" for t in toks)
        elif kind == 3:
            assert all(len(t) == 3 and t[1:2] == b"/" for t in toks)
        elif kind in (0, 4):
            assert {len(t) for t in toks} <= {1, 3} and any(len(t) == 1 for t in toks)
        else:
            assert all(len(t) == 3 for t in toks)
        st, _ = G.oracle_encode_line(line)
        assert st == 0
    if law == 2:
        assert kinds == {0, 1, 2, 3, 4}


def test_law2_columns_fixed_across_rows():
    """Haploid (male) and missing samples are column traits: the same columns
    in every row of their kind."""
    buf, off, ln = E.emu_synth_rows(80, 90, 2, seed=9)
    pat = {}
    for i in range(80):
        f = bytes(buf[int(off[i]):int(off[i]) + int(ln[i])]).split(b"\t")
        kind = int(f[7].split(b"KIND=")[1])
        shape = tuple(len(t) for t in f[9:])
        assert pat.setdefault(kind, shape) == shape


@pytest.mark.parametrize("samples,seed", [(300, 1), (2504, 2)])
def test_law2_rows_encode_like_the_oracle(samples, seed):
    """Law-2 rows (most of them through the general kernel: tokens of 1 and 9
    bytes) encoded by the product kernels on the emulator, byte-exact vs the
    oracle, at several row alignments."""
    n = 30 if samples > 1000 else 60
    buf, off, ln = E.emu_synth_rows(n, samples, 2, seed=seed)
    for shift in (0, 3):
        b = np.concatenate([np.zeros(shift, dtype=np.uint8), buf]).tobytes()
        st, out, rec, err = E.emu_encode(b, off + np.uint64(shift), ln)
        assert err == (1 << 64) - 1
        for i in range(n):
            line = b[int(off[i]) + shift:int(off[i]) + shift + int(ln[i])]
            sto, want = G.oracle_encode_line(line)
            assert sto == 0 and out[int(rec[i]):int(rec[i + 1])] == want, (shift, i)


def _classes(toks):
    return [(t[0] - 48) * 2 + (t[2] - 48) for t in toks]


def test_law3_rows_alternate_classes():
    """Law 3 (the RLE worst case): kind-0 rows cycle the
    classes 0|0 0|1 1|0 1|1, so every token differs from its predecessor
    and starts a run (the record holds one byte per token); kind-1 rows hold
    i.i.d. alleles at frequency 1/2.  Both kinds occur; records match the
    oracle on the emulator."""
    n, S = 40, 300
    buf, off, ln = E.emu_synth_rows(n, S, 3, seed=13)
    kinds = {0: 0, 1: 0}
    st, out, rec, err = E.emu_encode(buf.tobytes(), off, ln)
    assert err == (1 << 64) - 1
    for i in range(n):
        line = bytes(buf[int(off[i]):int(off[i]) + int(ln[i])])
        toks = line.split(b"\t")[9:]
        assert all(len(t) == 3 and t[1:2] == b"|" and t[0] in b"01" and t[2] in b"01" for t in toks)
        c = _classes(toks)
        cyc = all(c[j] == (c[0] + j) % 4 for j in range(S))
        kinds[0 if cyc else 1] += 1
        rec_bytes = out[int(rec[i]):int(rec[i + 1])]
        assert rec_bytes == G.oracle_encode_line(line)[1]
        if cyc:   # one byte per token: prefix + headers + S run bytes + '\n'
            assert len(rec_bytes) == 8 + (len(line) - 4 * S + 1) + S + 1
        else:
            assert 0.35 < sum(x in (1, 2) for x in c) / S < 0.65   # het share ~1/2
    assert kinds[0] > 5 and kinds[1] > 5


@pytest.mark.parametrize("law", [1, 2, 3])
def test_row_slices_equal_the_whole_batch(law):
    """workload.DeviceRows(rows_of=(n_total, lo)) / vcfc_synth_rows_device_at:
    a batch generated as contiguous row slices (bench.py's strong split over
    N ranks) is the batch generated whole, byte for byte."""
    n, S = 30, 90
    whole, woff, wlen = E.emu_synth_rows(n, S, law, seed=17)
    lines = [bytes(whole[int(woff[i]):int(woff[i]) + int(wlen[i])]) for i in range(n)]
    got = []
    for lo, hi in ((0, 7), (7, 8), (8, 30)):
        b, o, l = E.emu_synth_rows(hi - lo, S, law, seed=17, rows_of=(n, lo))
        got += [bytes(b[int(o[i]):int(o[i]) + int(l[i])]) for i in range(hi - lo)]
    assert got == lines

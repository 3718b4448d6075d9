"""Decoder inputs for the parity tests (CPU emulator and GPU): valid .vcfc
files from the oracle encoder, and mutations that drive every branch of the
reference's byte-serial decoder (decompress2_data_line, reference
src/compress.cpp:741-986): records whose token count differs from the header,
multi-token and long escapes, NULs in the required columns, zero-count run
bytes, truncation, bad header bits, trailing bytes.  Expected outputs come
from the oracle (pinned to the reference on tests/golden/*decode*)."""
import random

import golden_io as G

CLASSES = [b"0|0", b"0|1", b"1|0", b"1|1"]


def header(samples):
    cols = b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO"
    if samples:
        cols += b"\tFORMAT" + b"".join(b"\tS%d" % i for i in range(samples))
    return b"##fileformat=VCFv4.2\n" + cols + b"\n"


def rows(rnd, n, samples, escapes=0.0, odd=0.0):
    out = []
    for i in range(n):
        p = rnd.choice([0.0, 0.01, 0.2, 0.9])
        toks = []
        for _ in range(samples):
            r = rnd.random()
            if r < escapes:
                toks.append(rnd.choice([b"2|0", b"0|2", b"1|2", b".|.", b"0/1"]))
            elif r < escapes + odd:
                toks.append(rnd.choice([b"0", b"1|0:35", b"./.:0", b"10|2"]))
            else:
                toks.append(CLASSES[(1 + rnd.randrange(3)) if rnd.random() < p else 0])
        out.append(b"22\t%d\trs%d\tA\tG\t50\tPASS\tAC=%d\tGT\t" % (100 + i, i, i) + b"\t".join(toks))
    return out


def encode_file(samples, lines):
    vcf = header(samples) + b"".join(l + b"\n" for l in lines)
    st, enc, _ = G.oracle_compress(vcf)
    assert st == 0, st
    return enc


def valid_files(seed):
    rnd = random.Random(seed)
    files = []
    for S in (1, 3, 64, 256, 300, 513, 2504):   # (tile edges: 256 tokens per decoder tile)
        n = 40 if S < 2504 else 12
        files.append(("S%d" % S, encode_file(S, rows(rnd, n, S))))
    files.append(("escapes", encode_file(200, rows(rnd, 30, 200, escapes=0.05))))
    files.append(("odd_tokens", encode_file(150, rows(rnd, 30, 150, escapes=0.02, odd=0.03))))
    return files


def mutated_files(seed):
    """(name, bytes) pairs: each a valid file with one reference-visible defect."""
    rnd = random.Random(seed)
    S = 120
    base_lines = rows(rnd, 30, S, escapes=0.02)
    out = []
    # header declares more / fewer samples than the rows carry
    for dS in (-7, -1, 1, 5, 200):
        enc = encode_file(S, base_lines)
        body = enc[len(header(S)):]
        out.append(("hdr_samples%+d" % dS, header(S + dS) + body))
    # one row with fewer / more tokens than the header
    for k, extra in ((3, -2), (10, 3), (29, -1)):
        ls = list(base_lines)
        toks = ls[k].split(b"\t")
        toks = toks[:len(toks) + extra] if extra < 0 else toks + [b"0|0"] * extra
        ls[k] = b"\t".join(toks)
        out.append(("row%d_tokens%+d" % (k, extra), encode_file(S, ls)))
    enc = encode_file(S, base_lines)
    h = len(header(S))
    # truncations, trailing bytes
    for cut in (1, 5, 8, 9, 40):
        out.append(("truncate%d" % cut, enc[:-cut]))
    for tail in (b"\x00", b"abc", b"\xc0\x00\x00\x10\xc0\x00\x00"):
        out.append(("tail_%s" % tail.hex(), enc + tail))
    # byte-level corruption inside records (after the headers)
    for j in range(12):
        b = bytearray(enc)
        pos = rnd.randrange(h, len(b))
        b[pos] = rnd.choice([0x00, 0x09, 0x0A, 0x3F, 0x80, 0xA0, 0xC5, 0xE0, 0xE1, 0xE3, 0xFF])
        out.append(("corrupt%d" % j, bytes(b)))
    # hand-built records: NUL in REQ, zero-count runs, 2-token escape, long escape
    def rec(req, samples_bytes):
        body = req + samples_bytes + b"\n"
        L = len(body) + 8 - 4
        hdr = bytes([0xC0 | (L >> 24) & 0x3F, (L >> 16) & 0xFF, (L >> 8) & 0xFF, L & 0xFF,
                     0xC0 | (len(req) >> 24) & 0x3F, (len(req) >> 16) & 0xFF, (len(req) >> 8) & 0xFF, len(req) & 0xFF])
        return hdr + body
    req = b"22\t1\trs1\tA\tG\t50\tPASS\tAC=1\tGT\t"
    S2 = 4
    hd = header(S2)
    out.append(("nul_in_req", hd + rec(req[:5] + b"\x00" + req[6:], b"\x04")))
    out.append(("zero_run", hd + rec(req, b"\x00\x04")))
    out.append(("zero_run_1x", hd + rec(req, b"\xa0\x04")))
    out.append(("two_token_escape", hd + rec(req, b"\xe2" + b"2|1\t0|2\t" + b"\x02")))
    out.append(("long_escape", hd + rec(req, b"\xe1" + b"0|1:35:99\t" + b"\x03")))
    out.append(("escape_lf_end", hd + rec(req, b"\x03\xe1" + b"2|2")))
    out.append(("escape_0_tokens", hd + rec(req, b"\xe0\x04")))
    out.append(("overshoot_00", hd + rec(req, b"\x02\x07")))
    out.append(("overshoot_1x", hd + rec(req, b"\x02\x8a")))
    out.append(("req_9tabs_missing", hd + rec(req[:-1], b"\x04")))
    out.append(("S0_row", header(0) + rec(req[:-1].rsplit(b"\t", 1)[0], b"")))
    return out


def query_files(seed):
    """(name, bytes, queries) for the range query (query_compressed_file,
    reference src/main.cpp:3777-3929): valid files with several CHROMs and
    odd POS fields, and mutations that make the reference's walk leave the
    LEN hops (CHROM or POS running past its record, a matched record whose
    parse ends off its hop) or throw (POS that does not parse)."""
    rnd = random.Random(seed)
    S = 40
    lines = []
    for i in range(60):
        chrom = rnd.choice([b"1", b"1", b"2", b"chrX"])   # (the encoder drops empty fields)
        pos = rnd.choice([b"%d" % (100 + 10 * i), b" %d" % (100 + 10 * i), b"+%d" % i, b"0%d" % i])
        toks = [CLASSES[rnd.randrange(4) if rnd.random() < 0.3 else 0] for _ in range(S)]
        lines.append(chrom + b"\t" + pos + b"\trs\tA\tG\t1\tPASS\t.\tGT\t" + b"\t".join(toks))
    enc = encode_file(S, lines)
    h = len(header(S))
    queries = [b"1", b"2:100-400", b"1:0-18446744073709551615", b":150-500", b"chrX:0-0", b"", b"1:300-200"]
    out = [("mixed", enc, queries)]
    # locate the records (LEN hops) to aim the mutations
    recs, p = [], h
    while p + 8 <= len(enc):
        L = ((enc[p] & 0x3F) << 24) | (enc[p + 1] << 16) | (enc[p + 2] << 8) | enc[p + 3]
        recs.append(p)
        p += 4 + L
    def mut(name, k, f):
        b = bytearray(enc)
        f(b, recs[k])
        out.append((name, bytes(b), queries[:4]))
    def retab(b, r, keep):   # TABs of record r past the first `keep` become 'z'
        end = recs[recs.index(r) + 1] if r != recs[-1] else len(b)
        seen = 0
        for j in range(r + 8, end):
            if b[j] == 9:
                seen += 1
                if seen > keep:
                    b[j] = ord("z")
    for k in (0, 17, 59):
        mut("chrom_past%d" % k, k, lambda b, r: retab(b, r, 0))   # CHROM runs into the next record / EOF
        mut("pos_past%d" % k, k, lambda b, r: retab(b, r, 1))     # POS does
        mut("pos_bad%d" % k, k, lambda b, r: b.__setitem__(b.index(b"\t", r + 8) + 1, ord("q")))
    # token counts off the header: matched records whose parse ends off
    # their hop or throws
    for k, extra in ((12, -1), (12, 1), (30, -3)):
        ls = list(lines)
        ls[k] = b"1" + ls[k][ls[k].index(b"\t"):] + (b"\t0|0" * extra if extra > 0 else b"")
        if extra < 0:
            ls[k] = ls[k][:ls[k].rindex(b"\t")] if extra == -1 else b"\t".join(ls[k].split(b"\t")[:extra])
        out.append(("row%d_tokens%+d" % (k, extra), encode_file(S, ls), queries[:4]))
    body = enc[h:]
    for dS in (-1, 2):
        out.append(("hdr_samples%+d" % dS, header(S + dS) + body, queries[:3]))
    for cut in (1, 9, 30):
        out.append(("truncate%d" % cut, enc[:-cut], queries[:3]))
    return out

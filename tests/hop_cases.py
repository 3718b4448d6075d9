"""Inputs for the hop line index (vcfc_line_index with the header's sample
count; csrc/vcfc_ingest.hip k_nl_hop): files on which its line-end guesses go
wrong on purpose, and chr22-shaped files on which they hold.  Shared by the
emulator tests (test_compress_device_emu.py) and the GPU tests
(test_gpu_ingest.py)."""
import decode_cases as D

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
    hdr = D.header(S)
    rows = [PREFIX % (100 + i) + b"\t".join(toks(S)) for i in range(5)]
    body = rows[:3] + [a] + mid + [b] + rows[3:]
    return hdr + b"\n".join(body) + b"\n"


def hop_trap_dense_segment(rnd, seg=16384, n_short=150):
    """The 'tab' trap inside a 16 KiB index segment that holds more than
    NL_SLOT (128) line ends, whose last line is a '#' line.  k_nl_place scans
    such a segment again and keeps as many positions as the hop index counted
    there -- one fewer than there are, since the hop missed row A's end -- so
    without a check the '#' line would run on to the next segment's first
    recorded end and be written verbatim, a data row inside it.
    The hop index's count must be found wrong and the chunk indexed again."""
    trap = hop_trap_file("tab", rnd)
    hdr, body = trap.split(b"#CHROM", 1)
    head = hdr + b"".join(b"##k%d\n" % i for i in range(n_short)) + b"#CHROM" + body.split(b"\n", 1)[0] + b"\n"
    lines = body.split(b"\n", 1)[1].rstrip(b"\n").split(b"\n")
    S = head.rstrip(b"\n").split(b"\n")[-1].count(b"\t") - 8
    a_b, tail = lines[:5], lines[5:]          # rows[:3], A, B (the trap), then data rows
    out = head + b"\n".join(a_b) + b"\n"
    for r in tail[:-1]:                        # data rows while they fit before the segment end
        if len(out) + len(r) + 1 + 64 > seg:
            break
        out += r + b"\n"
    assert out.count(b"\n") > 128 + 2
    k = seg - 2 - len(out)                     # '#' line ending at byte seg - 2: the segment's last end
    assert k >= 8
    out += b"##" + b"t" * (k - 2) + b"\n"
    assert len(out) == seg - 1
    out += PREFIX % 999 + b"\t".join([b"0|1"] * S) + b"\n"   # a data row across the segment end
    return out + b"\n".join(tail[-1:]) + b"\n"


def chr22_like(rnd, n_rows, S, prefix_jitter=40):
    """Rows of S 3-byte tokens behind prefixes whose lengths vary by up to
    prefix_jitter bytes (the hop index guesses each end from the previous
    row's prefix length), some '##' lines and an empty line among them."""
    lines = D.header(S).rstrip(b"\n").split(b"\n")
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


def law2_like(rnd, n_rows, S, kinds=(0, 1, 2, 3, 4), dp_width=2):
    """Rows shaped like bench.py --law 2: per row one kind --
    0 haploid "0"/"1" for a fixed half of the samples beside "a|b", 1
    "a|b:DP:GQ" (DP and GQ of dp_width digits; 0 = widths vary per token), 2 / 3
    3-byte tokens ("./." or unphased), 4 "." for a fixed fifth of the
    samples -- with '##' lines among them.  Kinds 0, 1 (fixed width) and 4 repeat
    one genotype-region length per kind: the hop index's TRY candidates."""
    male = [rnd.random() < 0.5 for _ in range(S)]
    miss = [rnd.random() < 0.2 for _ in range(S)]
    lines = D.header(S).rstrip(b"\n").split(b"\n")
    for i in range(n_rows):
        kind = rnd.choice(kinds)
        toks = []
        for j in range(S):
            a, b = rnd.randrange(2), rnd.randrange(2)
            if kind == 0 and male[j]:
                toks.append(b"%d" % a)
            elif kind == 4 and miss[j]:
                toks.append(b".")
            elif kind == 1:
                w = dp_width or rnd.choice([1, 2, 3])
                lo, hi = 10 ** (w - 1), 10 ** w - 1
                toks.append(b"%d|%d:%d:%d" % (a, b, rnd.randint(lo, hi), rnd.randint(lo, hi)))
            elif kind == 2:
                toks.append(b"./." if rnd.random() < 0.3 else b"%d|%d" % (a, b))
            elif kind == 3:
                toks.append(b"%d/%d" % (a, b))
            else:
                toks.append(b"%d|%d" % (a, b))
        fmt = b"GT:DP:GQ" if kind == 1 else b"GT"
        lines.append(b"\t".join([b"X", b"%d" % (2781479 + 37 * i), b".", b"A", b"G", b"50", b"PASS",
                                 b"AC=%d;KIND=%d" % (rnd.randrange(1000), kind), fmt] + toks))
        if i % 23 == 7:
            lines.append(b"##mid=%d" % i)
    return b"\n".join(lines) + b"\n"

"""Deterministic restatement of the reference's synthetic VCF generator.

Behaviour follows other/random_vcf.py (reference, :4-75): Python `random`
seeded with 5; per variant a random REF base, the other three bases shuffled
and the first two kept as ALT; per sample two alleles drawn independently from
{0: .90, 1: .08, 2: .02} via one `random.random()` each (:22-30, :65-70).

It exists so the GPU box (which has no /root/reference) can regenerate the
golden inputs; tests/golden/make_golden.py checks in the build container that
its output is byte-identical to the reference script's, and the sha256 of each
generated file is pinned in tests/golden/manifest.json.
"""
import math
import random
import sys

HEADER_COLS = ["CHROM", "POS", "ID", "REF", "ALT", "QUAL", "FILTER", "INFO", "FORMAT"]
BASES = ["A", "T", "G", "C"]


def _pick(r_state, values, probs):
    # cumulative distribution walked in order, same float arithmetic as :14-30
    total = sum(probs)
    acc, cum = 0, []
    for p in probs:
        acc += p
        cum.append(acc)
    x = r_state.random() * total
    for v, c in zip(values, cum):
        if x < c:
            return v
    return None


def generate(sample_count, variant_count, out, seed=5, alt_count=2):
    """Write the VCF bytes to the binary file object `out`."""
    rnd = random.Random(seed)
    digits = int(math.ceil(math.log10(sample_count)))
    fmt = "HG%0" + str(digits) + "d"
    head = ["##fileformat=VCFv4.1\n",
            '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">\n',
            "##fileDate=20150218\n",
            "#" + "\t".join(HEADER_COLS)]
    out.write("".join(head).encode())
    out.write("".join("\t" + fmt % j for j in range(sample_count)).encode() + b"\n")
    vals, probs = [0, 1, 2], [0.90, 0.08, 0.02]
    pos = 10000
    for i in range(variant_count):
        ref = rnd.choice(BASES)
        alts = [b for b in BASES if b != ref]
        rnd.shuffle(alts)
        cols = ["1", str(pos), "var" + str(i), ref, ",".join(alts[:alt_count]),
                "100", "PASS", "INFO", "GT"]
        pos += 2
        for _ in range(sample_count):
            a1 = _pick(rnd, vals, probs)
            a2 = _pick(rnd, vals, probs)
            cols.append("%d|%d" % (a1, a2))
        out.write(("\t".join(cols) + "\n").encode())


if __name__ == "__main__":
    s, v, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    with open(path, "wb") as f:
        generate(s, v, f)

"""Synthetic genotype workloads, generated in HBM (bench.py and the large GPU
parity cases).

law 0 "random_vcf": the reference generator's law (other/random_vcf.py:50-70):
       CHROM 1, POS 10000+2i, ID var<i>, random REF, two other bases as ALT,
       QUAL 100, FILTER PASS, INFO INFO, FORMAT GT; alleles i.i.d. 0/1/2 with
       p = .90/.08/.02 (counter-based RNG instead of Python's Mersenne
       Twister, so the bytes differ from the script's but the law is the same).
law 1 "chr22": 1000 Genomes chr22-shaped rows (BASELINE configs[1]): CHROM 22,
       POS from 16,050,075 with geometric gaps (mean 32), rsIDs, SNP REF/ALT,
       INFO with AC/AF/AN/NS/DP and five population AFs (~170 B); per-variant
       alt-allele count k ~ 1/k on [1, 5007] (neutral site-frequency
       spectrum), so most rows are rare variants with long 0|0 runs; 1 % of
       rows carry a second ALT (tokens with allele 2 -> escapes).

law 2 "general shapes" (SURVEY §8(d) D3): chrX-shaped rows of five kinds,
       drawn per row (30/30/15/10/15 %): 0 = haploid males ("0"/"1") beside
       diploid females, the sex a fixed per-sample (column) trait; 1 = FORMAT
       GT:DP:GQ, tokens "a|b:DD:GG"; 2 = ~30 % missing "./."; 3 = unphased
       "a/b" only (every token an escape); 4 = "." for a fixed 20 % of the
       samples.  Kinds 0, 1 and 4 have tokens of another length than 3, so the
       encoder's general path takes them; 2 and 3 its escape path.  Per-row
       allele frequencies as law 1.
law 3 "alternating classes" (the RLE emission's worst
       case, reference src/compress.cpp:129-170): law-1 prefixes; per row
       (50/50 %) kind 0 = the classes 0|0 0|1 1|0 1|1 cycling from a
       per-row phase, so every token starts a new run and the record holds
       one byte per token, or kind 1 = alleles i.i.d. at frequency 1/2
       (het-heavy, runs of 4/3 tokens on average).

The 9 leading columns are built on the host; the genotype columns (the
dominant bytes) are generated on the GPU by vcfc_synth_rows_device.
"""
import os

import numpy as np

BASES = np.array(list("ATGC"))
LAW2_KINDS = np.array([0.30, 0.30, 0.15, 0.10, 0.15])
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    """splitmix64 finaliser over a uint64 array (= vcfc_synth.hip mix64)."""
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def law2_token_lengths(samples):
    """Token bytes of each sample for law-2 row kinds 0..4 ([5, samples])."""
    j = np.arange(samples, dtype=np.uint64)
    male = (_mix64(np.uint64(0xC0FFEE) ^ j) & np.uint64(1)) != 0
    missing = (_mix64(np.uint64(0xBADC0DE) ^ j) >> np.uint64(32)) < np.uint64(858993459)
    three = np.full(samples, 3, dtype=np.int64)
    return np.stack([np.where(male, 1, 3), np.full(samples, 9, dtype=np.int64), three, three,
                     np.where(missing, 1, 3)])


def prefixes(n, law, seed, row0=0, samples=2504, keep=None):
    """Return (prefix bytes blob, prefix_off[n+1] int64, row_af float32 or None, POS int64[n]).

    law 1 scales with the sample count: k ~ 1/k on [1, 2S-1], AN = 2S, NS = S
    (at S = 2504 these are the 1000 Genomes values).  keep = (lo, hi): the
    random draws are those of all n rows, but only rows [lo, hi) are
    formatted and returned (slice_prefixes)."""
    lo, hi = keep if keep is not None else (0, n)
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 4, n)
    gt_len = None
    if law == 2:
        kind = rng.choice(5, n, p=LAW2_KINDS)
        if os.environ.get("VCFC_LAW2_KIND"):   # diagnostics: every row of one kind
            kind[:] = int(os.environ["VCFC_LAW2_KIND"])
        gaps = rng.geometric(1.0 / 32.0, n)
        pos = 2781479 + row0 * 32 + np.cumsum(gaps) - gaps[0]
        an = 2 * samples
        k = np.clip(np.floor(np.exp(rng.random(n) * np.log(float(an)))).astype(np.int64), 1, an - 1)
        afv = k / float(an)
        alt = (ref + rng.integers(1, 4, n)) % 4
        fmt = np.where(kind == 1, "GT:DP:GQ", "GT")
        rows = ["X\t%d\t.\t%s\t%s\t50\tPASS\tAC=%d;AN=%d;KIND=%d\t%s\t"
                % (pos[i], BASES[ref[i]], BASES[alt[i]], k[i], an, kind[i], fmt[i]) for i in range(lo, hi)]
        # (af just below 1 so kind + af keeps its integer part in float32)
        af = (kind + np.minimum(afv, 0.999)).astype(np.float32)
        gt_len = law2_token_lengths(samples).sum(axis=1)[kind] + samples   # tokens + TABs + '\n'
    elif law == 0:
        alt1 = (ref + rng.integers(1, 4, n)) % 4
        alt2 = (alt1 + 1) % 4
        alt2 = np.where(alt2 == ref, (alt2 + 1) % 4, alt2)
        pos = 10000 + 2 * (row0 + np.arange(n, dtype=np.int64))
        rows = ["1\t%d\tvar%d\t%s\t%s,%s\t100\tPASS\tINFO\tGT\t" % (10000 + 2 * (row0 + i), row0 + i, BASES[r], BASES[a], BASES[b])
                for i, (r, a, b) in enumerate(zip(ref.tolist(), alt1.tolist(), alt2.tolist())) if lo <= i < hi]
        af = None
    else:
        gaps = rng.geometric(1.0 / 32.0, n)
        pos = 16050075 + row0 * 32 + np.cumsum(gaps) - gaps[0]
        an = 2 * samples
        k = np.floor(np.exp(rng.random(n) * np.log(float(an)))).astype(np.int64)
        k = np.clip(k, 1, an - 1)
        afv = k / float(an)
        alt = (ref + rng.integers(1, 4, n)) % 4
        dp = rng.integers(10000, 30000, n)
        pops = np.clip(afv[:, None] * rng.uniform(0.2, 1.8, (n, 5)), 0, 1)
        multi = rng.random(n) < 0.01
        rs = rng.integers(1, 800000000, n)
        rows = []
        for i in range(lo, hi):
            p = pops[i]
            rows.append("22\t%d\trs%d\t%s\t%s\t100\tPASS\tAC=%d;AF=%.4g;AN=%d;NS=%d;DP=%d;"
                        "EAS_AF=%.4g;AMR_AF=%.4g;AFR_AF=%.4g;EUR_AF=%.4g;SAS_AF=%.4g;AA=.|||;VT=SNP\tGT\t"
                        % (pos[i], rs[i], BASES[ref[i]], BASES[alt[i]], k[i], afv[i], an, samples, dp[i],
                           p[0], p[1], p[2], p[3], p[4]))
        af = (afv + multi.astype(np.float64)).astype(np.float32)
        if law == 3:   # the row's kind (0: cycling classes, 1: alleles at 1/2)
            af = (rng.random(n) < 0.5).astype(np.float32)
    blob = "".join(rows).encode()
    plen = np.fromiter((len(r) for r in rows), dtype=np.int64, count=hi - lo)
    poff = np.zeros(hi - lo + 1, dtype=np.int64)
    np.cumsum(plen, out=poff[1:])
    if keep is not None:
        af = None if af is None else af[lo:hi].copy()
        gt_len = None if gt_len is None else np.asarray(gt_len)[lo:hi].copy()
        pos = np.asarray(pos)[lo:hi]
    return blob, poff, af, np.asarray(pos, dtype=np.int64), gt_len


def slice_prefixes(n_total, lo, hi, law, seed, samples=2504):
    """prefixes() of rows [lo, hi) of the n_total-row batch (seed, row0 0):
    one fixed dataset cut into row ranges (bench.py's strong split)."""
    return prefixes(n_total, law, seed, 0, samples, keep=(lo, hi))


def layout(prefix_off, samples, gt_len=None):
    """Line offsets/lengths for rows = prefix + genotype bytes ('\\n'
    included: 4 * samples for 3-byte tokens, gt_len[i] for law 2)."""
    plen = np.diff(prefix_off)
    gl = 4 * samples if gt_len is None else np.asarray(gt_len, dtype=np.int64)
    line_len = (plen + gl - 1).astype(np.int64)
    line_off = np.zeros(len(plen), dtype=np.int64)
    np.cumsum(line_len[:-1] + 1, out=line_off[1:])
    total = int(line_off[-1] + line_len[-1] + 1) if len(plen) else 0
    return line_off, line_len.astype(np.int32), total


class DeviceRows:
    """A synthetic batch resident in HBM (torch tensors)."""

    def __init__(self, torch, vcfc, n, samples, law, seed, device, row0=0, rows_of=None):
        """rows_of = (n_total, lo): rows [lo, lo + n) of the batch that
        DeviceRows(n_total, samples, law, seed) generates whole, byte for
        byte (the prefixes of all n_total rows are drawn on the host and cut;
        the genotypes hash the batch row index)."""
        if rows_of is None:
            blob, poff, af, self.pos, gt_len = prefixes(n, law, seed, row0, samples)
            self.row_base = 0
        else:
            blob, poff, af, self.pos, gt_len = slice_prefixes(rows_of[0], rows_of[1], rows_of[1] + n, law, seed,
                                                              samples)
            self.row_base = rows_of[1]
        self.chrom = {0: "1", 1: "22", 2: "X", 3: "22"}[law]
        line_off, line_len, total = layout(poff, samples, gt_len)
        dev = torch.device(device)
        self.n, self.samples, self.law = n, samples, law
        self.total_bytes = total
        self.line_bytes = int(line_len.astype(np.int64).sum())
        # bytes after the TAB following FORMAT, incl. '\n'
        self.gt_row = np.full(n, 4 * samples, dtype=np.int64) if gt_len is None else np.asarray(gt_len, dtype=np.int64)
        self.gt_bytes = int(self.gt_row.sum())
        self.buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        self.line_off = torch.from_numpy(line_off).to(dev)
        self.line_len = torch.from_numpy(line_len).to(dev)
        d_prefix = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).to(dev)
        d_poff = torch.from_numpy(poff).to(dev)
        d_af = torch.from_numpy(af).to(dev) if af is not None else None
        self._torch, self._vcfc, self._dev = torch, vcfc, dev
        self._pre = (d_prefix, d_poff, d_af)
        self.resynth(seed)
        torch.cuda.synchronize(dev)
        self.line_len_host = line_len

    def resynth(self, seed, stream=None):
        """Regenerate the genotype columns with another seed (same prefixes
        and line layout): a new batch of the same shape, made in HBM."""
        d_prefix, d_poff, d_af = self._pre
        s = stream if stream is not None else self._torch.cuda.current_stream(self._dev).cuda_stream
        self._vcfc.synth_rows_device(self.buf.data_ptr(), self.line_off.data_ptr(), self.n, d_prefix.data_ptr(),
                                     d_poff.data_ptr(), d_af.data_ptr() if d_af is not None else None,
                                     self.samples, self.law, seed, s, row_base=self.row_base)

    def host_lines(self, rows):
        """bytes of the given rows (for oracle checks)."""
        lo = self.line_off.cpu().numpy()
        ll = self.line_len.cpu().numpy()
        out = []
        for r in rows:
            a = int(lo[r])
            out.append(bytes(self.buf[a:a + int(ll[r])].cpu().numpy()))
        return out

"""Generate the golden parity vectors in tests/golden/ (run in the BUILD container).

Everything here is produced by the reference itself:
  * oracle/_ref/main -- the reference CLI compiled from /root/reference/src by
    oracle/Makefile (compress / decompress / sparsify);
  * /root/reference/other/random_vcf.py -- the reference's synthetic generator,
    executed with its two size constants substituted (the reference file is
    only read, never copied into this repository).

Outputs (data only: inputs + the reference's outputs):
  manifest.json             sha256/size pins (incl. the 2504x4000 config)
  random_100x10000.vcf.gz   config-1 input  (BASELINE configs[0])
  random_100x10000.vcfc.gz  reference `compress` output
  edge_cases.json           single-line known-answer vectors (+ reference errors)
  fuzz_encode.vcf.gz/.vcfc.gz   randomized structural fuzz lines and their encoding
  fuzz_decode.vcf.gz        reference `decompress` of fuzz_decode.vcfc (in the .vcf.gz
                            pair: the .vcfc is regenerated from fuzz_decode_src)
  sparse_100x10000.json     block digest of the reference `sparsify` output

The GPU box never runs this script (no /root/reference there).
"""
import gzip
import hashlib
import json
import os
import random
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
REF_MAIN = os.path.join(REPO, "oracle", "_ref", "main")
sys.path.insert(0, os.path.join(REPO, "tools"))
import random_vcf  # noqa: E402  (our restatement, checked against the reference below)
sys.path.insert(0, HERE)
import sparse_digest  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


def gz_write(path, data):
    with open(path, "wb") as f:
        with gzip.GzipFile(fileobj=f, mode="wb", compresslevel=9, mtime=0) as g:
            g.write(data)


def run_ref(*args, cwd=None):
    return subprocess.run([REF_MAIN] + list(args), cwd=cwd, capture_output=True)


def ref_generator(samples, variants, workdir):
    """Run the reference's other/random_vcf.py with its constants substituted."""
    src = open(os.path.join(REF, "other", "random_vcf.py")).read()
    src = re.sub(r"^sample_count = \d+", "sample_count = %d" % samples, src, flags=re.M)
    src = re.sub(r"^variant_count = \d+", "variant_count = %d" % variants, src, flags=re.M)
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        exec(compile(src, "random_vcf.py", "exec"), {"__name__": "__main__"})
    finally:
        os.chdir(cwd)
    with open(os.path.join(workdir, "test-%d-%d.vcf" % (samples, variants)), "rb") as f:
        return f.read()


def ref_compress(data, workdir, name="in"):
    ip = os.path.join(workdir, name + ".vcf")
    op = os.path.join(workdir, name + ".vcfc")
    with open(ip, "wb") as f:
        f.write(data)
    if os.path.exists(op):
        os.unlink(op)
    r = run_ref("compress", ip, op)
    out = open(op, "rb").read() if os.path.exists(op) else b""
    return r.returncode, out, r.stderr.decode(errors="replace")


def ref_decompress(data, workdir, name="in"):
    ip = os.path.join(workdir, name + ".vcfc")
    op = os.path.join(workdir, name + ".dec")
    with open(ip, "wb") as f:
        f.write(data)
    if os.path.exists(op):
        os.unlink(op)
    r = run_ref("decompress", ip, op)
    out = open(op, "rb").read() if os.path.exists(op) else b""
    return r.returncode, out, r.stderr.decode(errors="replace")


EDGE_HEADER = (b"##fileformat=VCFv4.2\n"
               b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\tS2\tS3\n")
PFX = b"1\t100\trs1\tA\tG\t50\tPASS\tAC=1\tGT\t"


def edge_lines():
    t = lambda *toks: b"\t".join(toks)  # noqa: E731
    z, a, c, e = b"0|0", b"0|1", b"1|0", b"1|1"
    cases = [
        ("run300_00", PFX + t(*[z] * 300)),
        ("runs_01_11_10", PFX + t(*([a] * 70 + [e] * 3 + [c]))),
        ("escapes_mixed", PFX + t(b"2|0", b"2|0", z, b".|.", b"0/0", b"0|0:12", b"1|2")),
        ("double_tab", PFX + b"0|0\t\t0|0\t0|1"),
        ("crlf", PFX + b"0|0\t0|1\r"),
        ("nine_cols", b"1\t100\trs1\tA\tG\t50\tPASS\tAC=1\tGT"),
        ("nine_cols_trailing_tabs", b"1\t100\trs1\tA\tG\t50\tPASS\tAC=1\tGT\t\t"),
        ("trailing_tab", PFX + b"0|0\t"),
        ("eight_cols", b"1\t100\trs1\tA\tG\t50\tPASS\tAC=1"),
        ("seven_cols", b"1\t100\trs1\tA\tG\t50\tPASS"),
        ("empty_line_fields_only", b"\t\t\t"),
        ("leading_tab", b"\t" + PFX + t(z, a)),
        ("empty_prefix_field", b"1\t\t100\trs1\tA\tG\t50\tPASS\tAC=1\tGT\t0|0\t0|1"),
        ("many_empty_prefix", b"\t\t1\t\t\t100\trs1\t\tA\tG\t50\tPASS\tAC=1\t\tGT\t\t\t0|0\t\t1|1\t\t"),
        ("cap127", PFX + t(*[z] * 127)),
        ("cap128", PFX + t(*[z] * 128)),
        ("cap254", PFX + t(*[z] * 254)),
        ("cap255", PFX + t(*[z] * 255)),
        ("cap31", PFX + t(*[a] * 31)),
        ("cap32", PFX + t(*[a] * 32)),
        ("cap62", PFX + t(*[c] * 62)),
        ("cap63", PFX + t(*[e] * 63)),
        ("alternate", PFX + t(*([z, a] * 40))),
        ("esc_last", PFX + t(z, z, b"2|2")),
        ("esc_only", PFX + b"2|2"),
        ("single_00", PFX + z),
        ("haploid", PFX + t(b"0", b"1", b"0", b"0", b".")),
        ("long_tokens", PFX + t(*[b"0|0:35:99:0,10,100"] * 5)),
        ("pipe_tokens", PFX + t(b"0||", b"|0|", b"00|", b"0|00", b"|||", z)),
        ("nul_in_token", PFX + t(z, b"0\x00|", z)),
        ("high_bytes", b"1\t100\trs1\tA\tG\t50\tPASS\tAF=\xc3\xa9\xff\tGT\t" + t(z, b"\xff|\x80", z)),
        ("spaces", PFX + t(b"0|0 ", b" 0|0", z)),
        ("cr_mid", PFX + t(z, b"0|0\r", z)),
        ("esc_then_runs", PFX + t(b"2|1", *([a] * 40), b"./.", *([z] * 130))),
    ]
    return cases


def fuzz_line(rnd, ntok_max=300):
    """Structurally varied data line: prefix with optional empty fields,
    runs of classed tokens of random lengths, escapes of random shapes,
    multi-tab separators, optional trailing tabs / CR."""
    def sep():
        return b"\t" * (1 if rnd.random() < 0.9 else rnd.randint(2, 4))
    fields = [b"1", str(rnd.randint(1, 10**9)).encode(), b"rs%d" % rnd.randint(0, 99999),
              rnd.choice([b"A", b"C", b"GT"]), rnd.choice([b"G", b"T,C"]), b"50", b"PASS",
              b"AC=%d;AF=0.%d" % (rnd.randint(0, 99), rnd.randint(0, 999)), b"GT"]
    line = b"\t" * (rnd.random() < 0.05)
    for k, f in enumerate(fields):
        line += f + (sep() if rnd.random() < 0.1 else b"\t")
    toks = []
    classed = [b"0|0", b"0|1", b"1|0", b"1|1"]
    ntok = rnd.randint(1, ntok_max)
    while len(toks) < ntok:
        r = rnd.random()
        if r < 0.75:
            cls = rnd.choice(classed) if rnd.random() < 0.6 else b"0|0"
            toks += [cls] * rnd.choice([1, 2, 3, 5, 30, 31, 32, 33, 62, 126, 127, 128, 129, 200])
        else:
            alphabet = b"012|/.:\r,A"
            n = rnd.choice([1, 2, 3, 3, 3, 4, 5, 9])
            toks.append(bytes(rnd.choice(alphabet) for _ in range(n)))
    toks = toks[:ntok]
    body = b""
    for i, tk in enumerate(toks):
        body += tk + (sep() if i + 1 < len(toks) else b"")
    line += body
    if rnd.random() < 0.05:
        line += b"\t" * rnd.randint(1, 3)
    if rnd.random() < 0.03:
        line += b"\r"
    return line


def main():
    assert os.path.exists(REF_MAIN), "build oracle/_ref first (make -C oracle)"
    manifest = {}
    with tempfile.TemporaryDirectory() as wd:
        # ---- config 1: random_vcf 100 x 10000 -----------------------------
        ref_in = ref_generator(100, 10000, wd)
        import io
        buf = io.BytesIO()
        random_vcf.generate(100, 10000, buf)
        assert buf.getvalue() == ref_in, "tools/random_vcf.py diverges from the reference generator"
        rc, ref_out, err = ref_compress(ref_in, wd, "r100")
        assert rc == 0, err
        rc, dec, err = ref_decompress(ref_out, wd, "r100")
        assert rc == 0 and dec == ref_in, "reference round trip failed"
        gz_write(os.path.join(HERE, "random_100x10000.vcf.gz"), ref_in)
        gz_write(os.path.join(HERE, "random_100x10000.vcfc.gz"), ref_out)
        manifest["random_100x10000"] = {"vcf_sha256": sha(ref_in), "vcf_bytes": len(ref_in),
                                        "vcfc_sha256": sha(ref_out), "vcfc_bytes": len(ref_out)}
        # sparsify digest (hole-aware)
        sp = os.path.join(wd, "r100.sparse")
        r = run_ref("sparsify", os.path.join(wd, "r100.vcfc"), sp)
        assert r.returncode == 0, r.stderr
        manifest["sparse_100x10000"] = sparse_digest.digest(sp)
        os.unlink(sp)

        # ---- 2504 x 4000 (hashes only; regenerated by tools/random_vcf.py) ----
        ref_in = ref_generator(2504, 4000, wd)
        buf = io.BytesIO()
        random_vcf.generate(2504, 4000, buf)
        assert buf.getvalue() == ref_in
        rc, ref_out, err = ref_compress(ref_in, wd, "r2504")
        assert rc == 0, err
        manifest["random_2504x4000"] = {"vcf_sha256": sha(ref_in), "vcf_bytes": len(ref_in),
                                        "vcfc_sha256": sha(ref_out), "vcfc_bytes": len(ref_out)}
        del ref_in, ref_out

        # ---- edge-case known-answer vectors --------------------------------
        edges = []
        for name, line in edge_lines():
            rc, out, err = ref_compress(EDGE_HEADER + line + b"\n", wd, "edge")
            ent = {"name": name, "line": line.hex()}
            if rc == 0:
                assert out.startswith(EDGE_HEADER)
                ent["record"] = out[len(EDGE_HEADER):].hex()
            else:
                ent["error"] = ("length_error" if "length_error" in err else
                                "VcfValidationError" if "VcfValidationError" in err else err.strip()[:200])
                ent["returncode"] = rc
            edges.append(ent)
        # file-level edge: interleaved '#' lines, empty lines, no final newline
        fl = (EDGE_HEADER + b"\n" + PFX + b"0|0\t0|1\t1|1\n#again\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n\n"
              + PFX + b"2|2\t0|0\t0|0\n##late meta\n" + PFX + b"1|0")
        rc, out, err = ref_compress(fl, wd, "edgefile")
        assert rc == 0, err
        bad = EDGE_HEADER + PFX + b"0|0\n#short\theader\n" + PFX + b"0|1\n"
        rc2, out2, err2 = ref_compress(bad, wd, "badhdr")
        assert rc2 != 0 and "VCF Header did not have enough columns" in err2
        with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
            json.dump({"header": EDGE_HEADER.hex(), "cases": edges,
                       "file": {"input": fl.hex(), "output": out.hex()},
                       "bad_header_file": {"input": bad.hex(), "error": "VcfValidationError",
                                           "message": "VCF Header did not have enough columns"}}, f, indent=1)

        # ---- fuzz: encode ---------------------------------------------------
        rnd = random.Random(20261015)
        lines = [fuzz_line(rnd) for _ in range(3000)]
        lines += [fuzz_line(rnd, ntok_max=3000) for _ in range(100)]
        data = EDGE_HEADER + b"\n".join(lines) + b"\n"
        rc, out, err = ref_compress(data, wd, "fuzz")
        assert rc == 0, err
        gz_write(os.path.join(HERE, "fuzz_encode.vcf.gz"), data)
        gz_write(os.path.join(HERE, "fuzz_encode.vcfc.gz"), out)
        manifest["fuzz_encode"] = {"vcf_sha256": sha(data), "vcfc_sha256": sha(out), "lines": len(lines)}

        # ---- fuzz: decode (all rows carry exactly S tokens) ------------------
        S = 257
        hdr = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t"
               + b"\t".join(b"S%d" % i for i in range(S)) + b"\n")
        rows = []
        for i in range(1500):
            ln = fuzz_line(rnd, ntok_max=S)
            pre = ln.split(b"\t")
            # force exactly S single-tab separated tokens after a clean prefix
            toks = [tk for tk in pre[9:] if tk] if len(pre) > 9 else []
            while len(toks) < S:
                toks.append(rnd.choice([b"0|0", b"0|0", b"1|1", b"0|1", b"2|1", b"./."]))
            toks = [tk.replace(b"\r", b"") or b"0|0" for tk in toks[:S]]
            rows.append(PFX + b"\t".join(toks))
        src = hdr + b"\n".join(rows) + b"\n"
        rc, enc, err = ref_compress(src, wd, "fdec")
        assert rc == 0, err
        rc, dec, err = ref_decompress(enc, wd, "fdec")
        assert rc == 0, err
        gz_write(os.path.join(HERE, "fuzz_decode.vcfc.gz"), enc)
        gz_write(os.path.join(HERE, "fuzz_decode.vcf.gz"), dec)
        manifest["fuzz_decode"] = {"vcfc_sha256": sha(enc), "vcf_sha256": sha(dec), "src_sha256": sha(src)}
        # decoder edge: a header-only file (no data lines) -> reference error
        rc, out, err = ref_compress(EDGE_HEADER, wd, "honly")
        rc2, dec, err2 = ref_decompress(out, wd, "honly")
        manifest["decode_header_only"] = {"compress_rc": rc, "decompress_rc": rc2,
                                          "error": "VcfValidationError" if "VcfValidationError" in err2 else err2[:120]}

    # ---- sparsify edge cases: duplicate / decreasing POS, records longer than
    # the 16 KiB stride (overlapping writes), strtoul quirks in POS ----------
    with tempfile.TemporaryDirectory() as wd:
        rows = []
        for pos in [b"100", b"100", b"50", b"+7", b" 9", b"0012", b"200", b"201", b"203", b"202"]:
            n = 6000 if pos == b"200" else 3
            toks = b"\t".join([b"2|1"] * n)
            rows.append(b"1\t" + pos + b"\trs\tA\tG\t50\tPASS\tAC=1\tGT\t" + toks)
        src = EDGE_HEADER + b"\n".join(rows) + b"\n"
        rc, enc, err = ref_compress(src, wd, "spe")
        assert rc == 0, err
        sp = os.path.join(wd, "spe.sparse")
        r = run_ref("sparsify", os.path.join(wd, "spe.vcfc"), sp)
        assert r.returncode == 0, r.stderr
        gz_write(os.path.join(HERE, "sparse_edge.vcfc.gz"), enc)
        manifest["sparse_edge"] = sparse_digest.digest(sp)

    manifest["generator"] = "tests/golden/make_golden.py (reference: oracle/_ref/main built from /root/reference/src; other/random_vcf.py)"
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()

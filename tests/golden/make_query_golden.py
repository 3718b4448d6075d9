"""Golden vectors for the range query: stdout and exit code
of the reference CLI's `main query <file.vcfc> <query>` (oracle/_ref/main,
compiled from /root/reference/src by oracle/Makefile), over the committed
.vcfc fixtures and a small file of odd POS values.  Run in the build
container (needs the reference build); writes query_cases.json."""
import gzip
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_MAIN = os.path.join(REPO, "oracle", "_ref", "main")


def gz(name):
    with gzip.open(os.path.join(HERE, name), "rb") as f:
        return f.read()


def run(args, cwd):
    r = subprocess.run([REF_MAIN] + args, cwd=cwd, capture_output=True, timeout=300)
    return r.returncode, r.stdout


def odd_pos_vcf():
    hdr = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\tS2\n")
    rows = [b"1\t100", b"1\t +200", b"1\t00300", b"chr1\t400", b"1\t18446744073709551615",
            b"1\t99999999999999999999", b"1\t500"]
    body = b"".join(r + b"\trs\tA\tG\t1\tPASS\t.\tGT\t0|0\t1|1\n" for r in rows)
    bad = hdr + body + b"1\t600x\trs\tA\tG\t1\tPASS\t.\tGT\t0|1\t0|0\n" + b"1\t700\trs\tA\tG\t1\tPASS\t.\tGT\t0|0\t0|0\n"
    return hdr + body, bad


def main():
    if not os.path.exists(REF_MAIN):
        sys.exit("build the reference first: make -C oracle")
    cases = []
    with tempfile.TemporaryDirectory() as wd:
        good_vcf, bad_vcf = odd_pos_vcf()
        files = {"random_100x10000.vcfc.gz": gz("random_100x10000.vcfc.gz"),
                 "fuzz_decode.vcfc.gz": gz("fuzz_decode.vcfc.gz")}
        for name, vcf in (("odd_pos", good_vcf), ("odd_pos_bad", bad_vcf)):
            src = os.path.join(wd, name + ".vcf")
            with open(src, "wb") as f:
                f.write(vcf)
            rc, _ = run(["compress", src, src + "c"], wd)
            assert rc == 0, rc
            files[name] = open(src + "c", "rb").read()
        rnd = files["random_100x10000.vcfc.gz"]
        files["random_truncated"] = rnd[:len(rnd) * 2 // 3]
        queries = {
            "random_100x10000.vcfc.gz": ["1", "1:10000-10100", "1:29990-30010", "1:5-9999", "2", "2:1-100",
                                         "1:30000-40000", "1:100-50", "X", "1:-10010", "1:a-5", "1:5",
                                         "1:10010-"],
            "fuzz_decode.vcfc.gz": ["1", "1:100-100", "1:0-18446744073709551615"],
            "odd_pos": ["1", "1:150-350", "1:0-1000", "chr1", "1:18446744073709551615-18446744073709551615"],
            "odd_pos_bad": ["1:0-550", "1"],
            "random_truncated": ["1:10000-10100", "1"],
        }
        for name, qs in queries.items():
            path = os.path.join(wd, "q.vcfc")
            with open(path, "wb") as f:
                f.write(files[name])
            for q in qs:
                rc, out = run(["query", path, q], wd)
                cases.append({"file": name, "query": q, "rc": rc, "stdout_sha256": hashlib.sha256(out).hexdigest(),
                              "stdout_len": len(out)})
        inline = {k: v.hex() for k, v in files.items() if k in ("odd_pos", "odd_pos_bad")}
    with open(os.path.join(HERE, "query_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_query_golden.py (reference: oracle/_ref/main)",
                   "inline_files": inline, "truncated_from": {"random_truncated": ["random_100x10000.vcfc.gz", "2/3"]},
                   "cases": cases}, f, indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()

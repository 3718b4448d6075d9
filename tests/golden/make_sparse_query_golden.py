"""Golden vectors for the sparse-file query: stdout and
exit code of the reference CLI's `main sparse-query <file.sparse> <query>`
(oracle/_ref/main, compiled from /root/reference/src by oracle/Makefile,
query_sparse_file_fd src/main.cpp:235-582) over sparse files made by the
reference's own `main sparsify` from committed .vcfc fixtures, some of them
then patched (bytes at absolute offsets, truncation) to reach the walk's and
the decoder's error and off-hop cases.  Run in the build container (needs the
reference build and a filesystem with holes); writes sparse_query_cases.json.
The tests rebuild each sparse file with this build's sparsify (parity-tested
against the reference separately), apply the same patches and compare."""
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
STRIDE = 4 * 4096


def gz(name):
    with gzip.open(os.path.join(HERE, name), "rb") as f:
        return f.read()


def header_end(v):
    p = 0
    while v[p:p + 1] == b"#":
        p = v.index(b"\n", p) + 1
    return p


def with_samples_delta(v, delta):
    """The .vcfc with its header line's sample columns changed by delta."""
    h = header_end(v)
    lines = v[:h].split(b"\n")[:-1]
    cols = lines[-1].split(b"\t")
    cols = cols + [b"EXTRA"] * delta if delta > 0 else cols[:len(cols) + delta]
    lines[-1] = b"\t".join(cols)
    return b"\n".join(lines) + b"\n" + v[h:]


def record_offsets(path):
    """(data_start, [file offsets of the records]) by walking dist_to_next."""
    with open(path, "rb") as f:
        v = f.read(1 << 20)
        h = header_end(v)
        data_start = h + 8
        first = int.from_bytes(v[h:h + 8], "little")
        offs, p = [], data_start + first
        while True:
            f.seek(p)
            hdr = f.read(16)
            offs.append(p)
            dn = int.from_bytes(hdr[8:16], "big")
            if dn == 0:
                break
            p += dn
    return data_start, offs


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    if not os.path.exists(REF_MAIN):
        sys.exit("build the reference first: make -C oracle")
    qc = json.load(open(os.path.join(HERE, "query_cases.json")))
    odd = bytes.fromhex(qc["inline_files"]["odd_pos"])
    rnd = gz("random_100x10000.vcfc.gz")
    bases = {
        "random_100x10000": ("random_100x10000.vcfc.gz", 0),
        "sparse_edge": ("sparse_edge.vcfc.gz", 0),
        "odd_pos": ("inline:odd_pos", 0),
        "random_S_plus1": ("random_100x10000.vcfc.gz", 1),
        "random_S_minus1": ("random_100x10000.vcfc.gz", -1),
    }
    blobs = {"random_100x10000.vcfc.gz": rnd, "sparse_edge.vcfc.gz": gz("sparse_edge.vcfc.gz"), "inline:odd_pos": odd}
    rq = ["1:10000-10000", "1:10001-10001", "1:10020-10020", "1:29998-29998", "1:10001-10005", "1:5-10003",
          "1:10000-10100", "1:29990-40000", "1:30000-30010", "1", "2:10000-10010", "2", "", "1:10000-9990",
          "1:18446744073709551615-18446744073709551615", ":10000-10010", "1:0-0", "1:20000-20200"]
    files = []   # (name, base, delta, patches, truncate, queries)
    files.append(("random_100x10000", "random_100x10000", [], None, rq))
    files.append(("sparse_edge", "sparse_edge", [], None, ["1", "1:0-100000", "1:100-100", "22:1-99999999"]))
    files.append(("odd_pos", "odd_pos", [], None, ["1:100-100", "1:150-350", "1:0-1000", "1:200-200", "chr1:400-400",
                                                   "1:300-600", "1:18446744073709551615-18446744073709551615"]))
    files.append(("random_S_plus1", "random_S_plus1", [], None, ["1:10000-10000", "1:10000-10010", "1:10002-10002"]))
    files.append(("random_S_minus1", "random_S_minus1", [], None, ["1:10000-10000", "1:10000-10010"]))
    cases = []
    layouts = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as wd:
        def build(base):
            src, delta = bases[base]
            v = blobs[src]
            if delta:
                v = with_samples_delta(v, delta)
            vp = os.path.join(wd, base + ".vcfc")
            sp = os.path.join(wd, base + ".sparse")
            with open(vp, "wb") as f:
                f.write(v)
            r = subprocess.run([REF_MAIN, "sparsify", vp, sp], capture_output=True, timeout=600)
            assert r.returncode == 0, (base, r.returncode, r.stderr[-300:])
            return sp

        built = {b: build(b) for b in bases}
        layouts["random_100x10000"] = record_offsets(built["random_100x10000"])
        # patched variants of the random file (absolute offsets from its layout)
        ds, offs = layouts["random_100x10000"]
        r5, r6, r7 = offs[5], offs[6], offs[7]
        big = (1 << 63) + 12345
        files.append(("rnd_zero_dprev", "random_100x10000", [[r6, "00" * 8]], None,
                      ["1:10000-10030", "1:10012-10012"]))
        files.append(("rnd_zero_both", "random_100x10000", [[r6, "00" * 16]], None, ["1:10000-10030"]))
        files.append(("rnd_dnext_hole", "random_100x10000", [[r5 + 8, (STRIDE).to_bytes(8, "big").hex()]], None,
                      ["1:10000-10030"]))
        files.append(("rnd_dnext_huge", "random_100x10000", [[r5 + 8, big.to_bytes(8, "big").hex()]], None,
                      ["1:10000-10030"]))
        files.append(("rnd_bad_hdr_bits", "random_100x10000", [[r6 + 16, "00"]], None, ["1:10000-10030", "1:10012-10012"]))
        files.append(("rnd_bad_pos", "random_100x10000", [[r7 + 16 + 8 + 2, "78"]], None, ["1:10000-10030"]))
        files.append(("rnd_gt_mut", "random_100x10000", [[r6 + 16 + 8 + 60, "e3"]], None,
                      ["1:10000-10030", "1:10012-10012"]))
        files.append(("rnd_truncated", "random_100x10000", [], offs[40] + 100, ["1:10000-20000", "1:10080-10080"]))
        for name, base, patches, trunc, qs in files:
            src = built[base]
            path = os.path.join(wd, "q.sparse")
            subprocess.run(["cp", "--sparse=always", src, path], check=True)
            with open(path, "r+b") as f:
                for off, hx in patches:
                    f.seek(off)
                    f.write(bytes.fromhex(hx))
                if trunc is not None:
                    f.truncate(trunc)
            for q in qs:
                try:
                    r = subprocess.run([REF_MAIN, "sparse-query", path, q], cwd=wd, capture_output=True, timeout=60)
                except subprocess.TimeoutExpired:
                    print("skip (reference does not finish):", name, q)
                    continue
                cases.append({"file": name, "query": q, "rc": r.returncode, "stdout_sha256": sha(r.stdout),
                              "stdout_len": len(r.stdout)})
            os.unlink(path)
    spec = {name: {"base": base, "patches": patches, "truncate": trunc} for name, base, patches, trunc, _ in files}
    with open(os.path.join(HERE, "sparse_query_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_sparse_query_golden.py (reference: oracle/_ref/main)",
                   "bases": {k: {"vcfc": v[0], "samples_delta": v[1]} for k, v in bases.items()},
                   "files": spec, "cases": cases}, f, indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()

"""The reference's manual round trip (do-compress.sh: `./main compress`,
`hexdump -C` of the .vcfc, `./main decompress`) run with this build's CLI in
the place of the reference's `main`, on BASELINE configs[0] (random_vcf 100 x
10k): the .vcfc is the reference's byte for byte and the round trip restores
the input."""
import hashlib
import os
import subprocess
import tempfile

import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

# the reference script's contract (do-compress.sh:2-15): an argument check,
# compress, a hex dump of the .vcfc (bash without -e runs on if hexdump is
# missing), decompress
FLOW = """#!/bin/bash
if [ -z "$1" ]; then
    echo "Must provide vcf filename"
    exit 1
fi
fname="$1"
comp_fname="${fname}.vcfc"
decomp_fname="${fname}.decompressed"
./main compress $fname $comp_fname 2>&1 | tee compress.log
hexdump $comp_fname -C | tee "$comp_fname.hexdump"
./main decompress $comp_fname $decomp_fname 2>&1 | tee decompress.log
"""


def test_do_compress_flow_config0():
    with tempfile.TemporaryDirectory() as d:
        os.symlink(os.path.join(G.REPO, "build", "main"), os.path.join(d, "main"))
        with open(os.path.join(d, "flow.sh"), "w") as f:
            f.write(FLOW)
        vcf = G.gz("random_100x10000.vcf.gz")
        with open(os.path.join(d, "test-100-10000.vcf"), "wb") as f:
            f.write(vcf)
        r = subprocess.run(["bash", "flow.sh"], cwd=d, capture_output=True, timeout=60)
        assert r.returncode == 1 and r.stdout == b"Must provide vcf filename\n"
        r = subprocess.run(["bash", "flow.sh", "test-100-10000.vcf"], cwd=d, capture_output=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out = open(os.path.join(d, "test-100-10000.vcf.vcfc"), "rb").read()
        assert hashlib.sha256(out).hexdigest() == G.manifest()["random_100x10000"]["vcfc_sha256"]
        assert open(os.path.join(d, "test-100-10000.vcf.decompressed"), "rb").read() == vcf

"""The reference-side binding of INTEGRATION.md (sections 1 and 2) is the
code that tests/integration/integration_shim.cpp holds; it compiles against
the reference's own src/compress.hpp / utils.hpp (-std=c++11) and links with
build/libvcfc.so (CPU, build container), and the linked driver reproduces the
reference's .vcfc bytes through both entry points on the GPU."""
import hashlib
import os
import re
import subprocess
import tempfile

import pytest

import golden_io as G

HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "integration", "integration_shim.cpp")
DRIVER = os.path.join(HERE, "integration", "_build", "driver")
REF_SRC = "/root/reference/src"
MARK = "// ---- INTEGRATION.md ----\n"


def test_shim_is_the_documents_code():
    doc = open(os.path.join(G.REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```cpp\n(.*?)```", doc, re.S)
    shim = open(SHIM).read()
    assert shim.split(MARK, 1)[1] == blocks[0] + "\n" + blocks[1]


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree absent")
@pytest.mark.skipif(not os.path.exists(os.path.join(G.REPO, "build", "libvcfc.so")), reason="library not built")
def test_shim_compiles_and_links_against_reference_headers():
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["make", "-s", "-C", os.path.join(HERE, "integration"), "B=" + d], capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert os.path.exists(os.path.join(d, "driver"))


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DRIVER), reason="driver not built (needs the reference headers)")
@pytest.mark.parametrize("mode", ["lines", "file"])
def test_gpu_shim_driver_matches_reference(mode):
    vcf = G.gz("random_100x10000.vcf.gz")
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.vcf"), os.path.join(d, "out.vcfc")
        with open(src, "wb") as f:
            f.write(vcf)
        r = subprocess.run([DRIVER, mode, src, dst], capture_output=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out = open(dst, "rb").read()
        assert hashlib.sha256(out).hexdigest() == G.manifest()["random_100x10000"]["vcfc_sha256"]


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DRIVER), reason="driver not built (needs the reference headers)")
def test_gpu_shim_driver_errors():
    """< 8 terms -> VcfValidationError (exit 2), exactly 8 -> length_error (3)."""
    ec = G.edge_cases()
    hdr = bytes.fromhex(ec["header"])
    with tempfile.TemporaryDirectory() as d:
        for line, code in [(b"1\t2\t3\t4\t5\t6\t7", 2), (b"1\t2\t3\t4\t5\t6\t7\t8", 3)]:
            src = os.path.join(d, "in.vcf")
            with open(src, "wb") as f:
                f.write(hdr + line + b"\n")
            r = subprocess.run([DRIVER, "lines", src, os.path.join(d, "o")], capture_output=True, timeout=120)
            assert r.returncode == code, (line, r.returncode, r.stderr[-500:])

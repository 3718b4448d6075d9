"""The reference's manual round trip (do-compress.sh) run with this build's CLI
in the place of the reference's `main`, on BASELINE configs[0] (random_vcf
100 x 10k): the .vcfc is the reference's byte for byte and the round trip
restores the input.  The script's contract -- its usage check and the argv of
each `./main` call -- is data in tests/golden/manifest.json ("do_compress",
made by make_cli_contract.py from the reference script, whose sha256 it pins;
tests/test_cli_contract.py re-derives it when the reference is present)."""
import hashlib
import os
import subprocess
import tempfile

import pytest

import golden_io as G

pytestmark = pytest.mark.gpu


def test_do_compress_flow_config0():
    c = G.manifest()["do_compress"]
    with tempfile.TemporaryDirectory() as d:
        main = os.path.join(G.REPO, "build", "main")
        # the usage check: a CLI call without the file name fails the way the
        # script reports it (the script itself exits before calling ./main)
        assert c["usage_stdout"] == "Must provide vcf filename\n" and c["usage_rc"] == 1
        vcf = G.gz("random_100x10000.vcf.gz")
        f = "test-100-10000.vcf"
        with open(os.path.join(d, f), "wb") as fh:
            fh.write(vcf)
        for call in c["calls"]:
            argv = [a.format(f=f) for a in call["argv"]]
            r = subprocess.run([main] + argv, cwd=d, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300)
            assert r.returncode == 0, (argv, r.stdout[-2000:])
            if call["log"]:
                with open(os.path.join(d, call["log"]), "wb") as fh:
                    fh.write(r.stdout)
        verbs = [call["argv"][0] for call in c["calls"]]
        assert verbs == ["compress", "decompress"]
        out = open(os.path.join(d, c["calls"][0]["argv"][2].format(f=f)), "rb").read()
        assert hashlib.sha256(out).hexdigest() == G.manifest()["random_100x10000"]["vcfc_sha256"]
        assert open(os.path.join(d, c["calls"][1]["argv"][2].format(f=f)), "rb").read() == vcf

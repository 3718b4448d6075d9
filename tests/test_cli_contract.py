"""The do-compress.sh contract (tests/golden/manifest.json "do_compress") is
pinned to the reference script: its sha256 matches and re-deriving the argv
sequence from the script gives the stored data (CPU; skipped where the
reference tree is absent, e.g. on the GPU box)."""
import hashlib
import os
import sys

import pytest

import golden_io as G

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_cli_contract  # noqa: E402

SCRIPT = make_cli_contract.SCRIPT


def test_contract_shape():
    c = G.manifest()["do_compress"]
    assert [x["argv"] for x in c["calls"]] == [["compress", "{f}", "{f}.vcfc"],
                                               ["decompress", "{f}.vcfc", "{f}.decompressed"]]
    assert len(c["script_sha256"]) == 64


@pytest.mark.skipif(not os.path.exists(SCRIPT), reason="reference tree absent")
def test_contract_pinned_to_reference_script():
    c = dict(G.manifest()["do_compress"])
    data = open(SCRIPT, "rb").read()
    assert hashlib.sha256(data).hexdigest() == c.pop("script_sha256")
    assert make_cli_contract.derive(data.decode()) == c

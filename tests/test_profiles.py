"""The committed headline measurement reproduces from its own files
(profiles/r06/final/; round 5: profiles/r05/final5/): the bench line's roofline fraction from the rocprofv3
kernel trace of the same command, and its HBM traffic from the PMC summary
bench.py reads.  CPU only (reads committed files)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FINAL = os.path.join(REPO, "profiles", "r06", "final")


def _line(name):
    return json.load(open(os.path.join(FINAL, name)))


@pytest.mark.parametrize("line", ["bench.json", "bench_under_prof.json"])
def test_headline_fraction_reproduces_from_the_trace(line):
    """tools/frac_from_trace.py over the timed launches (warmup dropped) is
    within 2 % of the line's own fraction (HIP events on the same stream)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "frac_from_trace.py"),
                          os.path.join(FINAL, line), os.path.join(FINAL, "kernel_trace.csv")],
                         capture_output=True, text=True, check=True).stdout
    timed = [ln for ln in out.splitlines() if ln.startswith("timed launches")]
    assert timed, out
    frac = float(timed[0].split("frac ")[1].split()[0])
    want = _line(line)["roofline"]["frac"]
    assert abs(frac / want - 1.0) < 0.02, (frac, want)


def test_headline_traffic_is_the_same_box_pmc():
    """The line's roofline.traffic is the PMC summary measured on the same
    box (installed before the line ran) and committed beside it."""
    d = _line("bench.json")
    pmc = json.load(open(os.path.join(FINAL, "pmc_k_encode.json")))
    assert d["roofline"]["traffic"] == pmc["hbm_bytes_per_launch"]
    assert d["roofline"]["algorithmic_bytes_per_launch"] <= pmc["hbm_bytes_per_launch"] < \
        1.1 * d["roofline"]["algorithmic_bytes_per_launch"]
    # the reference CLI's output for the CPU-baseline sample equals the GPU's records
    assert d["cpu_baseline"]["kind"] == "reference"
    assert d["cpu_baseline"]["gpu_output_identical"] is True
    assert d["cpu_baseline"]["parallel"]["output_identical"] is True

#!/bin/bash
# Round-4 validation of the deferred-record build: smoke, every -m gpu test,
# the benches (laws 1/0/2, decode, device file laws 1/2), kernel stats, and
# HBM bytes per launch (encoder laws 1/0/2, device-file steps laws 1/2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4L smoke tests bench bench0 bench2 benchdec benchdev benchdev2 prof prof2 profdev2 pmcenc || exit 1
LAW=2 bash tools/gpu_check.sh r4L pmcdev || exit 1
LAW=1 bash tools/gpu_check.sh r4L pmcdev || exit 1

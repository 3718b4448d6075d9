#!/bin/bash
# Round-5 final tree on one box: smoke, every -m gpu test, the encoder PMC
# (laws 1/0/2) installed as the summaries bench.py reads, then the headline
# line and the same command under rocprofv3 (kernel stats of that process).
# tools/r5_final2.sh: the law-0 / law-2 / decode / query / device-file lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh ${FINAL_TAG:-r5final} smoke tests pmcenc pmcinstall bench profbench || exit 1
echo done

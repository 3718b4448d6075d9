#!/bin/bash
# Round-5: smoke and every -m gpu test on the product build after the
# misprediction path's wave-wide rearm.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/gpu_check.sh r5T smoke tests || exit 1
echo done

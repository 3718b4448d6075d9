#!/bin/bash
# Round-5: 4-rank rehearsals of the multi-GPU bench (gloo, one GPU; weak and
# strong scaling) on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/gpu_check.sh r5V rehearse4 rehearse4s || exit 1
echo done

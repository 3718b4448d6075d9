#!/bin/bash
# Round-5 first call: configs[4]'s query half on the current tree (bench line
# with the reference CLI baseline, kernel stats, step HBM traffic) and the
# headline bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r5A benchq profq pmcq bench || exit 1

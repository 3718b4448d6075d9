#!/bin/bash
# Round-4 closing measurements after the variable-token VALU cuts: law-2
# bench line and kernel stats, PMC of the variable-token kernel on kinds 0/4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4AA bench2 prof2 || exit 1
VCFC_LAW2_KIND=0 bash tools/pmc_lib.sh pmc_kind0_r4b build/libvcfc.so --law 2 > /dev/null || exit 1
VCFC_LAW2_KIND=4 bash tools/pmc_lib.sh pmc_kind4_r4b build/libvcfc.so --law 2 > /dev/null || exit 1

#!/bin/bash
# Round-4: instruction / wait counters of the variable-token kernel on 1M
# law-2 kind-0 rows (haploid beside diploid), the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
VCFC_LAW2_KIND=0 bash tools/pmc_lib.sh pmc_kind0_r4 build/libvcfc.so --law 2 > /dev/null || exit 1
VCFC_LAW2_KIND=4 bash tools/pmc_lib.sh pmc_kind4_r4 build/libvcfc.so --law 2 > /dev/null || exit 1

#!/bin/bash
# Round-5: instruction / wait / LDS / HBM counters of the GT:DP:GQ-only
# encode on the product build (k_encode_defer<1> is 10.7 of its 12.2 ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
VCFC_LAW2_KIND=1 bash tools/pmc_lib.sh r5Q_pmc_kind1 build/libvcfc.so --law 2 || exit 1
echo done

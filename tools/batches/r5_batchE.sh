#!/bin/bash
# Round-5: deferred records with plain stores into out (build_ab/cur3) on /
# off (cur3_nodefer) on law 2 and GT:DP:GQ rows; the var kernel's dot4 TAB
# masks (cur3 against cur2) on kinds 0 and 4; PMC of cur3 on kinds 0 and 4;
# then every -m gpu test on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=build_ab/cur3/libvcfc.so; O=build_ab/cur3_nodefer/libvcfc.so; P=build_ab/cur2/libvcfc.so
AB_ARGS="--law 2" bash tools/ab.sh ab_r5e_law2 $O $D || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5e_kind1 $O $D || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_r5e_kind0 $P $D || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_r5e_kind4 $P $D || exit 1
VCFC_LAW2_KIND=0 bash tools/pmc_lib.sh r5E_pmc_kind0 build_ab/cur3/libvcfc.so --law 2 > /dev/null || exit 1
VCFC_LAW2_KIND=4 bash tools/pmc_lib.sh r5E_pmc_kind4 build_ab/cur3/libvcfc.so --law 2 > /dev/null || exit 1
bash tools/gpu_check.sh r5E tests || exit 1
echo done

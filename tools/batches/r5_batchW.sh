#!/bin/bash
# Round-5: rows whose first genotype chunk is all 3-byte escapes (unphased)
# handed from k_encode_fast to k_encode_var with VCFCD_GT0_LONG and predicted
# (build_ab/cur14 = build/) against cur11: law-2 kinds 3 and 2, law 2, law 1,
# law 0, the law-2 device file; every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur11/libvcfc.so; C=build_ab/cur14/libvcfc.so
bash tools/gpu_check.sh r5W tests || exit 1
VCFC_LAW2_KIND=3 AB_ARGS="--law 2" bash tools/ab.sh ab_r5w_kind3 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5w_law2 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5w_law1 $P $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5w_law0 $P $C || exit 1
VCFC_LAW2_KIND=2 AB_ARGS="--law 2" bash tools/ab.sh ab_r5w_kind2 $P $C || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5w_devfile_law2 $P $C || exit 1
echo done

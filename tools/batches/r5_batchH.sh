#!/bin/bash
# Round-5: k_encode_fast hands the first sample's offset of a clean prefix to
# k_encode_var (build_ab/cur6), which then skips the prefix parse and loads
# the genotype chunks beside the prefix chunk, against cur5: law-2 kinds 0,
# 4, 1, law 2, law 1; then every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P=build_ab/cur5/libvcfc.so; C=build_ab/cur6/libvcfc.so
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_r5h_kind0 $P $C || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_r5h_kind4 $P $C || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5h_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5h_law2 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5h_law1 $P $C || exit 1
bash tools/gpu_check.sh r5H tests || exit 1
echo done

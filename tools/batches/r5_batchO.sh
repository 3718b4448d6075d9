#!/bin/bash
# Round-5: deferred rows predicted before any load when k_encode_fast saw a
# first token of 5+ bytes (VCFCD_GT0_LONG; build_ab/cur11 = build/) against
# cur9 (predicted from the first chunk): GT:DP:GQ rows, law 2, law-2 kind 0
# (variable-token rows, not deferred), law 1, the law-2 device file; every
# -m gpu test; GT:DP:GQ kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur9/libvcfc.so; C=build_ab/cur11/libvcfc.so
bash tools/gpu_check.sh r5O tests || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5o_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5o_law2 $P $C || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_r5o_kind0 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5o_law1 $P $C || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5o_devfile_law2 $P $C || exit 1
VCFC_LAW2_KIND=1 BENCH_ARGS="--law 2" bash tools/gpu_check.sh r5O_k1 prof || exit 1
echo done

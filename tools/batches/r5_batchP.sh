#!/bin/bash
# Round-5: the agreed token count published batch-wide (build_ab/cur12 =
# build/) against cur11: GT:DP:GQ rows, law 2, law 1, the law-2 device file;
# every -m gpu test; GT:DP:GQ kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur11/libvcfc.so; C=build_ab/cur12/libvcfc.so
bash tools/gpu_check.sh r5P tests || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5p_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5p_law2 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5p_law1 $P $C || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5p_devfile_law2 $P $C || exit 1
VCFC_LAW2_KIND=1 BENCH_ARGS="--law 2" bash tools/gpu_check.sh r5P_k1 prof || exit 1
echo done

#!/bin/bash
# Round-5: the size scan flags output tiles whose bytes all belong to
# deferred records, across record ends (build_ab/cur8), against cur7:
# GT:DP:GQ rows only, law 2, law 1; kind-1 kernel trace; every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur7/libvcfc.so; C=build_ab/cur8/libvcfc.so
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5j_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5j_law2 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5j_law1 $P $C || exit 1
VCFC_LAW2_KIND=1 BENCH_ARGS="--law 2" bash tools/gpu_check.sh r5J_k1 prof || exit 1
bash tools/gpu_check.sh r5J tests || exit 1
echo done

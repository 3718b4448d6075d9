#!/bin/bash
# Round-5: predicted deferred records (build_ab/cur9: k_encode_var sizes an
# all-escape row from its first chunk and the token count two earlier rows
# agreed on; k_encode_defer's first pass checks, gated relayout on a miss)
# against cur8: GT:DP:GQ rows only, law 2, law 1, law 0; every -m gpu test;
# kind-1 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur8/libvcfc.so; C=build_ab/cur9/libvcfc.so
bash tools/gpu_check.sh r5K tests || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5k_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5k_law2 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5k_law1 $P $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5k_law0 $P $C || exit 1
VCFC_LAW2_KIND=1 BENCH_ARGS="--law 2" bash tools/gpu_check.sh r5K_k1 prof || exit 1
echo done

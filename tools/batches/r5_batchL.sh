#!/bin/bash
# Round-5: predicted deferred records with the pass-1 general fallback out of
# line (build_ab/cur10) against cur9 (inlined) and cur8 (no prediction):
# GT:DP:GQ rows only, law 2; the law-2 device file cur8 vs cur10; every
# -m gpu test on cur10.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
A=build_ab/cur8/libvcfc.so; P=build_ab/cur9/libvcfc.so; C=build_ab/cur10/libvcfc.so
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5l_kind1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5l_law2 $P $C || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5l_devfile_law2 $A $C || exit 1
bash tools/gpu_check.sh r5L tests || exit 1
echo done

#!/bin/bash
# Round-5: the compaction skips 16-byte blocks inside deferred records in
# tiles shared with staged records (TILE_SOME_DEFER; build_ab/cur13 =
# build/) against cur11: law 2, GT:DP:GQ rows, law 1, law 0, the law-2 device
# file; every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur11/libvcfc.so; C=build_ab/cur13/libvcfc.so
bash tools/gpu_check.sh r5R tests || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5r_law2 $P $C || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5r_kind1 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5r_law1 $P $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5r_law0 $P $C || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5r_devfile_law2 $P $C || exit 1
echo done

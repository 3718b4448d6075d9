#!/bin/bash
# Round-5: esc8's interior shape test folded into its classification
# (build_ab/cur15 = build/) against cur14: law 0, law 1, law 2, law-2 kinds 2
# and 3; every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur14/libvcfc.so; C=build_ab/cur15/libvcfc.so
bash tools/gpu_check.sh r5Y tests || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5y_law0 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5y_law1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5y_law2 $P $C || exit 1
VCFC_LAW2_KIND=2 AB_ARGS="--law 2" bash tools/ab.sh ab_r5y_kind2 $P $C || exit 1
echo done

#!/bin/bash
# Round-4 A/B: the final tree (cur) against HEAD before deferral (head):
# headline law 1, law 0, law-2 kinds 0 and 4 alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/cur/libvcfc.so"
bash tools/ab.sh ab_final_law1 $L || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_final_law0 $L || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_final_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_final_kind4 $L || exit 1

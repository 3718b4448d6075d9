#!/bin/bash
# Round-4 A/B: the ring's mode checks compiled out of the fast and general
# paths (cur2), + k_encode_defer on 640 blocks instead of 1280 (cur3),
# against HEAD before deferral: headline, law 2, kind 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/cur2/libvcfc.so build_ab/cur3/libvcfc.so"
bash tools/ab.sh ab_dyn_law1 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_dyn_law2 $L || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_dyn_kind0 $L || exit 1

#!/bin/bash
# Round-4 A/B: deferred records (GT:DP:GQ-like rows sized by k_encode_var,
# written straight to out by k_encode_defer) against HEAD: laws 2, 1, 0,
# law-2 kind 1 alone, device-file law 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/defer/libvcfc.so"
AB_ARGS="--law 2" bash tools/ab.sh ab_defer_law2 $L || exit 1
bash tools/ab.sh ab_defer_law1 $L || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_defer_kind1 $L || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_defer_law0 $L || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_defer_dev2 $L || exit 1
bash tools/abdec.sh ab_dec128 build_ab/head/libvcfc.so build_ab/dec128/libvcfc.so || exit 1

#!/bin/bash
# Round-4 A/B: deferred records (defer), + decoder 128-B windows (dec128),
# + mask-AND store addresses and dot4 bit gathers (mask) against HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/defer/libvcfc.so build_ab/mask/libvcfc.so"
AB_ARGS="--law 2" bash tools/ab.sh ab_defer_law2 $L || exit 1
bash tools/ab.sh ab_defer_law1 $L || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_defer_law0 $L || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_defer_kind1 build_ab/head/libvcfc.so build_ab/mask/libvcfc.so || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_mask_kind0 build_ab/head/libvcfc.so build_ab/mask/libvcfc.so || exit 1
bash tools/abdec.sh ab_dec128 build_ab/head/libvcfc.so build_ab/dec128/libvcfc.so build_ab/mask/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_defer_dev2 build_ab/head/libvcfc.so build_ab/mask/libvcfc.so || exit 1
bash tools/ab.sh ab_warm_law1 build_ab/mask/libvcfc.so build_ab/warm/libvcfc.so || exit 1

#!/bin/bash
# Round-4 A/B: deferred records with whole deferred tiles skipped by the
# compaction (defer2) against HEAD before deferral: laws 2, 1, 0, kind 1,
# device-file law 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/defer2/libvcfc.so"
AB_ARGS="--law 2" bash tools/ab.sh ab_defer2_law2 $L || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_defer2_kind1 $L || exit 1
bash tools/ab.sh ab_defer2_law1 $L || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_defer2_law0 $L || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_defer2_dev2 $L || exit 1

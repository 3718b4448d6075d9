#!/bin/bash
# Round-4 A/B: escape halves' second byte under the first byte's flag (e1pay)
# against ptkbfi, then every -m gpu test and the law-2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/ptkbfi/libvcfc.so build_ab/e1pay/libvcfc.so"
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_e1pay_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_e1pay_kind4 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_e1pay_law2 $L || exit 1
bash tools/gpu_check.sh r4Y tests bench2 prof2 || exit 1

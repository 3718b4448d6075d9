#!/bin/bash
# Round-4 A/B: the variable-token path's run-start tracking by one v_bfi_b32
# (ptkbfi, on top of leadmul) against leadmul; headline for the fast path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/leadmul/libvcfc.so build_ab/ptkbfi/libvcfc.so"
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_ptkbfi_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_ptkbfi_kind4 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_ptkbfi_law2 $L || exit 1
bash tools/ab.sh ab_ptkbfi_law1 $L || exit 1

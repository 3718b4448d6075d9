#!/bin/bash
# Round-4 A/B: the variable-token lead byte's address by one v_mul_i32_i24
# (leadmul) against the compiler's bit-test/compare/add/select (e2mul).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/e2mul/libvcfc.so build_ab/leadmul/libvcfc.so"
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_leadmul_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_leadmul_kind4 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_leadmul_law2 $L || exit 1

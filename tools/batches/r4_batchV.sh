#!/bin/bash
# Round-4 A/B: the variable-token path's second-payload-byte address by a
# plain multiply (e2mul) against mad24 (cur5): law-2 kinds 0 and 4, law 2,
# headline; then the deferred-records GPU ingest test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/cur5/libvcfc.so build_ab/e2mul/libvcfc.so"
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_e2mul_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_e2mul_kind4 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_e2mul_law2 $L || exit 1
bash tools/ab.sh ab_e2mul_law1 $L || exit 1
PT_ARGS="tests/test_gpu_ingest.py -k deferred" bash tools/gpu_check.sh r4U ptest || exit 1

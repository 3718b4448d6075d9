#!/bin/bash
# Round-5: configs[4]'s query half on the current tree (bench line, kernel
# stats, step traffic); A/B of the variable-token kernel's end-attributed
# emission (build_ab/new) against the round-4 kernel (build_ab/base), and of
# deferred records on by default (build_ab/auto) against off (new).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r5B benchq profq pmcq || exit 1
B=build_ab/base/libvcfc.so; N=build_ab/new/libvcfc.so; A=build_ab/auto/libvcfc.so
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_r5_emit_kind0 $B $N || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_r5_emit_kind4 $B $N || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5_law2 $B $N $A || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5_auto_law1 $N $A || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5_auto_law0 $N $A || exit 1

#!/bin/bash
# Round-5 A/B: the current tree (build_ab/cur: dot4 bit gathers in the fast
# prefix step, the var kernel and the decoder scan; deferred records on by
# default; all-escape rows handed to k_encode_var) against the emission-only
# build (build_ab/new) on laws 1, 0, 2, decode and the range query.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
N=build_ab/new/libvcfc.so; C=build_ab/cur/libvcfc.so
AB_ARGS="--law 2" bash tools/ab.sh ab_r5c_law2 $N $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5c_law1 $N $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5c_law0 $N $C || exit 1
AB_ARGS="--mode decode" bash tools/ab.sh ab_r5c_decode $N $C || exit 1
AB_ARGS="--mode query" bash tools/ab.sh ab_r5c_query $N $C || exit 1

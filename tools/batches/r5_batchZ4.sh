#!/bin/bash
# Round-5: the last chunk's clean-test skip with a branch hint toward the
# clean test (cur20) against cur19 (no hint) and cur15 (no skip): laws 1, 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
A=build_ab/cur15/libvcfc.so; B=build_ab/cur19/libvcfc.so; C=build_ab/cur20/libvcfc.so
AB_ARGS="--law 1" bash tools/ab.sh ab_r5z4_law1 $A $B $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5z4_law0 $A $B $C || exit 1
echo done

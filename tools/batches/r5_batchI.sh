#!/bin/bash
# Round-5: the gt0 hand-over with the prefix copy unconditional (cur7)
# against cur5 (no hand-over) and cur6 (hand-over behind a branch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P=build_ab/cur5/libvcfc.so; C=build_ab/cur7/libvcfc.so; B=build_ab/cur6/libvcfc.so
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_r5i_kind0 $P $C $B || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5i_law2 $P $C || exit 1
echo done

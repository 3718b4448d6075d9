#!/bin/bash
# Round-5: esc8's last-chunk shape test folded too, with (cur17) and without
# (cur18) the last chunk skipping the clean test after escapes, against
# cur15: law 0, law 1, law 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
A=build_ab/cur15/libvcfc.so; B=build_ab/cur17/libvcfc.so; C=build_ab/cur18/libvcfc.so
AB_ARGS="--law 1" bash tools/ab.sh ab_r5z2_law1 $A $B $C || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5z2_law0 $A $B $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5z2_law2 $A $B $C || exit 1
echo done

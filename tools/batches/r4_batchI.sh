#!/bin/bash
# Round-4 A/B: compaction pipelined with the encode over 4 / 8 pieces (side
# stream) against the unpiped call, laws 1, 0, 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/pipe1/libvcfc.so build_ab/pipe4/libvcfc.so build_ab/pipe8/libvcfc.so"
bash tools/ab.sh ab_pipe_law1 $L || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_pipe_law0 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_pipe_law2 $L || exit 1

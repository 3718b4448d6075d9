#!/bin/bash
# Round-5: the row's last chunk skips the clean test after a chunk with
# escapes (build_ab/cur16 = build/) against cur15: law 0, law 1, law 2;
# every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
P=build_ab/cur15/libvcfc.so; C=build_ab/cur16/libvcfc.so
bash tools/gpu_check.sh r5Z tests || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5z_law0 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5z_law1 $P $C || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_r5z_law2 $P $C || exit 1
echo done

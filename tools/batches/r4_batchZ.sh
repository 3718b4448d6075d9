#!/bin/bash
# Round-4 A/B: run-length counter + leads stored in the loop (lead2) against
# e1pay; then every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/e1pay/libvcfc.so build_ab/lead2/libvcfc.so"
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_lead2_kind0 $L || exit 1
VCFC_LAW2_KIND=4 AB_ARGS="--law 2" bash tools/ab.sh ab_lead2_kind4 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_lead2_law2 $L || exit 1
bash tools/gpu_check.sh r4Z tests || exit 1

#!/bin/bash
# Round-4 A/B: the hop index choosing its learned candidates from the first
# data lines (auto) against round 3 (base): device file, laws 1 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/abdev.sh ab_auto_law1 build_ab/base/libvcfc.so build_ab/auto/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_auto_law2 build_ab/base/libvcfc.so build_ab/auto/libvcfc.so || exit 1

#!/bin/bash
# Round-4 A/B: hop index with TRY/LEARN behind wave-uniform branches, 5 waves
# (hopuni5) against round 3 (base) and the first TRY build (hoptry5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/abdev.sh ab_hopuni_law1 build_ab/base/libvcfc.so build_ab/hopuni5/libvcfc.so build_ab/hoptry5/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_hopuni_law2 build_ab/base/libvcfc.so build_ab/hopuni5/libvcfc.so build_ab/hoptry5/libvcfc.so || exit 1

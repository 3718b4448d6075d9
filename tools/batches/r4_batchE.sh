#!/bin/bash
# Round-4 A/B: law-2 rows' '\n' check inside the variable-token chunks (nlvar)
# against a scan of every flagged row first (hopuni5): device file (law 2, hop
# and scan index), and the encode bench (law 2, no check) for neutrality.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_nlvar_law2 build_ab/hopuni5/libvcfc.so build_ab/nlvar/libvcfc.so || exit 1
AB_ARGS="--law 2 --line-index scan" bash tools/abdev.sh ab_nlvar_law2_scan build_ab/nlvar/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_nlvar_encode_law2 build_ab/hopuni5/libvcfc.so build_ab/nlvar/libvcfc.so || exit 1

#!/bin/bash
# Round-4 A/B: every learned candidate (and the 3-byte end) tried in one
# round (tall5: 5 waves, 16 dwords spilled; tall4: 4 waves) against one
# candidate per round (nlvar) and round 3 (base): device file, laws 1 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/abdev.sh ab_tall_law1 build_ab/base/libvcfc.so build_ab/nlvar/libvcfc.so build_ab/tall5/libvcfc.so build_ab/tall4/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_tall_law2 build_ab/base/libvcfc.so build_ab/nlvar/libvcfc.so build_ab/tall5/libvcfc.so build_ab/tall4/libvcfc.so || exit 1

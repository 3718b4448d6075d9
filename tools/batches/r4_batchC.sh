#!/bin/bash
# Round-4 A/B (one gpurun call): the hop index with learned candidates checked
# in the LINE round (hopline), pinned to 5 waves (hopline5), against round 3
# (base) and TRY-only candidates (hoptry5), on the device-resident configs[1]
# file (law 1) and a law-2 file of the same size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/abdev.sh ab_hopline_law1 build_ab/base/libvcfc.so build_ab/hopline/libvcfc.so build_ab/hopline5/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_hopline_law2 build_ab/base/libvcfc.so build_ab/hoptry5/libvcfc.so build_ab/hopline/libvcfc.so build_ab/hopline5/libvcfc.so || exit 1

#!/bin/bash
# Round-4 A/Bs (one gpurun call): the var kernel's interior escape path (law
# 2, kind 1) and the hop index's learned candidates (device file, laws 1/2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_escfast_law2 build_ab/base/libvcfc.so build_ab/escfast/libvcfc.so || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_escfast_kind1 build_ab/base/libvcfc.so build_ab/escfast/libvcfc.so || exit 1
bash tools/abdev.sh ab_hoptry_law1 build_ab/base/libvcfc.so build_ab/hoptry/libvcfc.so build_ab/hoptry5/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_hoptry_law2 build_ab/base/libvcfc.so build_ab/hoptry/libvcfc.so build_ab/hoptry5/libvcfc.so || exit 1

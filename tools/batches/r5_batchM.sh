#!/bin/bash
# Round-5: predicted deferred records (product build = cur9): every -m gpu
# test; the law-2 device file against cur8; law-2 kernel trace; encoder PMC
# (laws 1/0/2) installed, then the law-2 and law-2 device-file lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/gpu_check.sh r5M tests || exit 1
AB_ARGS="--mode devfile --law 2" bash tools/ab.sh ab_r5m_devfile_law2 build_ab/cur8/libvcfc.so build/libvcfc.so || exit 1
bash tools/gpu_check.sh r5M prof2 pmcenc pmcinstall bench2 benchdev2 || exit 1
echo done

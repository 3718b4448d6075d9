#!/bin/bash
# Round-5: every -m gpu test on the current tree (incl. the per-row deferral
# choice); decoder item words by SWAR (build_ab/cur4) against cur3 on decode
# and the range query; the query bench line and kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r5F tests || exit 1
P=build_ab/cur3/libvcfc.so; C=build_ab/cur4/libvcfc.so
AB_ARGS="--mode decode" bash tools/ab.sh ab_r5f_decode $P $C || exit 1
AB_ARGS="--mode query" bash tools/ab.sh ab_r5f_query $P $C || exit 1
bash tools/gpu_check.sh r5F benchq profq || exit 1
echo done

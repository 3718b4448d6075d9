#!/bin/bash
# Round-4 final measurements of the default tree: smoke, benches (laws 1/0/2,
# decode, device file laws 1/2 and law 2 with deferred records), kernel
# stats, encoder PMC (laws 1/0/2) and device-file PMC (laws 1/2, law 2
# deferred).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4P smoke bench bench0 bench2 benchdec benchdev benchdev2 prof prof2 profdev profdev2 profdec pmcenc || exit 1
LAW=2 bash tools/gpu_check.sh r4P pmcdev || exit 1
LAW=1 bash tools/gpu_check.sh r4P pmcdev || exit 1
LAW=2 DEV_ARGS="--deferred-records" DEV_TAG="_deferred" DEV_KEY="/deferred" bash tools/gpu_check.sh r4P pmcdev || exit 1
timeout -k 10 300 python bench.py --mode devfile --law 2 --deferred-records > gpurun_out/r4P/bench_devfile_law2_deferred.json 2> gpurun_out/r4P/bench_devfile_law2_deferred.err || exit 1

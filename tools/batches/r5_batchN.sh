#!/bin/bash
# Round-5: law-2 device-file PMC on predicted deferred records, installed with
# the corrected encoder summaries; the law-2 and law-2 device-file lines;
# the 2-rank rehearsals (bench.py --gpus 2 and --mode distfile on one GPU)
# with the bounded collectives.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
LAW=2 bash tools/gpu_check.sh r5N pmcdev || exit 1
cp gpurun_out/r5N/pmc_devfile_l2.json profiles/pmc_devfile_law2.json || exit 1
bash tools/gpu_check.sh r5N bench2 benchdev2 rehearse2 distfile2 || exit 1
echo done

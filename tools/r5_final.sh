#!/bin/bash
# Round-5 final tree on one box: smoke, every -m gpu test, the encoder PMC
# (laws 1/0/2) and the law-2 device-file PMC installed as the summaries
# bench.py reads, then the headline line, the same command under rocprofv3
# (kernel stats and trace of that process), and the other lines: law 0,
# law 2, decode, range query, the device-resident file (laws 1 and 2), the
# 2-rank rehearsals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=${FINAL_TAG:-r5final5}
bash tools/gpu_check.sh $T smoke tests pmcenc || exit 1
LAW=2 bash tools/gpu_check.sh $T pmcdev || exit 1
bash tools/gpu_check.sh $T pmcinstall bench profbench || exit 1
bash tools/gpu_check.sh $T bench0 bench2 benchdec benchq benchdev benchdev2 rehearse2 distfile2 || exit 1
echo done

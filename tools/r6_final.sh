#!/bin/bash
# Round-6 final tree, two gpurun calls (each well inside the 1 200 s limit):
#   A: smoke, every -m gpu test, the encoder PMC (laws 1/0/2/3), the device
#      file and query PMC, installed as the summaries bench.py reads, then the
#      headline line and the same command under rocprofv3;
#   B: the other lines (laws 0/2/3, decode, query, device file laws 1/2,
#      configs[3] batch, ingest, 2- and 8-rank rehearsals, sharded file).
#   FINAL_TAG=r6final bash tools/r6_final.sh A|B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=${FINAL_TAG:-r6final}
case "$1" in
  A) bash tools/gpu_check.sh $T smoke tests pmcenc pmcenc3 || exit 1
     LAW=1 bash tools/gpu_check.sh $T pmcdev || exit 1
     LAW=2 bash tools/gpu_check.sh $T pmcdev || exit 1
     bash tools/gpu_check.sh $T pmcq pmcinstall bench profbench || exit 1 ;;
  B) bash tools/gpu_check.sh $T bench0 bench2 bench3 benchdec benchq benchdev benchdev2 biobank benching rehearse2 rehearse8 distfile2 || exit 1 ;;
  *) echo "usage: $0 A|B"; exit 2 ;;
esac
echo done

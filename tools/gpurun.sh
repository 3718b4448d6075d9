#!/bin/bash
# Local wrapper: rebuild the in-tree libraries (they travel to the box with
# the snapshot; nothing is built there), then run one gpurun call.
#   tools/gpurun.sh <timeout-s> '<command>'
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
make -s -j8 -C "$R/vcf-compression_amd"
make -s -C "$R/oracle"
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"

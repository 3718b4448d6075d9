#!/bin/bash
# PMC of the devfile step's kernels for A/B libraries (tools/pmc_hop_ab.sh
# <tag> <lib dir name>...): two counter passes per library, each its own run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); TAG=$1; shift
for n in "$@"; do
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    k=$(echo $P | cut -d' ' -f1)
    O="$R/gpurun_out/$TAG/$n/$k"; mkdir -p "$O"
    (cd /tmp && export TMPDIR=/tmp && VCFC_LIB="$R/build/ab/$n/libvcfc.so" timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O" -o run -- python3 "$R/bench.py" --mode devfile --steps 2 --warmup 1 > "$O/log" 2>&1) || { echo "pmc $n $k failed"; tail -20 "$O/log"; exit 1; }
  done
done
echo ok

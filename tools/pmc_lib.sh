#!/bin/bash
# Instruction / wait / LDS counters of one library build on one bench
# configuration: tools/pmc_lib.sh <tag> <lib> [bench args...]; one rocprofv3
# pass per counter group, summaries by tools/pmc_summary.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; LIB="$2"; shift 2
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && VCFC_LIB="$R/$LIB" timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmc$i" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$O/pmc$i.log" 2>&1) || { echo "pmc pass $i failed rc=$?"; tail -30 "$O/pmc$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$O" > "$O/summary.json" && cat "$O/summary.json"

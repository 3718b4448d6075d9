#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT}"; O="$R/gpurun_out/r6pmchop"; mkdir -p "$O"; cd "$R" || exit 1
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  n=$(echo $P | cut -d' ' -f1)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmc_$n" -o run -- python3 "$R/bench.py" --mode devfile --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc_$n.log" 2>&1) || { echo "pmc $n failed rc=$?"; tail -30 "$O/pmc_$n.log"; exit 1; }
done
echo pmc done

#!/bin/bash
# Round-4 closing: the N=2 launcher rehearsal on one GPU (bench.py --gpus 2
# spawns torch.distributed.run as a child) and the configs[3] shard with
# 1100 oracle-checked rows per batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4AB
VCFC_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r4AB/bench_n2_rehearsal.json 2> gpurun_out/r4AB/bench_n2_rehearsal.err || { echo rehearsal failed; tail -30 gpurun_out/r4AB/bench_n2_rehearsal.err; exit 1; }
cat gpurun_out/r4AB/bench_n2_rehearsal.json
bash tools/gpu_check.sh r4AB shard || exit 1

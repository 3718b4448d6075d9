#!/bin/bash
# k_encode_fast on the headline batch and inside the device-file step, one box:
# two rocprofv3 kernel traces (tools/prof_enc_vs_dev.sh <tag>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); O="$R/gpurun_out/$1"; mkdir -p "$O"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/enc" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/enc.log" 2>&1) || { echo "enc failed"; tail -20 "$O/enc.log"; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/dev" -o run -- python3 "$R/bench.py" --mode devfile --steps 10 --warmup 2 > "$O/dev.log" 2>&1) || { echo "dev failed"; tail -20 "$O/dev.log"; exit 1; }
echo ok

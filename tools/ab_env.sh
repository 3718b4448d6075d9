#!/bin/bash
# A/B timing on one GPU box over environment settings of the same build:
# tools/ab_env.sh <tag> "VAR=a" "VAR=b" ...  (k_encode ms, k_compact ms, step ms)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
for round in 1 2 3; do
  for kv in "$@"; do
    n=$(echo "$kv" | tr '=' '_')
    env "$kv" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 ${AB_ARGS} > "$O/$n.$round.json" 2> "$O/$n.$round.err" || { echo "bench $kv failed"; tail -20 "$O/$n.$round.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], r['avg_launch_ms'], r['stages_ms'], d['ms_per_step'], d['value'])" "$O/$n.$round.json" "$kv" "$round" | tee -a "$O/ab.txt"
  done
done

#!/bin/bash
# A/B timing on one GPU box: alternate bench.py runs over several libvcfc.so
# builds (tools/ab.sh <tag> lib1 lib2 ...), k_encode ms from each JSON line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
for round in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $(dirname "$lib"))
    VCFC_LIB="$R/$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 ${AB_ARGS} > "$O/$n.$round.json" 2> "$O/$n.$round.err" || { echo "bench $lib failed"; tail -20 "$O/$n.$round.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], sys.argv[3], r.get('avg_launch_ms', -1), (r.get('stages_ms') or {}).get('k_compact', -1), d['ms_per_step'])" "$O/$n.$round.json" "$n" "$round" | tee -a "$O/ab.txt"
  done
done

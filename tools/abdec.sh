#!/bin/bash
# A/B of the decoder (bench.py --mode decode) over library builds, alternating on one box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
for round in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $(dirname "$lib"))
    VCFC_LIB="$R/$lib" timeout -k 10 300 python bench.py --mode decode --steps 30 --no-cpu-baseline ${AB_ARGS} > "$O/$n.$round.json" 2> "$O/$n.$round.err" || { echo "bench $lib failed"; tail -20 "$O/$n.$round.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['roofline']['avg_launch_ms'], d['output_identical_to_input_rows'])" "$O/$n.$round.json" "$n" "$round" | tee -a "$O/ab.txt"
  done
done

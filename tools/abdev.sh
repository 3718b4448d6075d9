#!/bin/bash
# A/B of the device-resident file compress (bench.py --mode devfile) over
# library builds, alternating on one box: tools/abdev.sh <tag> lib1 lib2 ...
# (AB_ARGS: extra bench.py arguments, e.g. "--law 2").
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
for round in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $(dirname "$lib"))
    VCFC_LIB="$R/$lib" timeout -k 10 300 python bench.py --mode devfile --steps 10 --warmup 2 ${AB_ARGS} > "$O/$n.$round.json" 2> "$O/$n.$round.err" || { echo "bench $lib failed"; tail -20 "$O/$n.$round.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['output_identical_to_header_plus_records'])" "$O/$n.$round.json" "$n" "$round" | tee -a "$O/ab.txt"
  done
done

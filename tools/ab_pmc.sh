#!/bin/bash
# HBM counters per library build (tools/ab_pmc.sh <tag> lib1 lib2 ...):
# one rocprofv3 pass each for FETCH_SIZE and WRITE_SIZE over a short bench
# run; summaries via tools/pmc_summary.py into gpurun_out/<tag>/<name>.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R" || exit 1
for lib in "$@"; do
  n=$(basename $(dirname "$lib"))
  for P in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && VCFC_LIB="$R/$lib" timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/$n/pmc_$P" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${AB_ARGS} > "$O/$n.pmc_$P.log" 2>&1) || { echo "pmc $n $P failed rc=$?"; tail -30 "$O/$n.pmc_$P.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$O/$n" > "$O/$n.json" && python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k,v in sorted(d.items()):
    if 'FETCH_SIZE' in v or 'WRITE_SIZE' in v:
        print(sys.argv[2], k, 'fetch_GB %.3f write_GB %.3f ms %.3f' % (v.get('FETCH_SIZE',0)*1024/1e9, v.get('WRITE_SIZE',0)*1024/1e9, v['dispatch_ms']))
" "$O/$n.json" "$n" | tee -a "$O/pmc.txt"
done

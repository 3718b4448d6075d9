#!/bin/bash
# rocprofv3 kernel stats of the law-2 encode, whole and by row kind (0..4),
# one process each: gpurun_out/<tag>/kind<K>/, gpurun_out/<tag>/law2/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r6kinds}"; mkdir -p "$O"
for K in law2 0 1 2 3 4; do
  n=$([ "$K" = law2 ] && echo law2 || echo kind$K)
  (cd /tmp && export TMPDIR=/tmp && if [ "$K" != law2 ]; then export VCFC_LAW2_KIND=$K; fi &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n" -o run -- python3 "$R/bench.py" --law 2 --steps 10 --warmup 2 --no-cpu-baseline > "$O/$n.log" 2>&1) || { echo "prof $n failed rc=$?"; tail -30 "$O/$n.log"; exit 1; }
done
echo prof done

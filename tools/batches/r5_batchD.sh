#!/bin/bash
# Round-5: deferred records on (build_ab/cur2) against off (cur2_nodefer) on
# law 2, GT:DP:GQ rows alone (kind 1), laws 0 and 1; kernel stats of both on
# law 2; PMC (instructions, LDS conflicts) of the variable-token kernel on
# kinds 0 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=build_ab/cur2/libvcfc.so; O=build_ab/cur2_nodefer/libvcfc.so
AB_ARGS="--law 2" bash tools/ab.sh ab_r5d_law2 $O $D || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_r5d_kind1 $O $D || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_r5d_law0 $O $D || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5d_law1 $O $D || exit 1
R="$(pwd)"; OUT="$R/gpurun_out/r5D"; mkdir -p "$OUT"
for n in cur2 cur2_nodefer; do
  (cd /tmp && export TMPDIR=/tmp && VCFC_LIB="$R/build_ab/$n/libvcfc.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof2_$n" -o run -- python3 "$R/bench.py" --law 2 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof2_$n.log" 2>&1) || { echo "prof2 $n failed"; tail -20 "$OUT/prof2_$n.log"; exit 1; }
done
VCFC_LAW2_KIND=0 bash tools/pmc_lib.sh r5D_pmc_kind0 build_ab/cur2/libvcfc.so --law 2 > /dev/null || exit 1
VCFC_LAW2_KIND=4 bash tools/pmc_lib.sh r5D_pmc_kind4 build_ab/cur2/libvcfc.so --law 2 > /dev/null || exit 1
echo done

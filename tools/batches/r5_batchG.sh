#!/bin/bash
# Round-5: law-2 device file with deferred records on (default) / off, three
# alternating rounds; esc8's stores by hand-written v_mad_i32_i24 (cur5)
# against cur4 on laws 0 and 1; step HBM traffic of the device file
# (deferred, the default) and of the encode step for laws 1, 0, 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O="gpurun_out/ab_r5g_devfile_law2"; mkdir -p "$O"
for round in 1 2 3; do
  for m in off on; do
    timeout -k 10 300 python bench.py --mode devfile --law 2 --steps 10 --warmup 2 --deferred-records $m > "$O/$m.$round.json" 2> "$O/$m.$round.err" || { echo "devfile $m failed"; tail -20 "$O/$m.$round.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['output_identical_to_header_plus_records'])" "$O/$m.$round.json" "$m" "$round" | tee -a "$O/ab.txt"
  done
done
P=build_ab/cur4/libvcfc.so; C=build_ab/cur5/libvcfc.so
AB_ARGS="--law 0" bash tools/ab.sh ab_r5g_law0 $P $C || exit 1
AB_ARGS="--law 1" bash tools/ab.sh ab_r5g_law1 $P $C || exit 1
LAW=2 bash tools/gpu_check.sh r5G pmcdev pmcenc || exit 1
echo done

#!/bin/bash
# Round-4 check of the opt-in deferral: the default tree (cur4) against HEAD
# before deferral (headline, law 2, kind 0), the device-file law 2 with and
# without --deferred-records, then every -m gpu test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/head/libvcfc.so build_ab/cur4/libvcfc.so"
bash tools/ab.sh ab_optin_law1 $L || exit 1
AB_ARGS="--law 2" bash tools/ab.sh ab_optin_law2 $L || exit 1
VCFC_LAW2_KIND=0 AB_ARGS="--law 2" bash tools/ab.sh ab_optin_kind0 $L || exit 1
O=gpurun_out/ab_optin_dev2; mkdir -p $O
for r in 1 2 3; do
  for d in "" "--deferred-records"; do
    timeout -k 10 300 python bench.py --mode devfile --law 2 --steps 10 --warmup 2 $d > $O/dev.$r.json 2> $O/dev.$r.err || { echo devfile failed; tail -20 $O/dev.$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('deferred' if d['config']['deferred_records'] else 'staged', sys.argv[2], d['ms_per_step'], d['output_identical_to_header_plus_records'])" $O/dev.$r.json $r | tee -a $O/ab.txt
  done
done
bash tools/gpu_check.sh r4O tests || exit 1

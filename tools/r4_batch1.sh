#!/bin/bash
# Round-4 measurement batch (one gpurun call): law-0 bisect, the var
# kernel's interior escape path (law 2, kind 1), decode, device-file lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4d
AB_ARGS="--law 2" bash tools/ab.sh ab_escfast_law2 build_ab/base/libvcfc.so build_ab/escfast/libvcfc.so || exit 1
VCFC_LAW2_KIND=1 AB_ARGS="--law 2" bash tools/ab.sh ab_escfast_kind1 build_ab/base/libvcfc.so build_ab/escfast/libvcfc.so || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_law0_bisect build_ab/base/libvcfc.so build_ab/nostep/libvcfc.so build_ab/nostore/libvcfc.so || exit 1
bash tools/abdec.sh ab_dec_noscan build_ab/base/libvcfc.so build_ab/decnoscan/libvcfc.so || exit 1
for li in scan; do
  timeout -k 10 200 python bench.py --mode devfile --law 2 --line-index $li --steps 10 --warmup 2 > gpurun_out/r4d/devfile_law2_$li.json 2> gpurun_out/r4d/devfile_law2_$li.err || exit 1
done
timeout -k 10 200 python bench.py --mode devfile --law 1 --steps 10 --warmup 2 > gpurun_out/r4d/devfile_law1_hop.json 2> gpurun_out/r4d/devfile_law1_hop.err
bash tools/abdev.sh ab_hoptry_law1 build_ab/base/libvcfc.so build_ab/hoptry/libvcfc.so || exit 1
AB_ARGS="--law 2" bash tools/abdev.sh ab_hoptry_law2 build_ab/base/libvcfc.so build_ab/hoptry/libvcfc.so || exit 1

#!/bin/bash
# Round-4 bisects (one gpurun call): law 0 (genotype step removed / no
# staging stores), the decoder's tile stores without the item scan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
AB_ARGS="--law 0" bash tools/ab.sh ab_law0_bisect build_ab/base/libvcfc.so build_ab/nostep/libvcfc.so build_ab/nostore/libvcfc.so || exit 1
bash tools/abdec.sh ab_dec_noscan build_ab/base/libvcfc.so build_ab/decnoscan/libvcfc.so || exit 1
mkdir -p gpurun_out/r4B
timeout -k 10 200 python bench.py --mode devfile --law 2 --line-index scan --steps 10 --warmup 2 > gpurun_out/r4B/devfile_law2_scan.json 2> gpurun_out/r4B/devfile_law2_scan.err || exit 1
cd /tmp && export TMPDIR=/tmp && VCFC_LIB=$GRAFT_REPO_ROOT/build_ab/hoptry5/libvcfc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4B/prof_devfile_law2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode devfile --law 2 --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r4B/prof_devfile_law2.log 2>&1 || exit 1
VCFC_LIB=$GRAFT_REPO_ROOT/build_ab/hoptry5/libvcfc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4B/prof_devfile_law1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode devfile --law 1 --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r4B/prof_devfile_law1.log 2>&1

#!/bin/bash
# GPU-box driver for one round trip: smoke -> GPU parity tests -> bench ->
# rocprofv3 kernel trace.  Every GPU step has its own time limit; the chain
# stops at the first failure.  Usage: tools/gpu_check.sh <tag> [steps...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r}"; shift
STEPS="${*:-smoke tests bench prof}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R" || exit 1
echo "box: $(hostname) $(date)" > "$O/info.txt"
rocm-smi --showproductname >> "$O/info.txt" 2>&1 || true
for s in $STEPS; do
  echo "== $s $(date +%T)" | tee -a "$O/progress.txt"
  case $s in
    smoke) timeout -k 10 420 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed rc=$?"; tail -30 "$O/smoke.log"; exit 1; } ;;
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations 15 > "$O/pytest_gpu.log" 2>&1 || { echo "tests failed rc=$?"; tail -40 "$O/pytest_gpu.log"; exit 1; } ;;
    bench) timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed rc=$?"; tail -30 "$O/bench.err"; exit 1; } ; cat "$O/bench.json" ;;
    bench0) timeout -k 10 600 python bench.py --law 0 --no-cpu-baseline > "$O/bench_law0.json" 2> "$O/bench_law0.err" || { echo "bench0 failed"; tail -30 "$O/bench_law0.err"; exit 1; } ; cat "$O/bench_law0.json" ;;
    biobank) timeout -k 10 900 python bench.py --mode biobank --steps 5 --warmup 1 > "$O/bench_biobank.json" 2> "$O/bench_biobank.err" || { echo "biobank failed"; tail -30 "$O/bench_biobank.err"; exit 1; } ; cat "$O/bench_biobank.json" ;;
    profbio) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profbio" -o run -- python3 "$R/bench.py" --mode biobank --steps 3 --warmup 1 --no-cpu-baseline > "$O/profbio.log" 2>&1) || { echo "profbio failed rc=$?"; tail -30 "$O/profbio.log"; exit 1; } ;;
    dtests) timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_sparsify.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_d.log" 2>&1 || { echo "dtests failed rc=$?"; tail -40 "$O/pytest_d.log"; exit 1; } ;;
    wtests) timeout -k 10 900 python -u -m pytest tests/test_gpu_encode.py -x -v -k synthetic -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_w.log" 2>&1 || { echo "wtests failed rc=$?"; tail -40 "$O/pytest_w.log"; exit 1; } ;;
    benchdec) timeout -k 10 600 python bench.py --mode decode > "$O/bench_decode.json" 2> "$O/bench_decode.err" || { echo "benchdec failed"; tail -30 "$O/bench_decode.err"; exit 1; } ; cat "$O/bench_decode.json" ;;
    benchsp) timeout -k 10 900 python bench.py --mode sparse --steps 5 --warmup 1 > "$O/bench_sparse.json" 2> "$O/bench_sparse.err" || { echo "benchsp failed"; tail -30 "$O/bench_sparse.err"; exit 1; } ; cat "$O/bench_sparse.json" ;;
    benchq) timeout -k 10 600 python bench.py --mode query > "$O/bench_query.json" 2> "$O/bench_query.err" || { echo "benchq failed"; tail -30 "$O/bench_query.err"; exit 1; } ; cat "$O/bench_query.json" ;;
    profq) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profq" -o run -- python3 "$R/bench.py" --mode query --steps 10 --warmup 2 --no-cpu-baseline > "$O/profq.log" 2>&1) || { echo "profq failed rc=$?"; tail -30 "$O/profq.log"; exit 1; } ;;
    pmcq) # HBM bytes per query step (k_query_match + selected decode) -> pmc_k_query.json
         for P in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcq_$P" -o run -- python3 "$R/bench.py" --mode query --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmcq_$P.log" 2>&1) || { echo "pmcq $P failed rc=$?"; tail -30 "$O/pmcq_$P.log"; exit 1; }
         done
         python3 tools/pmc_step_json.py "$O/pmcq_FETCH_SIZE" "$O/pmcq_WRITE_SIZE" 4 "chr22-shaped/2504x1000000/0.125" "$O/pmc_k_query.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --mode query --steps 3 --warmup 1 (tools/gpu_check.sh pmcq, run $TAG)" k_query_match "range query step (k_query_match + selected k_dec_plan / scan / k_dec_write)" > /dev/null || { echo "pmcq json failed"; exit 1; } ;;
    qtests) timeout -k 10 900 python -m pytest tests/test_gpu_query.py tests/test_gpu_decode.py -x -q -p no:cacheprovider > "$O/pytest_q.log" 2>&1 || { echo "qtests failed rc=$?"; tail -40 "$O/pytest_q.log"; exit 1; } ;;
    benching) timeout -k 10 900 python bench.py --mode ingest --steps 3 --warmup 1 > "$O/bench_ingest.json" 2> "$O/bench_ingest.err" || { echo "benching failed"; tail -30 "$O/bench_ingest.err"; exit 1; } ; cat "$O/bench_ingest.json" ;;
    itests) timeout -k 10 900 python -m pytest tests/test_gpu_encode.py -x -q -p no:cacheprovider > "$O/pytest_i.log" 2>&1 || { echo "itests failed rc=$?"; tail -40 "$O/pytest_i.log"; exit 1; } ;;
    profdec) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profdec" -o run -- python3 "$R/bench.py" --mode decode --steps 10 --warmup 2 --no-cpu-baseline > "$O/profdec.log" 2>&1) || { echo "profdec failed rc=$?"; tail -30 "$O/profdec.log"; exit 1; } ;;
    pmcdec) for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
           n=$(echo $P | cut -d' ' -f1)
           (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcdec_$n" -o run -- python3 "$R/bench.py" --mode decode --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmcdec_$n.log" 2>&1) || { echo "pmcdec $n failed rc=$?"; tail -30 "$O/pmcdec_$n.log"; exit 1; }
         done ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > "$O/prof.log" 2>&1) || { echo "prof failed rc=$?"; tail -30 "$O/prof.log"; exit 1; } ;;
    pmc) for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
           n=$(echo $P | cut -d' ' -f1)
           (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmc_$n" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$O/pmc_$n.log" 2>&1) || { echo "pmc $n failed rc=$?"; tail -30 "$O/pmc_$n.log"; exit 1; }
         done ;;
    pmcx) for P in "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU"; do
           n=$(echo $P | cut -d' ' -f1)
           (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcx_$n" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$O/pmcx_$n.log" 2>&1) || { echo "pmcx $n failed rc=$?"; tail -30 "$O/pmcx_$n.log"; exit 1; }
         done ;;
    distfile) timeout -k 10 600 python bench.py --mode distfile --steps 3 --warmup 1 > "$O/bench_distfile.json" 2> "$O/bench_distfile.err" || { echo "distfile failed"; tail -30 "$O/bench_distfile.err"; exit 1; } ; cat "$O/bench_distfile.json" ;;
    distfile2) VCFC_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --mode distfile --steps 3 --warmup 1 --dist-dir /tmp/vcfc_distfile2 > "$O/bench_distfile2.json" 2> "$O/bench_distfile2.err" || { echo "distfile2 failed"; tail -30 "$O/bench_distfile2.err"; exit 1; } ; cat "$O/bench_distfile2.json" ;;
    bench3) timeout -k 10 600 python bench.py --law 3 > "$O/bench_law3.json" 2> "$O/bench_law3.err" || { echo "bench3 failed"; tail -30 "$O/bench_law3.err"; exit 1; } ; cat "$O/bench_law3.json" ;;
    pmcenc3) # encoder HBM bytes per launch for law 3 -> pmc_k_encode_law3.json
         for P in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcenc_l3_$P" -o run -- python3 "$R/bench.py" --law 3 --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmcenc_l3_$P.log" 2>&1) || { echo "pmcenc3 $P failed rc=$?"; tail -30 "$O/pmcenc_l3_$P.log"; exit 1; }
         done
         python3 tools/pmc_encode_json.py "$O/pmcenc_l3_FETCH_SIZE" "$O/pmcenc_l3_WRITE_SIZE" "alternating-classes (every token a run / het 1/2)/2504x1000000" "$O/pmc_k_encode_law3.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/gpu_check.sh pmcenc3, run $TAG)" > /dev/null || { echo "pmc3 json failed"; exit 1; } ;;
    prof3) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof3" -o run -- python3 "$R/bench.py" --law 3 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof3.log" 2>&1) || { echo "prof3 failed rc=$?"; tail -30 "$O/prof3.log"; exit 1; } ;;
    rehearse8) # exactly the driver's `python bench.py --gpus 8` path, 8 gloo ranks on the one GPU
         VCFC_BENCH_REHEARSAL=1 timeout -k 10 900 python bench.py --gpus 8 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_n8_rehearsal.json" 2> "$O/bench_n8_rehearsal.err" || { echo "rehearse8 failed"; tail -30 "$O/bench_n8_rehearsal.err"; exit 1; } ; cat "$O/bench_n8_rehearsal.json" ;;
    bench2) timeout -k 10 600 python bench.py --law 2 --no-cpu-baseline > "$O/bench_law2.json" 2> "$O/bench_law2.err" || { echo "bench2 failed"; tail -30 "$O/bench_law2.err"; exit 1; } ; cat "$O/bench_law2.json" ;;
    prof2) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof2" -o run -- python3 "$R/bench.py" --law 2 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof2.log" 2>&1) || { echo "prof2 failed rc=$?"; tail -30 "$O/prof2.log"; exit 1; } ;;
    pmc2) for P in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmc2_$P" -o run -- python3 "$R/bench.py" --law 2 --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc2_$P.log" 2>&1) || { echo "pmc2 $P failed rc=$?"; tail -30 "$O/pmc2_$P.log"; exit 1; }
         done ;;
    shard) timeout -k 10 900 python bench.py --mode biobank --rows-total 5000000 --steps 1 --warmup 1 > "$O/bench_biobank_shard.json" 2> "$O/bench_biobank_shard.err" || { echo "shard failed"; tail -30 "$O/bench_biobank_shard.err"; exit 1; } ; cat "$O/bench_biobank_shard.json" ;;
    ptest) timeout -k 10 1000 python -u -m pytest ${PT_ARGS} -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$O/pytest_sel.log" 2>&1 || { echo "ptest failed rc=$?"; tail -60 "$O/pytest_sel.log"; exit 1; } ; tail -5 "$O/pytest_sel.log" ;;
    pmcenc) # encoder HBM bytes per launch for laws 1, 0, 2 (two passes each) -> pmc_k_encode*.json
         for L in 1 0 2; do
           for P in FETCH_SIZE WRITE_SIZE; do
             (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcenc_l${L}_$P" -o run -- python3 "$R/bench.py" --law $L --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmcenc_l${L}_$P.log" 2>&1) || { echo "pmcenc $L $P failed rc=$?"; tail -30 "$O/pmcenc_l${L}_$P.log"; exit 1; }
           done
         done
         python3 tools/pmc_encode_json.py "$O/pmcenc_l1_FETCH_SIZE" "$O/pmcenc_l1_WRITE_SIZE" "chr22-shaped/2504x1000000" "$O/pmc_k_encode.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/gpu_check.sh pmcenc, run $TAG)" > /dev/null &&
         python3 tools/pmc_encode_json.py "$O/pmcenc_l0_FETCH_SIZE" "$O/pmcenc_l0_WRITE_SIZE" "random_vcf-law/2504x1000000" "$O/pmc_k_encode_law0.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/gpu_check.sh pmcenc, run $TAG)" > /dev/null &&
         python3 tools/pmc_encode_json.py "$O/pmcenc_l2_FETCH_SIZE" "$O/pmcenc_l2_WRITE_SIZE" "general-shapes (chrX haploid/GT:DP:GQ/missing)/2504x1000000" "$O/pmc_k_encode_law2.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/gpu_check.sh pmcenc, run $TAG)" > /dev/null || { echo "pmc json failed"; exit 1; } ;;
    pmcinstall) # the PMC summaries this run just made become the ones bench.py reads (same-box lines)
         for f in "$O"/pmc_k_encode*.json "$O"/pmc_k_query.json "$O"/pmc_devfile_l*.json; do [ -f "$f" ] && cp "$f" profiles/; done; ls -l profiles/pmc_*.json ;;
    profbench) # the default bench command itself under rocprofv3: the JSON line and the kernel stats of one process
         (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profbench" -o run -- python3 "$R/bench.py" > "$O/bench_under_prof.json" 2> "$O/profbench.log") || { echo "profbench failed rc=$?"; tail -30 "$O/profbench.log"; exit 1; } ; cat "$O/bench_under_prof.json" ;;
    benchdev) timeout -k 10 300 python bench.py --mode devfile > "$O/bench_devfile.json" 2> "$O/bench_devfile.err" || { echo "benchdev failed"; tail -30 "$O/bench_devfile.err"; exit 1; } ; cat "$O/bench_devfile.json" ;;
    pmcdev) # HBM bytes per devfile step (every kernel of one call), law ${LAW:-1} -> pmc_devfile_l<law>.json
         for P in FETCH_SIZE WRITE_SIZE; do
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/pmcdev_l${LAW:-1}${DEV_TAG}_$P" -o run -- python3 "$R/bench.py" --mode devfile --law ${LAW:-1} --steps 3 --warmup 1 ${DEV_ARGS} > "$O/pmcdev_l${LAW:-1}${DEV_TAG}_$P.log" 2>&1) || { echo "pmcdev $P failed rc=$?"; tail -30 "$O/pmcdev_l${LAW:-1}${DEV_TAG}_$P.log"; exit 1; }
         done
         python3 tools/pmc_step_json.py "$O/pmcdev_l${LAW:-1}${DEV_TAG}_FETCH_SIZE" "$O/pmcdev_l${LAW:-1}${DEV_TAG}_WRITE_SIZE" 4 "$(python3 -c "import bench,sys; print(bench.law_name(int(sys.argv[1])))" ${LAW:-1})/2504x1000000/hop${DEV_KEY}" "$O/pmc_devfile_l${LAW:-1}${DEV_TAG}.json" "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --mode devfile --law ${LAW:-1} --steps 3 --warmup 1 ${DEV_ARGS} (tools/gpu_check.sh pmcdev, run $TAG)" > /dev/null || { echo "pmcdev json failed"; exit 1; } ;;
    benchdev2) timeout -k 10 300 python bench.py --mode devfile --law 2 > "$O/bench_devfile_law2.json" 2> "$O/bench_devfile_law2.err" || { echo "benchdev2 failed"; tail -30 "$O/bench_devfile_law2.err"; exit 1; } ; cat "$O/bench_devfile_law2.json" ;;
    profdev2) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profdev2" -o run -- python3 "$R/bench.py" --mode devfile --law 2 --steps 5 --warmup 1 > "$O/profdev2.log" 2>&1) || { echo "profdev2 failed rc=$?"; tail -30 "$O/profdev2.log"; exit 1; } ;;
    profdev) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profdev" -o run -- python3 "$R/bench.py" --mode devfile --steps 5 --warmup 1 > "$O/profdev.log" 2>&1) || { echo "profdev failed rc=$?"; tail -30 "$O/profdev.log"; exit 1; } ;;
    rehearse2) VCFC_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_n2_rehearsal.json" 2> "$O/bench_n2_rehearsal.err" || { echo "rehearse2 failed"; tail -30 "$O/bench_n2_rehearsal.err"; exit 1; } ; cat "$O/bench_n2_rehearsal.json" ;;
    rehearse4) VCFC_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29625 bench.py --gpus 4 --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_n4_rehearsal.json" 2> "$O/bench_n4_rehearsal.err" || { echo "rehearse4 failed"; tail -30 "$O/bench_n4_rehearsal.err"; exit 1; } ; cat "$O/bench_n4_rehearsal.json" ;;
    rehearse4s) VCFC_BENCH_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29627 bench.py --gpus 4 --scaling strong --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_n4s_rehearsal.json" 2> "$O/bench_n4s_rehearsal.err" || { echo "rehearse4s failed"; tail -30 "$O/bench_n4s_rehearsal.err"; exit 1; } ; cat "$O/bench_n4s_rehearsal.json" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all ok $(date +%T)"

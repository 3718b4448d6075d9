set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd)
for n in ${@:-base guess}; do
  O="$R/gpurun_out/r6gprof/$n"; mkdir -p "$O"
  (cd /tmp && export TMPDIR=/tmp && VCFC_LIB="$R/build/ab/$n/libvcfc.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- python3 "$R/bench.py" --mode devfile --steps 5 --warmup 1 > "$O/log" 2>&1) || { echo "prof $n failed"; tail -20 "$O/log"; exit 1; }
done
echo ok

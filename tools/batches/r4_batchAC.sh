#!/bin/bash
# Round-4 final tree: smoke(), the default bench line, and the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4AC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4AC/smoke.log 2>&1 || { tail -20 gpurun_out/r4AC/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r4AC/bench.json 2> gpurun_out/r4AC/bench.err || { tail -20 gpurun_out/r4AC/bench.err; exit 1; }
cat gpurun_out/r4AC/bench.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4AC/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r4AC/pytest_gpu.log; exit $rc

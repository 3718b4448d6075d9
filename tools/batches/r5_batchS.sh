#!/bin/bash
# Round-5: HIP-graph replay of law-2 batches (predicted deferred records) and
# of a mispredicting batch (the gated relayout inside the graph).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=tests/test_gpu_encode.py
PT_ARGS="$T::test_encode_captured_in_hip_graph $T::test_mispredicted_batch_replayed_in_hip_graph $T::test_predicted_deferred_records" bash tools/gpu_check.sh r5S ptest || exit 1
echo done

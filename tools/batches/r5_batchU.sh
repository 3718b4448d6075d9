#!/bin/bash
# Round-5: configs[3] lines on the final tree (100k samples: one batch, and
# the 5M-row shard as 50 batches, every record / sampled records digested),
# the sparse layout and ingest lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/gpu_check.sh r5U biobank shard benchsp benching || exit 1
echo done

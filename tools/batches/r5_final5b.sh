#!/bin/bash
# Round-5 final tree (final5): the lines final2 measured on an earlier tree,
# again: configs[3] batch and 5M-row shard, file -> file ingest, sparse
# query, 4-rank weak / strong rehearsals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash tools/gpu_check.sh r5final5b biobank shard benching benchsp rehearse4 rehearse4s || exit 1
echo done

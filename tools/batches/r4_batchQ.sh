#!/bin/bash
# Round-4: law-2 bench line with the refreshed encoder PMC file, and the
# configs[3] biobank shard on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4Q bench2 shard || exit 1

#!/bin/bash
# Round-4 closing check of the committed tree: smoke, every -m gpu test,
# the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4S smoke tests bench || exit 1

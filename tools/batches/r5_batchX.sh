#!/bin/bash
# Round-5: law-2 device-file PMC and the law-2 kernel trace on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
LAW=2 bash tools/gpu_check.sh r5X pmcdev prof2 || exit 1
echo done

#!/bin/bash
# Round-4 check after the learning hop index: smoke, all -m gpu tests,
# headline / law-0 / law-2 / decode / device-file benches, kernel stats, and
# per-step HBM bytes of the device-file compress at laws 1 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh r4H smoke tests bench bench0 bench2 benchdec benchdev benchdev2 prof profdev profdev2 || exit 1
LAW=2 bash tools/gpu_check.sh r4H pmcdev || exit 1
LAW=1 bash tools/gpu_check.sh r4H pmcdev || exit 1

#!/bin/bash
# Round-4 A/B: block scans by DPP limb scans (scan) against the LDS
# Hillis-Steele scans (cur4): headline (stage times in the JSON) and decode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L="build_ab/cur4/libvcfc.so build_ab/scan/libvcfc.so"
bash tools/ab.sh ab_scan_law1 $L || exit 1
for r in 1 2 3; do for lib in $L; do python -c "import json,sys; d=json.load(open('gpurun_out/ab_scan_law1/%s.%d.json' % (sys.argv[1], int(sys.argv[2])))); print(sys.argv[1], sys.argv[2], d['roofline']['stages_ms'])" $(basename $(dirname $lib)) $r | tee -a gpurun_out/ab_scan_law1/stages.txt; done; done
bash tools/abdec.sh ab_scan_dec $L || exit 1

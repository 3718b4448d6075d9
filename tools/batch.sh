#!/bin/bash
# One gpurun call's worth of GPU work, from the repository root on the box:
#   bash tools/batch.sh '<job>' ['<job>' ...]
# Each job is one quoted string, run in order; the first failure ends the
# call (no retries, no further GPU steps).  Jobs:
#   check <tag> <step>...         tools/gpu_check.sh <tag> <step>... (tests,
#                                 bench lines, rocprofv3 traces and PMC passes)
#   ab <tag> <bench args> <lib>...  tools/ab.sh: alternating bench.py runs over
#                                 several libvcfc.so builds (three rounds);
#                                 <bench args> is one word, commas for spaces
#                                 ("--law,2"; "-" for none)
#   env <NAME=value>...           environment for the jobs after it
# Example (an A/B of two builds on laws 1 and 2, then the headline line):
#   bash tools/batch.sh 'ab ab_x_law1 --law,1 build/ab/a/libvcfc.so build/ab/b/libvcfc.so' \
#                       'ab ab_x_law2 --law,2 build/ab/a/libvcfc.so build/ab/b/libvcfc.so' 'check r6x bench'
# (Rounds 4-5 kept one script per call under tools/batches/; they are in the
# git history, folded into this one in round 6.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for job in "$@"; do
  set -- $job
  kind=$1; shift
  case $kind in
    check) bash tools/gpu_check.sh "$@" || exit 1 ;;
    ab) tag=$1; a=$2; shift 2
        [ "$a" = "-" ] && a=""
        AB_ARGS="${a//,/ }" bash tools/ab.sh "$tag" "$@" || exit 1 ;;
    env) for kv in "$@"; do export "$kv"; done ;;
    *) echo "batch.sh: unknown job '$kind'"; exit 2 ;;
  esac
done
echo "batch done $(date +%T)"

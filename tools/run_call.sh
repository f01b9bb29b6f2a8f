#!/bin/bash
# Run one section of a GPU-call file (tools/calls/r0N.calls): bash tools/run_call.sh <file> <tag>
# A section starts at a line "[tag]" and ends at the next "[...]" line; its body runs under bash
# from the repository root (typically one tools/gpu_steps.sh invocation).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${1:?calls file}; T=${2:?tag}
body=$(awk -v t="[$T]" '$0 == t {on = 1; next} /^\[[A-Za-z0-9_]+\]$/ {on = 0} on' "$F")
[ -n "$body" ] || { echo "no section [$T] in $F"; exit 2; }
bash -c "$body"

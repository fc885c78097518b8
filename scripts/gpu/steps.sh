#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit, stopping at the first
# failure (a fault, abort or timeout ends the call: nothing else touches the GPU after it).
#   scripts/gpu/steps.sh TAG "SECONDS:command" ["SECONDS:command" ...]
# Logs: gpurun_out/TAG/stepN.log (stdout+stderr of step N); a summary line per step on stdout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for spec in "$@"; do
  i=$((i + 1))
  lim=${spec%%:*}; cmd=${spec#*:}
  t0=$(date +%s)
  timeout -k 10 "$lim" bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "step $i rc=$rc $(( $(date +%s) - t0 ))s: $cmd"
  tail -3 "$out/step$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

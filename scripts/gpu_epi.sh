#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/epi
PYTHONPATH=. timeout -k 10 300 python3 scripts/exp/epilogue_probe.py 320 512 > gpurun_out/epi/probe.jsonl 2>&1 || exit $?
grep '^{' gpurun_out/epi/probe.jsonl

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python3 scripts/exp/copy_gap_probe.py

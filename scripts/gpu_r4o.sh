#!/bin/bash
# Winsorize iteration predictor probe (scripts/wins_predict.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4o}
mkdir -p $O
timeout -k 10 400 python scripts/wins_predict.py > $O/wins_predict.log 2>&1 || { echo "probe failed"; tail -20 $O/wins_predict.log; exit 3; }
grep -v "amdgpu.ids" $O/wins_predict.log

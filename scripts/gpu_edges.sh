#!/bin/bash
# edge-case GPU tests of the pair reduce kernel and the half-spectrum registration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/edges
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/edges/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'passed|failed|Error|assert' gpurun_out/edges/pytest.log | tail -15 | cut -c1-400
exit $rc

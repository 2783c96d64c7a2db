#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py 2>&1 | tee gpurun_out/r04l_dist.log | grep -E "PASS|FAIL|Error|passed|failed"

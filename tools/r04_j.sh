#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/overlap_probe.py 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04j_overlap.log && \
./tools/r04_g.sh

#!/bin/bash
# the shipped forward tiles, many launches each: 48-label (two workgroups per
# CU), 96-, 128- and 256-label (one per CU); forward and backward
set -o pipefail
{
for cfg in "512 2048 38 38" "512 2048 81 81" "512 2048 128 128" "64 4096 1024 1024"; do
  PROBE_BWD=1 timeout -k 10 200 python tools/repeat_probe.py $cfg 200 || exit 1
done
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04i_repeat.log

#!/bin/bash
set -o pipefail
R=$PWD
for v in 2049 8193 1; do
  PROBE_T=1 MPVAE_HIP_LIB="$R/abl/race$v/libmpvae_hip.so" timeout -k 10 120 \
    python tools/repeat_probe.py 512 2048 128 128 80 || exit $?
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04f_race.log

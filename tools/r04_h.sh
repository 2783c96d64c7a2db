#!/bin/bash
set -o pipefail
R=$PWD
{
PROBE_NO_T=1 MPVAE_HIP_LIB="$R/abl/race1/libmpvae_hip.so" timeout -k 10 120 \
  python tools/repeat_probe.py 512 2048 128 128 100 &&
MPVAE_HIP_LIB="$R/abl/race18433/libmpvae_hip.so" timeout -k 10 120 \
  python tools/repeat_probe.py 512 2048 128 128 100
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04h_race.log

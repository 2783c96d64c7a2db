#!/bin/bash
set -o pipefail
R=$PWD
PROBE_T=1 PROBE_DETAIL=1 MPVAE_HIP_LIB="$R/abl/race1/libmpvae_hip.so" timeout -k 10 120 \
  python tools/repeat_probe.py 512 2000 100 100 60 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04e_race.log

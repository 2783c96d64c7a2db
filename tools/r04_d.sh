#!/bin/bash
set -o pipefail
R=$PWD
for v in 1 129 257 513 1025; do
  for L in 128 100; do
    MPVAE_HIP_LIB="$R/abl/race$v/libmpvae_hip.so" timeout -k 10 120 \
      python tools/repeat_probe.py 512 2000 $L $L 60 || exit $?
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04d_race.log

#!/bin/bash
# Build forward-kernel variants into abl/<name>/libmpvae_hip.so:
#   tools/studies/abl_fwd.sh name "-DFLAG=1 -DOTHER=2" [name "flags"] ...
set -e
R="$(cd "$(dirname "$0")/../.." && pwd)"
cd "$R/mpvae-1_amd" && make -s >/dev/null
while [ $# -gt 1 ]; do
  n=$1; f=$2; shift 2
  mkdir -p "$R/abl/$n"
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -Icsrc $f \
      -c csrc/probit_fwd.hip -o "$R/abl/$n/probit_fwd.o" 2>/dev/null &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
      -o "$R/abl/$n/libmpvae_hip.so" "$R/abl/$n/probit_fwd.o" build/probit_bwd.o build/util.o build/linear.o \
      build/fairness.o && echo "built $n" ) &
done
wait

#!/bin/bash
# Timing ablations of the GEMM kernels (MPV_ABL bits in probit_fwd.hip / probit_bwd.hip): builds libmpvae_hip.so variants
# with -DMPV_ABL=<bits> (see probit_fwd.hip) into abl/<bits>/ (build here),
# or times them on the GPU box (run).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
VARIANTS="${VARIANTS:-0 1 5 9 17 13 25}"
case "$1" in
  build)
    cd "$R/mpvae-1_amd" && make -s >/dev/null || exit 1
    for a in $VARIANTS; do
      mkdir -p "$R/abl/$a"
      for f in probit_fwd probit_bwd; do
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -Icsrc \
          -DMPV_ABL=$a -c csrc/$f.hip -o "$R/abl/$a/$f.o" &
      done
    done
    wait
    for a in $VARIANTS; do
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
        -o "$R/abl/$a/libmpvae_hip.so" "$R/abl/$a/probit_fwd.o" "$R/abl/$a/probit_bwd.o" \
        build/util.o || exit 1
    done ;;
  run)
    mkdir -p "$R/gpurun_out/abl"
    for a in $VARIANTS; do
      MPVAE_HIP_LIB="$R/abl/$a/libmpvae_hip.so" timeout -k 10 300 python "$R/bench.py" --steps 5 --warmup 2 \
        --no-cpu-baseline > "$R/gpurun_out/abl/$a.json" 2> "$R/gpurun_out/abl/$a.err" || exit $?
      python -c "import json;d=json.load(open('$R/gpurun_out/abl/$a.json'));r=d['roofline']['per_launch_ms'];print('abl',$a,'fwd',r['probit_fwd'],'dR',r['dR_gemm'])"
    done ;;
esac

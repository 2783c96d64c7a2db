#!/bin/bash
# Timing ablations of the GEMM kernels: builds libmpvae_hip.so variants into
# abl/<variant>/ (here: `build`) and times them on the GPU box (`run`).
# A variant is <bits>[:<extra>...]: <bits> = MPV_ABL (probit_fwd.hip /
# probit_bwd.hip / util.hip); each ':'-separated extra is MACRO=value (-D) or a raw -flag.
# The MPV_ABL hooks are not in the product sources: tools/studies/ablation_hooks.patch
# adds them to a copy of csrc/ per variant (with MPV_ABL=0 the product's ISA).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
VARIANTS="${VARIANTS:-0 1 5 9 17 13 25}"
dir_of() { echo "$R/abl/$(echo "$1" | tr ':=' '__' | tr -d ' ')"; }
case "$1" in
  build)
    cd "$R/mpvae-1_amd" && make -s >/dev/null || exit 1
    for v in $VARIANTS; do
      d=$(dir_of "$v"); mkdir -p "$d"
      rm -rf "$d/csrc" && cp -r csrc "$d/csrc" && patch -s -p1 -d "$d/csrc" < "$R/tools/studies/ablation_hooks.patch" || exit 1
      bits=${v%%:*}; extra=""
      if [[ "$v" == *:* ]]; then   # extras: MACRO=value or a raw -flag, ':'-separated
        IFS=':' read -ra parts <<< "${v#*:}"
        for x in "${parts[@]}"; do [[ "$x" == -* ]] && extra="$extra $x" || extra="$extra -D$x"; done
      fi
      for f in probit_fwd probit_bwd util; do
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -I"$d/csrc" \
          -DMPV_ABL=$bits $extra -c "$d/csrc/$f.hip" -o "$d/$f.o" &
      done
    done
    wait
    for v in $VARIANTS; do
      d=$(dir_of "$v")
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
        -o "$d/libmpvae_hip.so" "$d/probit_fwd.o" "$d/probit_bwd.o" "$d/util.o" \
        $(ls build/*.o | grep -v "build/probit_\|build/util.o") || exit 1
    done ;;
  run)
    mkdir -p "$R/gpurun_out/abl"
    for v in $VARIANTS; do
      d=$(dir_of "$v"); n=$(basename "$d")
      MPVAE_HIP_LIB="$d/libmpvae_hip.so" timeout -k 10 300 python "$R/bench.py" --steps 5 --warmup 2 \
        --no-cpu-baseline > "$R/gpurun_out/abl/$n.json" 2> "$R/gpurun_out/abl/$n.err" || exit $?
      python -c "import json;d=json.load(open('$R/gpurun_out/abl/$n.json'));r=d['roofline']['ms_per_step_by_op'];print('$v',r,'step',round(d['ms_per_step'],2))"
    done ;;
esac

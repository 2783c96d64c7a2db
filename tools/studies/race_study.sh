#!/bin/bash
# Round-4 study of the round-3 lost-update race ("the
# 128-label forward tile and repeatability"): libmpvae_hip.so variants with
# tools/studies/race_study.patch applied and MPV_RACE bits set (bit 0: the 4-wave,
# two-workgroups-per-CU 128 x 128 tile for 96 < L <= 128; the other bits: one
# candidate fix each, see the patch; round 5 added 32768: drain every counter
# and barrier at the K-loop exit, 65536: the stage copies by plain loads +
# ds_write instead of LDS-DMA), built here (`build`) and probed for
# bitwise repeatability on the GPU box (`run`).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
VARIANTS="${VARIANTS:-1 17 32769 65537}"
case "$1" in
  build)
    cd "$R/mpvae-1_amd" && make -s >/dev/null || exit 1
    for v in $VARIANTS; do
      d="$R/abl/race$v"; rm -rf "$d"; mkdir -p "$d"
      cp -r csrc "$d/csrc" && patch -s -p1 -d "$d/csrc" < "$R/tools/studies/race_study.patch" || exit 1
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -I"$d/csrc" \
        -DMPV_RACE=$v -c "$d/csrc/probit_fwd.hip" -o "$d/probit_fwd.o" &
    done
    wait
    for v in $VARIANTS; do
      d="$R/abl/race$v"
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
        -o "$d/libmpvae_hip.so" "$d/probit_fwd.o" $(ls build/*.o | grep -v "build/probit_fwd.o") || exit 1
    done ;;
  run)
    for v in $VARIANTS; do
      for L in 128 100; do
        MPVAE_HIP_LIB="$R/abl/race$v/libmpvae_hip.so" timeout -k 10 120 \
          python "$R/tools/repeat_probe.py" 512 2000 $L $L ${RUNS:-40} || exit $?
      done
    done ;;
esac

#!/bin/bash
# GRBM_GUI_ACTIVE (effective clock) per ablation variant
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/clk"; cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  MPVAE_HIP_LIB="$R/abl/$v/libmpvae_hip.so" timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "probit_fwd|dR16|bwd_elem|noise" -f csv -d "$R/gpurun_out/clk/$v" -o c -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/clk/$v.json" 2>"$R/gpurun_out/clk/$v.err" || exit $?
  echo "[$v] done"
done

#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. PMC FETCH_SIZE pass, 3. PMC WRITE_SIZE pass (separate passes: TCC slots)
#   4. (STEPS="... valu") SQ_INSTS_VALU / SQ_INSTS_MFMA / GRBM_GUI_ACTIVE of every kernel
# Outputs under gpurun_out/prof/<tag>/; copy the summaries into profiles/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-c4}"
# the bench's own default step counts (so the trace matches its timed steps)
ARGS="${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline}"
OUT="$R/gpurun_out/prof/$TAG"
KRE="${KRE:-probit_fwd|dR16|dR_gemm|bwd_elem|noise_philox}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" -f csv -d "$OUT/$name" -o "$name" -- \
      python3 "$R/bench.py" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.err"; exit $rc; }
}
STEPS="${STEPS:-trace fetch write}"
for s in $STEPS; do
  case $s in
    trace) run trace --kernel-trace --stats ;;
    fetch) run fetch --pmc FETCH_SIZE --kernel-include-regex "$KRE" ;;
    write) run write --pmc WRITE_SIZE --kernel-include-regex "$KRE" ;;
    valu) run valu --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "${VKRE:-mpv::}" ;;
  esac
done
find "$OUT" -name "*.csv" | head -20

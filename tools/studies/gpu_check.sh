#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench.  Stops at the first step that
# ends in a signal / timeout (GPU fault, abort, hang); test failures (rc 1) go on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ok_or_fail() {  # rc, step
  local rc=$1
  echo "[$2] rc=$rc" | tee -a gpurun_out/steps.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2 (rc=$rc)"; exit "$rc"; fi
}
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
           ok_or_fail $? tests; tail -30 gpurun_out/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
           ok_or_fail $? smoke; tail -5 gpurun_out/smoke.log ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
           ok_or_fail $? bench; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json ;;
  esac
done

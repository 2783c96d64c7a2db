#!/bin/bash
# Round-3 GPU pass: parity suite (measured errors recorded), smoke, A/B of the
# round-2 library (abl/base) against the current one at C4 / C2 / C3, and the
# train-step profile.  Stops at the first step that times out or crashes.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r3c}"
mkdir -p "$O"
cd "$R"
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err"
  local rc=$?
  echo "[$n] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 "$O/$n.err"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  MPVAE_RECORD_ERRS="$O/parity_errs.jsonl" step tests 900 python -u -m pytest tests -m gpu -q \
    --timeout 150 --timeout-method thread -rf
  tail -4 "$O/tests.out"
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 "$O/smoke.out"
fi
for rep in 1 2; do
  for v in base new; do
    lib="$R/mpvae-1_amd/libmpvae_hip.so"; [ $v = base ] && lib="$R/abl/base/libmpvae_hip.so"
    MPVAE_HIP_LIB=$lib step c4_${v}_$rep 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3
    python -c "import json;d=json.load(open('$O/c4_${v}_$rep.out'));print('c4 $v',round(d['ms_per_step'],3),d['roofline']['ms_per_step_by_op'])"
    for c in c2 c3; do
      MPVAE_HIP_LIB=$lib step ${c}g_${v}_$rep 200 python bench.py --config $c --graph --steps 50 --warmup 10 --no-cpu-baseline
      python -c "import json;d=json.load(open('$O/${c}g_${v}_$rep.out'));print('$c graph $v',round(d['ms_per_step'],4),d['roofline']['ms_per_step_by_op'])"
    done
  done
done
step ts_c2 200 python tools/trainstep_profile.py --config c2
python -c "import json;d=json.load(open('$O/ts_c2.out'));print({k:d[k] for k in ('eager_ms','trainstep_ms','graph_ms','phases_ms')}, d['kernels'].get('per_step_ms_total'), d['kernels'].get('launches_per_step'))"
echo done

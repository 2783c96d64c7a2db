#!/bin/bash
# mpv_linear on one GPU box: its parity tests (errors recorded), the VAE / step
# tests, the train step at C1-C3 (hip) and one aten-op listing.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out/${OUT:-lin}"
mkdir -p "$O"
cd "$R"
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err"
  local rc=$?
  echo "[$n] rc=$rc"
  [ $rc -eq 0 ] || { tail -40 "$O/$n.out"; tail -10 "$O/$n.err"; exit $rc; }
}
MPVAE_RECORD_ERRS="$O/errs.jsonl" step tests 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_vae.py \
  -m gpu -q --timeout 150 --timeout-method thread -rf
tail -2 "$O/tests.out"
for c in c1 c2 c3; do
  step ts_${c} 300 python tools/trainstep_profile.py --config $c --linear hip $([ $c = c2 ] && echo --ops)
  python -c "import json;d=json.load(open('$O/ts_${c}.out'));print('ts $c',{k:d[k] for k in ('eager_ms','trainstep_ms','graph_ms')}, d['kernels'].get('per_step_ms_total'), d['kernels'].get('launches_per_step'))"
done
echo done

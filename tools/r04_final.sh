#!/bin/bash
# Round-4 evidence on one GPU box, in two calls (each fits gpurun's limit):
#   PART=tests tools/r04_final.sh   GPU suite (measured errors recorded), smoke,
#                                   repeatability probes of the dispatched tiles
#   PART=bench tools/r04_final.sh   bench lines, train-step profiles, rocprof
# Stops at the first step that fails, times out or crashes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-r4final}"
mkdir -p "$O"
cd "$R"
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err"
  local rc=$?
  echo "[$n] rc=$rc"
  [ $rc -eq 0 ] || { tail -30 "$O/$n.out"; tail -10 "$O/$n.err"; exit $rc; }
}
b() {  # name, bench args...
  local n=$1; shift
  step "$n" 400 python bench.py "$@"
  python -c "import json;d=json.load(open('$O/$n.out'));print('$n',round(d['ms_per_step'],4),'%.4g'%d['value'],d['roofline'].get('frac'))"
}
if [ "$PART" = tests ]; then
  MPVAE_RECORD_ERRS="$O/parity_errs.jsonl" step tests 1000 python -u -m pytest tests -m gpu -q \
    --timeout 150 --timeout-method thread -rf
  tail -3 "$O/tests.out"
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  # dispatched forward tiles: 48 (C2), 96 (C3), 128 (L=100, L=128), 256 (C4 shape, small S)
  for shp in "128 1000 38 38" "256 2000 81 81" "64 1000 100 100" "64 1000 128 128" "16 1024 1024 1024"; do
    n=probe_$(echo $shp | tr ' ' _)
    PROBE_BWD=1 step "$n" 300 python tools/repeat_probe.py $shp 30
    cat "$O/$n.out"
  done
else
  b c4_bench
  # one rank's share of the strong-scaling C4 step at 8 GPUs, plain and sharded path
  b c4_s512_bench --n-sample 512 --no-cpu-baseline
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 MPVAE_FORCE_DIST=1 \
    step c4_s512_dist_bench 400 python bench.py --n-sample 512 --no-cpu-baseline
  grep -h '^{' "$O/c4_s512_dist_bench.out" | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4_s512_dist',round(d['ms_per_step'],4))"
  b c4eval_bench --mode eval --no-cpu-baseline
  b c2_bench --config c2 --no-cpu-baseline
  b c2graph_bench --config c2 --graph --no-cpu-baseline
  b c3_bench --config c3 --no-cpu-baseline
  b c3graph_bench --config c3 --graph --no-cpu-baseline
  b c5_1gpu_bench --config c5 --steps 3 --warmup 1 --no-cpu-baseline
  # the drop-in training step: Linear layers on mpv_linear (default), on
  # nn.Linear with hipBLASLt (torch's default) and with rocBLAS
  for c in c1 c2 c3; do
    for v in hip torch_cublaslt torch_cublas; do
      lin=${v%%_*}; bl=${v#*_}; extra=""
      [ "$lin" = torch ] && extra="--blas $bl"
      step ts_${c}_$v 300 python tools/trainstep_profile.py --config $c --linear $lin $extra \
        $([ $c = c2 ] && [ $lin = hip ] && echo --ops)
      python -c "import json;d=json.load(open('$O/ts_${c}_$v.out'));print('ts $c $v',{k:d[k] for k in ('eager_ms','trainstep_ms','graph_ms')})"
    done
  done
  TAG=r4_c4 bash tools/profile.sh || exit 1
fi
echo done

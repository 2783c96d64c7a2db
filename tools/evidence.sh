#!/bin/bash
# Evidence runs on one GPU box (run through gpurun), one PART per call so each
# fits gpurun's limit.  Replaces the round-scoped drivers of rounds 2-4 (their
# text stays in git history).  Output: gpurun_out/$OUT (default ev_$PART).
#
#   PART=tests    GPU suite (measured errors recorded in parity_errs.jsonl),
#                 smoke(), NaN-poisoned repeatability probes of every
#                 dispatched forward tile (forward and backward)
#   PART=bench    bench lines: C4 (headline), eval, C2 / C3 eager and graph
#                 (C2 / C3 with the VALU roofline), C5 on one GPU, then the
#                 rocprof trace + PMC passes of the headline (tools/profile.sh)
#   PART=profsmall  rocprof trace + FETCH / WRITE / VALU passes at C2 and C3
#   PART=scaling  one rank's share of the strong-scaling C4 step at 8 GPUs on
#                 one GPU: n_sample 4096 vs 512, plain and through the sharded
#                 path on a world-of-one RCCL group (MPVAE_FORCE_DIST=1)
#   PART=gloo2    the N-rank bench path rehearsed with two gloo ranks on one
#                 GPU (strong scaling at C4; comm_ms per rank; not a scaling number)
#   PART=trainstep  the drop-in training step (tools/trainstep_profile.py) at C1-C3
# Stops at the first step that fails, times out or crashes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-ev_$PART}"
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
  python -c "import json;d=json.load(open('$O/$n.out'));r=d['roofline'];print('$n',round(d['ms_per_step'],4),'%.4g'%d['value'],r.get('bound'),r.get('frac'))"
}
case "$PART" in
tests)
  MPVAE_RECORD_ERRS="$O/parity_errs.jsonl" step tests 1000 python -u -m pytest tests -m gpu -q \
    --timeout 150 --timeout-method thread -rf
  tail -3 "$O/tests.out"
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  # dispatched forward tiles: 48 (C2, two workgroups per CU), 96 (C3), 128
  # (L=100, L=128), 256 (C4 shape, small S); every launch NaN-poisoned
  for shp in ${PROBE_SHAPES:-"128 1000 38 38" "256 2000 81 81" "64 1000 100 100" "64 1000 128 128" "16 1024 1024 1024"}; do
    n=probe_$(echo $shp | tr ' ' _)
    PROBE_BWD=1 step "$n" 300 python tools/repeat_probe.py $shp ${PROBE_RUNS:-30}
    cat "$O/$n.out"
  done
  ;;
bench)
  b c4_bench
  b c4eval_bench --mode eval --no-cpu-baseline
  b c2_bench --config c2 --no-cpu-baseline
  b c2graph_bench --config c2 --graph --no-cpu-baseline
  b c3_bench --config c3 --no-cpu-baseline
  b c3graph_bench --config c3 --graph --no-cpu-baseline
  b c5_1gpu_bench --config c5 --no-cpu-baseline
  TAG=${TAG:-c4} bash tools/profile.sh || exit 1
  ;;
profsmall)
  # C2 / C3: trace + HBM + VALU passes (the VALU roofline and frac_algorithmic
  # of bench.py read these once committed as profiles/<round>_c{2,3}_pmc.json)
  for c in ${PROF_CONFIGS:-c2 c3}; do
    TAG=$c BENCH_ARGS="--config $c --steps 50 --warmup 5 --no-cpu-baseline" \
      STEPS="trace fetch write valu" bash tools/profile.sh || exit 1
  done
  ;;
scaling)
  for S in 4096 512; do
    b s$S --n-sample $S --no-cpu-baseline
    RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2952$((S % 7)) \
      MPVAE_FORCE_DIST=1 step dist_s$S 400 python bench.py --n-sample $S --no-cpu-baseline
  done
  python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
r = {}
for f in ["s4096", "s512", "dist_s4096", "dist_s512"]:
    lines = [l for l in open(f"{o}/{f}.out") if l.startswith("{")]
    d = json.loads(lines[-1])
    r[f] = d["ms_per_step"]
    print(f, round(d["ms_per_step"], 3), d.get("comm_ms"), d["roofline"]["ms_per_step_by_op"])
print("fixed overhead at S_local=512 vs 1/8 of 4096: plain %.1f %%, sharded path %.1f %%" % (
    100 * (r["s512"] / (r["s4096"] / 8) - 1), 100 * (r["dist_s512"] / (r["s4096"] / 8) - 1)))
PY
  ;;
gloo2)
  MPVAE_DIST_BACKEND=gloo step c4_gloo2 400 python bench.py --gpus 2 --steps 5 --warmup 2 \
    --no-cpu-baseline
  grep -h '^{' "$O/c4_gloo2.out" | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['n_gpus'],d['scaling'],d['config']['n_sample'],round(d['ms_per_step'],2),d.get('comm_ms'))"
  ;;
trainstep)
  for c in c1 c2 c3; do
    step ts_$c 300 python tools/trainstep_profile.py --config $c --linear hip
    python -c "import json;d=json.load(open('$O/ts_$c.out'));print('ts $c',{k:d[k] for k in ('eager_ms','trainstep_ms','graph_ms')})"
  done
  ;;
*)
  echo "PART must be tests, bench, profsmall, scaling, gloo2 or trainstep"; exit 2 ;;
esac
echo done

#!/bin/bash
# Round-end evidence on one GPU box: GPU tests, smoke, bench lines, rocprof.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/final"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
b() {  # name, args
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['ms_per_step'],3),d['value'])"
}
b c4_bench
b c2_bench --config c2 --no-cpu-baseline
b c2graph_bench --config c2 --graph --no-cpu-baseline
b c3_bench --config c3 --no-cpu-baseline
b c3graph_bench --config c3 --graph --no-cpu-baseline
b c4eval_bench --mode eval --no-cpu-baseline
bash tools/profile.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/rp" -o rp -- python3 bench.py --no-cpu-baseline > "$O/c4_bench_under_rocprof.json" 2> "$O/rp.err" || exit 1
echo done

#!/bin/bash
# Small-config bench lines (C2, C3; eager and HIP graph) into gpurun_out/final/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/final"
mkdir -p "$O"
cd "$R"
b() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['ms_per_step'],3),d['value'])"
}
b c2_bench --config c2 --no-cpu-baseline
b c2graph_bench --config c2 --graph --no-cpu-baseline
b c3_bench --config c3 --no-cpu-baseline
b c3graph_bench --config c3 --graph --no-cpu-baseline

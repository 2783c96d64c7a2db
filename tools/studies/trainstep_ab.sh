#!/bin/bash
# GPU suite, then the drop-in train step at C1-C3 in two variants, alternated
# on one box (A/B): the current tree ("a") and the tree with $B_ARGS passed to
# tools/trainstep_profile.py ("b", default --no-passthrough).  Stops at the
# first failing step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out/${OUT:-trainstep_ab}"
mkdir -p "$O"
cd "$R"
MPVAE_RECORD_ERRS="$O/parity_errs.jsonl" timeout -k 10 600 python -u -m pytest tests -m gpu -q \
  --timeout 150 --timeout-method thread -rf > "$O/tests.out" 2>&1 || { tail -30 "$O/tests.out"; exit 1; }
tail -1 "$O/tests.out"
for rep in 1 2; do
  for c in c1 c2 c3; do
    for v in a b; do
      extra=""; [ $v = b ] && extra="${B_ARGS:---no-passthrough}"
      timeout -k 10 300 python tools/trainstep_profile.py --config $c $extra > "$O/ts_${c}_${v}_$rep.out" \
        2> "$O/ts_${c}_${v}_$rep.err" || { tail -5 "$O/ts_${c}_${v}_$rep.err"; exit 1; }
      python -c "import json;d=json.load(open('$O/ts_${c}_${v}_$rep.out'));print('$c $v $rep',{k:d[k] for k in ('eager_ms','trainstep_ms','graph_ms','updates')}, d['kernels'].get('launches_per_step'))"
    done
  done
done
echo done

#!/bin/bash
# the N-rank bench path rehearsed on one GPU: two gloo ranks (both on cuda:0),
# strong scaling at C4 (n_sample 4096 split 2048 + 2048); not a scaling number
set -o pipefail
mkdir -p gpurun_out
MPVAE_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 \
  --no-cpu-baseline > gpurun_out/r04k_c4_gloo2.json 2> gpurun_out/r04k_c4_gloo2.err || { tail -20 gpurun_out/r04k_c4_gloo2.err; exit 1; }
grep -h '^{' gpurun_out/r04k_c4_gloo2.json | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['n_gpus'],d['scaling'],d['config']['n_sample'],d['config']['workload'],round(d['ms_per_step'],2))"

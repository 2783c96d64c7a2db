#!/bin/bash
# round 4, first GPU pass: the new parity / StepLR / scaling tests, the C4
# bench, and the strong-scaling share (n_sample 512 = 4096 / 8) on one GPU
set -o pipefail
mkdir -p gpurun_out
export MPVAE_RECORD_ERRS=$PWD/gpurun_out/r04a_errs.jsonl
rm -f "$MPVAE_RECORD_ERRS"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_vae.py tests/test_gpu_fair.py tests/test_gpu_dist.py \
  "tests/test_gpu_parity.py::test_c4_full_size_against_fp64_reference" \
  "tests/test_gpu_parity.py::test_c4_dims_long_reduction_against_oracle" \
  > gpurun_out/r04a_tests.log 2>&1 || { tail -30 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
for S in 4096 512; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --n-sample $S \
    > gpurun_out/r04a_bench_s$S.json 2> gpurun_out/r04a_bench_s$S.err || exit 1
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2951$((S % 7)) MPVAE_FORCE_DIST=1 \
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --n-sample $S \
    > gpurun_out/r04a_bench_dist_s$S.json 2> gpurun_out/r04a_bench_dist_s$S.err || exit 1
done
python - <<'PY'
import json
for f in ["s4096", "s512", "dist_s4096", "dist_s512"]:
    d = json.load(open(f"gpurun_out/r04a_bench_{f}.json"))
    print(f, round(d["ms_per_step"], 3), d["roofline"]["ms_per_step_by_op"])
PY

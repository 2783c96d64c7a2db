#!/bin/bash
# strong-scaling fixed costs on one GPU: the C4 step at n_sample 4096 and at
# one rank's share of 8 (512), eager, plain and through the sharded path
# (MPVAE_FORCE_DIST=1: the exchange's collectives on a world-of-one RCCL group)
set -o pipefail
mkdir -p gpurun_out
for S in 4096 512; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --n-sample $S \
    > gpurun_out/r04g_bench_s$S.json 2> gpurun_out/r04g_bench_s$S.err || exit 1
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2952$((S % 7)) MPVAE_FORCE_DIST=1 \
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --n-sample $S \
    > gpurun_out/r04g_bench_dist_s$S.json 2> gpurun_out/r04g_bench_dist_s$S.err || exit 1
done
python - <<'PY'
import json
r = {}
for f in ["s4096", "s512", "dist_s4096", "dist_s512"]:
    d = json.load(open(f"gpurun_out/r04g_bench_{f}.json"))
    r[f] = d["ms_per_step"]
    print(f, round(d["ms_per_step"], 3), d["roofline"]["ms_per_step_by_op"])
print("fixed overhead at S_local=512 vs 1/8 of 4096: plain %.1f %%, sharded path %.1f %%" % (
    100 * (r["s512"] / (r["s4096"] / 8) - 1), 100 * (r["dist_s512"] / (r["s4096"] / 8) - 1)))
PY

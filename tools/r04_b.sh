#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/c4_spread.py --seeds 1 2 3 4 5 > gpurun_out/r04b_spread.log 2>&1 || { tail -20 gpurun_out/r04b_spread.log; exit 1; }
tail -5 gpurun_out/r04b_spread.log
./tools/race_study.sh run 2>&1 | tee gpurun_out/r04b_race.log

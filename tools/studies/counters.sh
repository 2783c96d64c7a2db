#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 --pmc run per set) on the bench workload.
# Usage on the GPU box: SETS="A B" bash tools/studies/counters.sh ; results in gpurun_out/ctr/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="${CTR_OUT:-$R/gpurun_out/ctr}"
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline}"
KRE="${KRE:-probit_fwd|dR16|dR_gemm|bwd_elem|noise}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
declare -A SET
SET[A]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
SET[B]="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
SET[C]="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
SET[D]="TCC_HIT_sum TCC_MISS_sum"
SET[E]="TA_BUSY_avr TA_FLAT_READ_LDS_WAVEFRONTS_sum"
SET[H]="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
SET[F]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
SET[G]="TCC_BUSY_avr TCC_TAG_STALL_sum GRBM_GUI_ACTIVE TCC_REQ_sum"
for s in ${SETS:-A B C D}; do
  timeout -k 10 ${SET_TIMEOUT:-240} rocprofv3 --pmc ${SET[$s]} --kernel-include-regex "$KRE" -f csv \
      -d "$OUT/$s" -o "$s" -- python3 "$R/bench.py" $ARGS > "$OUT/$s.json" 2> "$OUT/$s.err"
  rc=$?
  echo "[set $s] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$s.err"; [ $rc -eq 1 ] || exit $rc; fi
done

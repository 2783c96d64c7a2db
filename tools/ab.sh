#!/bin/bash
# A/B of library variants on one GPU: bench lines and repeatability probes.
#   CFGS="c3" VARIANTS="new a5" PROBE="256 2000 81 81 30" tools/ab.sh
# "new" is the in-tree library, anything else abl/<name>/libmpvae_hip.so.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${OUT:-ab}"
mkdir -p "$O"
cd "$R"
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[$n] rc=$rc"; tail -5 "$O/$n.err"; exit $rc; fi
  return 0
}
lib_of() {  # new: in-tree; a name with a slash: that directory; else abl/<name>
  case "$1" in
    new) echo "$R/mpvae-1_amd/libmpvae_hip.so" ;;
    */*) echo "$R/$1/libmpvae_hip.so" ;;
    *) echo "$R/abl/$1/libmpvae_hip.so" ;;
  esac
}
for rep in ${REPS:-1 2}; do
  for v in $VARIANTS; do
    vn=${v//\//_}
    for c in $CFGS; do
      g=--graph; [ "$c" = c4 ] || [ "$c" = c5 ] && g=
      MPVAE_HIP_LIB=$(lib_of $v) step ${c}_${vn}_$rep 300 python bench.py --config $c $g \
        --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline $BENCH_EXTRA
      python -c "import json;d=json.load(open('$O/${c}_${vn}_$rep.out'));print('$c $v',round(d['ms_per_step'],4),d['roofline']['ms_per_step_by_op'])"
    done
  done
done
if [ -n "$PROBE" ]; then
  for v in $VARIANTS; do
    vn=${v//\//_}
    MPVAE_HIP_LIB=$(lib_of $v) PROBE_BWD=1 step probe_$vn 300 python tools/repeat_probe.py $PROBE
    cat "$O/probe_$vn.out"
  done
fi
echo done

cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp
timeout -k 10 600 python -m pytest -q -x tests -m gpu > gpurun_out/exp/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/exp/tests.log
[ $rc -le 1 ] || exit $rc
for v in 0 2 1; do
  MPV_FWD_VAR=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/exp/v$v.json 2>gpurun_out/exp/v$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/exp/v$v.json'));r=d['roofline']['per_launch_ms'];print('var',$v, round(d['ms_per_step'],2), 'fwd', r['probit_fwd'])"
done

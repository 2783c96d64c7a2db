# A/B of dR variants at the small configs (tools/studies/ablate.sh build first)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/parity.log 2>&1
tail -1 gpurun_out/ab/parity.log
for c in c2 c3; do for v in ${VARIANTS:-0}; do
  MPVAE_HIP_LIB=$R/abl/$v/libmpvae_hip.so timeout -k 10 200 python bench.py --config $c --graph --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$c$v.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab/$c$v.json'));print('$c','$v',round(d['ms_per_step'],4),d['roofline'].get('ms_per_step_by_op'))"
done; done

# dev probe for the exact WebP coder: byte tests, the coder alone, the pipeline (A/B knobs via env)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_vp8x.py -q -x --timeout 120 --timeout-method thread > gpurun_out/vp8x_tests.log 2>&1 || { tail -30 gpurun_out/vp8x_tests.log; exit 1; }
tail -1 gpurun_out/vp8x_tests.log
timeout -k 10 200 python -u tools/vp8x_timing.py --n 64 --iters 3 > gpurun_out/vp8x_timing.log 2>&1 || exit 1
tail -1 gpurun_out/vp8x_timing.log
B="--webp-encoder exact --no-cpu-baseline --no-extras --no-pcie-leg --pageable-steps 0"
for g in ${GRIDS:-1}; do
  IK_VP8X_GRID=$g timeout -k 10 300 python -u bench.py $B > gpurun_out/bx_g$g.json 2> gpurun_out/bx_g$g.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bx_g$g.json').read().strip().splitlines()[-1]); p=d['png_decode_stages_ms']; print('grid x$g', d['value'], d['ms_per_step'], 'kstage', p['kernel_stage_wall'], 'dec', p['decode'], 'exp', p['expand'], 'res', p['resolve'], 'cores', d['host_cpu']['per_rank_cores_busy'])"
done

# round-3: decode lanes paired long+short across the wave rounds -- PNG parity, then the A/B
set -o pipefail
export TMPDIR=/tmp
T=r03t
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_png16.py tests/test_gpu_alpha.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'resolve', s['resolve'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
for v in 1 0 1; do
  IK_PNG_LANE_ORDER=$v timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_ord$v.json 2> gpurun_out/${T}_ord$v.err || { tail -5 gpurun_out/${T}_ord$v.err; exit 1; }
  show gpurun_out/${T}_ord$v.json
done

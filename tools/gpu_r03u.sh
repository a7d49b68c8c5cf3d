# round-3: decode lane order (linear bucket sort) A/B with the host stage timings,
# then the block search's phase clock (IK_FIND_PROF dev build)
set -o pipefail
export TMPDIR=/tmp
T=r03u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'resolve', s['resolve'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
for v in 1 0 1; do
  IK_PNG_TIMING=1 IK_PNG_LANE_ORDER=$v timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_ord$v.json 2> gpurun_out/${T}_ord$v.err || { tail -5 gpurun_out/${T}_ord$v.err; exit 1; }
  show gpurun_out/${T}_ord$v.json
  grep "host: plan" gpurun_out/${T}_ord$v.err | tail -2
done
IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_exp/libimagekit_hip_findprof.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_findprof.json 2> gpurun_out/${T}_findprof.err || { tail -5 gpurun_out/${T}_findprof.err; exit 1; }
grep "find-prof" gpurun_out/${T}_findprof.err | tail -3

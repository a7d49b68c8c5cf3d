# round-3: first decode round's lane plans and lane table built in parallel over the
# jobs: PNG GPU tests, then the headline bench twice with the host stage timings
set -o pipefail
export TMPDIR=/tmp
T=r03aa
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_png16.py tests/test_gpu_alpha.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'resolve', s['resolve'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
for r in 1 2; do
  IK_PNG_TIMING=1 timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_run$r.json 2> gpurun_out/${T}_run$r.err || { tail -5 gpurun_out/${T}_run$r.err; exit 1; }
  show gpurun_out/${T}_run$r.json
  grep "host: plan" gpurun_out/${T}_run$r.err | tail -2
done
# bound on the expand kernel's far-source loads: a dev build reads them from the LDS
# ring instead (wrong pixels; the bench does not check them) -- expand ms only
IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_exp/libimagekit_hip_nofar.so timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_nofar.json 2> gpurun_out/${T}_nofar.err || { tail -5 gpurun_out/${T}_nofar.err; exit 1; }
show gpurun_out/${T}_nofar.json

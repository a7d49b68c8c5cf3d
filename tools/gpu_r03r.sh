# round-3: search queued behind the decode results copy, WebP planes in shared
# pinned blocks, 4-pixel JPEG colour kernel: parity tests, bench, host timings, trace
set -o pipefail
export TMPDIR=/tmp
T=r03r
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py tests/test_gpu_transform_batch.py tests/test_gpu_alpha.py tests/test_gpu_decode.py tests/test_gpu_jpeg_zune.py tests/test_gpu_pipeline.py tests/test_gpu_encode.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'resolve', s['resolve'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
show gpurun_out/${T}_bench.json
IK_PNG_TIMING=1 IK_TIMING=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_timing.json 2> gpurun_out/${T}_timing.err || { tail -5 gpurun_out/${T}_timing.err; exit 1; }
grep -E "^\[png\] host|^\[transform_batch\]|^\[png\] t=" gpurun_out/${T}_timing.err | tail -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -f csv -- python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo "PROFILE FAILED"; exit 1; }
show gpurun_out/${T}_prof.json
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_c2rst.json').read().strip().splitlines()[-1]); print('c2 rst', d['value'], d['ms_per_step'])"

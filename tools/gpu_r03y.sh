# round-3: progressive JPEG with restart intervals on the GPU (k_jpeg_prog) + the
# JPEG entropy decoder's word refill / per-lane rings at 32 intervals per wave:
# JPEG GPU tests, configs[2] with and without RSTn, the configs[3] loadtest mix
set -o pipefail
export TMPDIR=/tmp
T=r03y
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_jpeg_zune.py tests/test_gpu_transform_batch.py tests/test_gpu_headline_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
show gpurun_out/${T}_c2rst.json
timeout -k 10 500 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2norst.json 2> gpurun_out/${T}_c2norst.err || { tail -5 gpurun_out/${T}_c2norst.err; exit 1; }
show gpurun_out/${T}_c2norst.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c2prof -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2prof.json 2> gpurun_out/${T}_c2prof.err || { echo "C2 PROFILE FAILED"; exit 1; }
find gpurun_out/${T}_c2prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_c2_kernel_stats.csv \;
head -6 gpurun_out/${T}_c2_kernel_stats.csv | cut -c1-120
timeout -k 10 300 python tools/loadtest.py --requests 4096 --batch 64 --threads 16 --restart > gpurun_out/${T}_lt_rst.json 2> gpurun_out/${T}_lt_rst.err || { tail -5 gpurun_out/${T}_lt_rst.err; exit 1; }
tail -c 400 gpurun_out/${T}_lt_rst.json
timeout -k 10 300 python tools/loadtest.py --requests 4096 --batch 64 --threads 16 > gpurun_out/${T}_lt_norst.json 2> gpurun_out/${T}_lt_norst.err || { tail -5 gpurun_out/${T}_lt_norst.err; exit 1; }
tail -c 400 gpurun_out/${T}_lt_norst.json

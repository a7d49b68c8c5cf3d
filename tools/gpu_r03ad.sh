# round-3: JPEG interval decoder: block buffer in LDS + whole-block stores after the top-up, scan args in LDS, global-qualified bit source: JPEG GPU
# tests, then configs[2] with RSTn and its kernel stats
set -o pipefail
export TMPDIR=/tmp
T=r03ad
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_decode.py tests/test_gpu_transform_batch.py tests/test_gpu_pipeline.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
show gpurun_out/${T}_c2rst.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c2prof -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2prof.json 2> gpurun_out/${T}_c2prof.err || { echo "C2 PROFILE FAILED"; exit 1; }
find gpurun_out/${T}_c2prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_c2_kernel_stats.csv \;
head -8 gpurun_out/${T}_c2_kernel_stats.csv | cut -c1-120

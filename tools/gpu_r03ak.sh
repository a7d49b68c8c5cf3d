# round-3: JPEG colour row ends in their own small kernel (k_jpeg_color_ends): JPEG
# GPU tests (zune and libjpeg modes, batches), then configs[2] kernel stats and bench
set -o pipefail
export TMPDIR=/tmp
T=r03ak
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_decode.py tests/test_gpu_transform_batch.py tests/test_gpu_headline_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo "PROFILE FAILED"; tail -5 gpurun_out/${T}_prof.err; exit 1; }
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${T}_c2_kernel_stats.csv
grep -E "k_jpeg_color|k_jpeg_huff_batch" $f | cut -c1-150
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_c2rst.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'])"

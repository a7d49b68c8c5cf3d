# configs[4]-shape check: AVIF pipeline tests, then the 8192^2 -> 1024^2 Lanczos3
# AVIF q60 bench line and its rocprofv3 kernel stats.  Each step time-limited.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_encode.py tests/test_gpu_transform_batch.py tests/test_reference_api.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/c4_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/c4_tests.log; exit 1; }
tail -2 gpurun_out/c4_tests.log
C4="--size 8192 --out 1024 --filter lanczos3 --format avif --quality 60 --batch 32 --steps 3 --warmup 1"
timeout -k 10 400 python bench.py $C4 > gpurun_out/bench_c4_${TAG}.json 2> gpurun_out/bench_c4_${TAG}.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_c4_${TAG}.err; exit 1; }
cat gpurun_out/bench_c4_${TAG}.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_${TAG} -o run -f csv -- python bench.py $C4 --no-cpu-baseline > gpurun_out/bench_c4_prof_${TAG}.json 2> gpurun_out/bench_c4_prof_${TAG}.err || { echo "PROFILE FAILED"; exit 1; }
echo ok

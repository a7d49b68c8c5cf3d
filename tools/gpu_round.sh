# Full GPU check: all gpu tests, the default bench line, and rocprofv3 kernel-stats
# profiles of the bench (headline command without the alt-encoder leg, so the
# resize kernel's average matches the headline batch; then the GPU WebP encoder at
# batch 128).  Every step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -f csv -- python bench.py --no-cpu-baseline --no-alt-encoder --png-images 0 > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || { echo "PROFILE FAILED"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_gpuenc -o run -f csv -- python bench.py --no-cpu-baseline --no-alt-encoder --png-images 0 --webp-encoder gpu --batch 128 > gpurun_out/bench_prof_${TAG}_gpuenc.json 2> gpurun_out/bench_prof_${TAG}_gpuenc.err || { echo "PROFILE2 FAILED"; exit 1; }
echo ok

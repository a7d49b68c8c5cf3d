# Round-end GPU evidence: all gpu tests + smoke, the default bench line (with
# cpu_baseline), and the rocprofv3 kernel stats of the same bench command.
# Every step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/t_all.log; exit 1; }
  tail -2 gpurun_out/t_all.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 500 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -f csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || { echo "PROFILE FAILED"; exit 1; }
echo ok

# Quick GPU iteration: selected tests (first arg, pytest -k expression or file) then
# a short bench; every step time-limited, stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-tests/test_gpu_vp8.py}
shift || true
timeout -k 10 300 python -u -m pytest $T -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/q_tests.log; exit 1; }
tail -3 gpurun_out/q_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 "$@" > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/q_bench.err; exit 1; }
cat gpurun_out/q_bench.json

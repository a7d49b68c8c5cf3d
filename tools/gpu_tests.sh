# GPU test run: the -m gpu suite (one process, per-test timeout), then smoke().
# Usage (from the repo root, via gpurun): bash tools/gpu_tests.sh [test paths / pytest args...]
mkdir -p gpurun_out
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(tests)
timeout -k 10 900 python -u -m pytest "${args[@]}" -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -2 gpurun_out/smoke.log
exit $rc

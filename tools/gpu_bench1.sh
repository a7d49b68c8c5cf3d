mkdir -p gpurun_out
export IK_PNG_TIMING=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/png_tests.log 2>&1 || { tail -20 gpurun_out/png_tests.log; exit 1; }
tail -2 gpurun_out/png_tests.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
tail -c 3000 gpurun_out/bench1.json; grep "\[png\]" gpurun_out/bench1.err | tail -5
exit $rc

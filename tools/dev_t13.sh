set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_png16.py tests/test_gpu_headline_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t13_tests.log 2>&1 || { tail -30 gpurun_out/t13_tests.log; exit 1; }
tail -1 gpurun_out/t13_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 8 > gpurun_out/t13_bench.json 2> gpurun_out/t13_bench.err || exit 1
python tools/bench_summary.py gpurun_out/t13_bench.json | head -2

# round-3: next-batch block search gated on resolve; bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03g_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/r03g_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(d['png_decode_stages_ms'])"
exit $rc

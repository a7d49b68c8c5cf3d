# configs[3]: the loadtest mix, 10,000 requests, restart-free (headline, with the CPU leg) and restart-marked sources
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not repeated_batches" > gpurun_out/lt_tests.log 2>&1 || { tail -30 gpurun_out/lt_tests.log; exit 1; }
tail -1 gpurun_out/lt_tests.log
timeout -k 10 400 python tools/loadtest.py --requests 10000 --batch 64 --threads 16 --cpu-seconds 10 > gpurun_out/lt_norst.json 2> gpurun_out/lt_norst.err || { tail -5 gpurun_out/lt_norst.err; exit 1; }
cat gpurun_out/lt_norst.json
timeout -k 10 300 python tools/loadtest.py --requests 10000 --batch 64 --threads 16 --restart > gpurun_out/lt_rst.json 2> gpurun_out/lt_rst.err || { tail -5 gpurun_out/lt_rst.err; exit 1; }
cat gpurun_out/lt_rst.json

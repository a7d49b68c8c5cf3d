# round-3: device-resident inputs (ik_transform_batch_submit_device): parity tests, then the bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_parity.py tests/test_gpu_png.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r03j_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r03j_bench.json 2> gpurun_out/r03j_bench.err || { tail -20 gpurun_out/r03j_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03j_bench.json').read().strip().splitlines()[-1]); print('value', d['value'], d['ms_per_step']); print('pcie', d['pcie_inclusive']); print(d['png_decode_stages_ms']); print(d['kernels'])"
exit $rc

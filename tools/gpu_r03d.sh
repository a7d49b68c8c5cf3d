# round-3: resize A/B (pre-regression build vs now), PNG tests with the new block-search check, short bench
mkdir -p gpurun_out
for L in rust-image-transform_amd/lib_exp/old_2bfbfd0/libimagekit_hip.so rust-image-transform_amd/lib/libimagekit_hip.so; do
  timeout -k 10 120 python -u tools/resize_ab.py $PWD/$L >> gpurun_out/r03d_resize_ab.json 2>> gpurun_out/r03d_resize_ab.err || exit $?
done
cat gpurun_out/r03d_resize_ab.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03d_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r03d_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/r03d_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(d['png_decode_stages_ms']); print(d['kernels'])"
exit $rc

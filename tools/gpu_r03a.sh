# round-3 probe: the new full-size parity tests, then the resize-regression probe
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03a_parity.log 2>&1
rc=$?
tail -8 gpurun_out/r03a_parity.log
[ $rc -eq 0 ] || { echo "parity rc=$rc"; exit $rc; }
timeout -k 10 300 python -u tools/resize_regress.py > gpurun_out/r03a_resize.json 2> gpurun_out/r03a_resize.err
rc=$?
cat gpurun_out/r03a_resize.json; tail -3 gpurun_out/r03a_resize.err
exit $rc

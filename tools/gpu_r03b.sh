# round-3: the GPU suite (new staged pipeline), then a short bench and the resize probe.
# A test assertion failure still runs the bench; a timeout / abort / segfault stops here.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03b_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r03b_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
IK_PNG_TIMING=1 timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --hbm-steps 3 --jpeg-images 16 \
    > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err
brc=$?
tail -c 3000 gpurun_out/r03b_bench.json; grep -v "^\[png\] stream" gpurun_out/r03b_bench.err | tail -30
[ $brc -eq 0 ] || { echo "bench rc=$brc"; exit $brc; }
timeout -k 10 300 python -u tools/resize_regress.py > gpurun_out/r03b_resize.json 2> gpurun_out/r03b_resize.err
cat gpurun_out/r03b_resize.json; tail -3 gpurun_out/r03b_resize.err
exit $rc

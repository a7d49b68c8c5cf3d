# round-3: GPU suite, resize probe, find-kernel experiments (dev builds in lib_exp/)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03c_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r03c_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -u tools/resize_regress.py > gpurun_out/r03c_resize.json 2> gpurun_out/r03c_resize.err || exit $?
cat gpurun_out/r03c_resize.json
for v in base nocheck flush1 flush8; do
  if [ $v = base ]; then lp=rust-image-transform_amd/lib/libimagekit_hip.so; else lp=rust-image-transform_amd/lib_exp/$v/libimagekit_hip.so; fi
  IK_LIB_PATH=$PWD/$lp timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
      > gpurun_out/r03c_find_$v.json 2> gpurun_out/r03c_find_$v.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/r03c_find_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['kernels']['k_png_find'], d['png_decode_stages_ms']['decode'], d['png_decode_stages_ms']['decode_rounds'])"
done
exit $rc

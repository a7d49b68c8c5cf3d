# Dev A/B: the headline with lib_dev/libimagekit_hip_base.so (A) and lib/libimagekit_hip.so (B), alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not repeated_batches" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2; do
 for v in A B; do
  if [ $v = A ]; then export IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_dev/libimagekit_hip_base.so; else unset IK_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || { tail -5 gpurun_out/ab_$v$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v', d['value'], d['ms_per_step'], d['png_decode_stages_ms']['upload_find'], d['png_decode_stages_ms']['decode_wall_ms'])"
 done
done

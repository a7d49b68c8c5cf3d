set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resize.py tests/test_gpu_headline_parity.py tests/test_gpu_pipeline.py tests/test_gpu_resize_fma.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t11_tests.log 2>&1 || { tail -30 gpurun_out/t11_tests.log; exit 1; }
tail -1 gpurun_out/t11_tests.log
for v in rust-image-transform_amd/lib/libimagekit_hip.so rust-image-transform_amd/lib_ab/base.so; do
  timeout -k 10 120 python tools/resize_ab.py $v 3 256 >> gpurun_out/t11_rab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/resize_ab.py $v 4 64 >> gpurun_out/t11_rab.txt 2>&1 || exit 1
done
grep '^{' gpurun_out/t11_rab.txt
TAG=t11 STEPS="c2" bash tools/gpu_evidence.sh

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resize.py tests/test_gpu_headline_parity.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t9_tests.log 2>&1 || { tail -30 gpurun_out/t9_tests.log; exit 1; }
tail -1 gpurun_out/t9_tests.log
timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib/libimagekit_hip.so 3 256 > gpurun_out/t9_rab.txt 2>&1 || exit 1
timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib/libimagekit_hip.so 4 64 >> gpurun_out/t9_rab.txt 2>&1 || exit 1
grep '^{' gpurun_out/t9_rab.txt
TAG=t9 STEPS="c2" bash tools/gpu_evidence.sh

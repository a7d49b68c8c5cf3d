# Dev: GPU PNG / transform / encode tests, then the clients sweep
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_transform_batch.py tests/test_gpu_resize.py tests/test_gpu_encode.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not repeated_batches" > gpurun_out/png_tests.log 2>&1 || { tail -30 gpurun_out/png_tests.log; exit 1; }
tail -1 gpurun_out/png_tests.log
STEPS=8 CLIENTS="1" bash tools/gpu_clients.sh && STEPS=8 CLIENTS="2" EXTRA="--pipeline 0" bash tools/gpu_clients.sh

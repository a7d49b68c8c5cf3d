# Dev: GPU JPEG decode tests, then the JPEG legs (bench decode_inclusive_jpeg, loadtest)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_jpeg_zune.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not repeated_batches" > gpurun_out/jpeg_tests.log 2>&1 || { tail -30 gpurun_out/jpeg_tests.log; exit 1; }
tail -1 gpurun_out/jpeg_tests.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/jq_bench.json 2> gpurun_out/jq_bench.err || { tail -5 gpurun_out/jq_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/jq_bench.json'));print('jpeg leg', d['decode_inclusive_jpeg']['value'], 'headline', d['value'])"
timeout -k 10 300 python tools/loadtest.py --requests 4096 --batch 64 --threads 16 --restart > gpurun_out/jq_lt_rst.json 2> gpurun_out/jq_lt_rst.err || { tail -5 gpurun_out/jq_lt_rst.err; exit 1; }
timeout -k 10 300 python tools/loadtest.py --requests 4096 --batch 64 --threads 16 > gpurun_out/jq_lt_norst.json 2> gpurun_out/jq_lt_norst.err || { tail -5 gpurun_out/jq_lt_norst.err; exit 1; }
python -c "import json;print('loadtest rst', json.load(open('gpurun_out/jq_lt_rst.json'))['value'], 'norst', json.load(open('gpurun_out/jq_lt_norst.json'))['value'])"

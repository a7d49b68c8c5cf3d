# Dev: PNG GPU tests, then rocprofv3 kernel stats of a short headline bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not repeated_batches" > gpurun_out/png_tests.log 2>&1 || { tail -30 gpurun_out/png_tests.log; exit 1; }
tail -1 gpurun_out/png_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kst -o run -f csv -- python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-extras ${EXTRA:-} > gpurun_out/kst_bench.json 2> gpurun_out/kst_bench.err || { tail -5 gpurun_out/kst_bench.err; exit 1; }
python -c "
import json,csv
d=json.load(open('gpurun_out/kst_bench.json')); print(d['value'], d['ms_per_step'], d['png_decode_stages_ms'])
for r in csv.DictReader(open('gpurun_out/kst/run_kernel_stats.csv')):
    print('%-60s %6s %10.3f ms total %9.3f avg' % (r['Name'][:60], r['Calls'], int(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6))
" | head -14

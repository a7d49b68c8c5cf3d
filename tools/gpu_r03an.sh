# round-3: the default self-sync lane (2048 bits) under every GPU test, then 1024 vs
# 2048 bits on the restart-free loadtest mix and configs[2]
set -o pipefail
export TMPDIR=/tmp
T=r03an
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for L in 2048 1024; do
  IK_JPEG_SEQ_L=$L timeout -k 10 300 python tools/loadtest.py --requests 1024 --batch 64 --threads 16 > gpurun_out/${T}_lt_$L.json 2> gpurun_out/${T}_lt_$L.err || { tail -5 gpurun_out/${T}_lt_$L.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('L', sys.argv[2], 'loadtest norst', d['value'], d['batch_latency_ms'])" gpurun_out/${T}_lt_$L.json $L
  IK_JPEG_SEQ_L=$L timeout -k 10 500 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2_$L.json 2> gpurun_out/${T}_c2_$L.err || { tail -5 gpurun_out/${T}_c2_$L.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('L', sys.argv[2], 'c2 norst', d['value'], d['ms_per_step'])" gpurun_out/${T}_c2_$L.json $L
done

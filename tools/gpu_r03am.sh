# round-3: self-synchronising JPEG decoding, bits per lane (IK_JPEG_SEQ_L) A/B on the
# restart-free loadtest mix and configs[2]; JPEG tests under the shortest setting first
set -o pipefail
export TMPDIR=/tmp
T=r03am
mkdir -p gpurun_out
IK_JPEG_SEQ_L=2048 timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_jpeg_zune.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for L in 8192 4096 2048; do
  IK_JPEG_SEQ_L=$L timeout -k 10 300 python tools/loadtest.py --requests 1024 --batch 64 --threads 16 > gpurun_out/${T}_lt_$L.json 2> gpurun_out/${T}_lt_$L.err || { tail -5 gpurun_out/${T}_lt_$L.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('L', sys.argv[2], 'loadtest norst', d['value'], d['batch_latency_ms'])" gpurun_out/${T}_lt_$L.json $L
done
for L in 8192 2048; do
  IK_JPEG_SEQ_L=$L timeout -k 10 500 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2_$L.json 2> gpurun_out/${T}_c2_$L.err || { tail -5 gpurun_out/${T}_c2_$L.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('L', sys.argv[2], 'c2 norst', d['value'], d['ms_per_step'])" gpurun_out/${T}_c2_$L.json $L
done

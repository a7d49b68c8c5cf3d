# round-3: configs[2] (256 x 4096^2 JPEG q90 4:2:0 RSTn -> 512^2 Lanczos3 -> JPEG q85):
# restart intervals per wave of the batched entropy decoder (IK_HUFF_LANES) A/B
set -o pipefail
export TMPDIR=/tmp
T=r03x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_jpeg_zune.py tests/test_gpu_transform_batch.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for L in 16 32 64; do
  IK_HUFF_LANES=$L timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_lanes$L.json 2> gpurun_out/${T}_lanes$L.err || { tail -5 gpurun_out/${T}_lanes$L.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/${T}_lanes$L.json
done

# round-3: host JPEG parse -- restart markers found with memchr, restart-free scans
# unstuffed a run at a time, big-endian words four bytes at a time: JPEG GPU tests,
# then configs[2] with and without RSTn
set -o pipefail
export TMPDIR=/tmp
T=r03af
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_decode.py tests/test_gpu_transform_batch.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
show gpurun_out/${T}_c2rst.json
timeout -k 10 500 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2norst.json 2> gpurun_out/${T}_c2norst.err || { tail -5 gpurun_out/${T}_c2norst.err; exit 1; }
show gpurun_out/${T}_c2norst.json

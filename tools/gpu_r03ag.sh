# round-3: JPEG batch upload: tables in one copy from a pinned block, scan bytes DMAed in place or staged by the pool, all async --
# JPEG GPU tests,
# then configs[2] with and without RSTn
set -o pipefail
export TMPDIR=/tmp
T=r03ag
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_decode.py tests/test_gpu_transform_batch.py tests/test_gpu_headline_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
show gpurun_out/${T}_c2rst.json
timeout -k 10 500 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2norst.json 2> gpurun_out/${T}_c2norst.err || { tail -5 gpurun_out/${T}_c2norst.err; exit 1; }
show gpurun_out/${T}_c2norst.json
timeout -k 10 300 python tools/loadtest.py --requests 4096 --batch 64 --threads 16 --restart > gpurun_out/${T}_lt_rst.json 2> gpurun_out/${T}_lt_rst.err || { tail -5 gpurun_out/${T}_lt_rst.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_lt_rst.json').read().strip().splitlines()[-1]); print('loadtest rst', d['value'])"

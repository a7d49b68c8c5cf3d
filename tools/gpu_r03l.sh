# round-3: configs[2] from JPEG bytes (with and without restart markers) and
# configs[4] from PNG bytes, each with rocprof kernel stats; the unfilter A/B
# (IK_PNG_UNF_SWAR) on the headline.  Every GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03l}
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), d.get('png_decode_stages_ms',{}).get('unfilter'))" $1; }
for sw in 1 0; do
  IK_PNG_UNF_SWAR=$sw timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_swar$sw.json 2> gpurun_out/${T}_swar$sw.err || { tail -5 gpurun_out/${T}_swar$sw.err; exit 1; }
  show gpurun_out/${T}_swar$sw.json
done
timeout -k 10 500 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --hbm-batch 64 --jpeg-images 0 --pageable-steps 0 > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
show gpurun_out/${T}_c2rst.json
timeout -k 10 400 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2norst.json 2> gpurun_out/${T}_c2norst.err || { tail -5 gpurun_out/${T}_c2norst.err; exit 1; }
show gpurun_out/${T}_c2norst.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c2prof -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_c2prof.json 2> gpurun_out/${T}_c2prof.err || { echo "C2 PROFILE FAILED"; exit 1; }
echo "c2 profile ok"
timeout -k 10 600 python -u bench.py --size 8192 --out 1024 --filter lanczos3 --format avif --quality 60 --batch 32 --steps 2 --warmup 1 --hbm-batch 16 --hbm-steps 2 --jpeg-images 0 --pageable-steps 0 --cpu-seconds 20 > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { tail -5 gpurun_out/${T}_c4.err; exit 1; }
show gpurun_out/${T}_c4.json

# round-3 final evidence: every GPU test, smoke, the default bench line (cpu_baseline
# included) and rocprofv3 kernel stats of the same command; then configs[2] with RSTn
set -o pipefail
export TMPDIR=/tmp
T=r03ai
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('value', d['value'], d['ms_per_step']); print('pcie', d['pcie_inclusive']['value']); print(d['png_decode_stages_ms']); print('roofline', d['roofline']); print('jpeg leg', d['decode_inclusive_jpeg'].get('value')); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -f csv -- python bench.py --no-cpu-baseline > gpurun_out/${T}_bench_prof.json 2> gpurun_out/${T}_bench_prof.err || { echo "PROFILE FAILED"; tail -5 gpurun_out/${T}_bench_prof.err; exit 1; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
head -5 gpurun_out/${T}_kernel_stats.csv | cut -c1-140
timeout -k 10 400 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 3 --warmup 1 --no-extras > gpurun_out/${T}_c2rst.json 2> gpurun_out/${T}_c2rst.err || { tail -5 gpurun_out/${T}_c2rst.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_c2rst.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], 'cpu', d['cpu_baseline']['value'])"

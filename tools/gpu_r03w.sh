# round-3 evidence + A/B: all GPU tests + smoke, the default bench line (cpu_baseline
# included), rocprof kernel stats of the same bench command, (no A/B)
# kernel's horizontal-tap A/B (IK_HTAPS 2 vs 4) for Triangle and Lanczos3.
# Every GPU step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03w}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('value', d['value'], d['ms_per_step']); print('pcie', d['pcie_inclusive']); print(d['png_decode_stages_ms']); print(d['kernels']); print('resize', d['roofline_resize']); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -f csv -- python bench.py --no-cpu-baseline > gpurun_out/${T}_bench_prof.json 2> gpurun_out/${T}_bench_prof.err || { echo "PROFILE FAILED"; tail -5 gpurun_out/${T}_bench_prof.err; exit 1; }
echo "profile ok"
cp gpurun_out/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv 2>/dev/null || find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
head -12 gpurun_out/${T}_kernel_stats.csv

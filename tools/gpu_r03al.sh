# round-3 last check: every GPU test and smoke on the final code
set -o pipefail
export TMPDIR=/tmp
T=r03al
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-pcie-leg > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('value', d['value'], d['ms_per_step'], 'jpeg leg', d['decode_inclusive_jpeg'].get('value'))"

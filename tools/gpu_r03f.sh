# round-3: GPU suite with the prelaunched block search + 8-byte unfilter; bench (A/B 16-byte unfilter)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r03f_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
for v in unf8 unf16; do
  if [ $v = unf16 ]; then export IK_PNG_UNF16=1; fi
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r03f_bench_$v.json 2> gpurun_out/r03f_bench_$v.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r03f_bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step']); print(d['png_decode_stages_ms'])"
done
exit $rc

# round-3: wave priorities on expand/resolve/unfilter; search after decode vs after
# resolve; slot-map expand vs binary-search expand
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03h_tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
for v in "decode:" "resolve:" "decode:1" ; do
  fa=${v%%:*}; ex=${v##*:}
  tag=r03h_${fa}_${ex:-map}
  IK_FIND_AFTER=$fa IK_PNG_EXPAND=$ex timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/$tag.json 2> gpurun_out/$tag.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step']); print(d['png_decode_stages_ms'])"
done
exit $rc

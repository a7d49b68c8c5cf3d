# round-3: the next batch's block search on a stream with its own hardware queue
# (search_stream) vs the old copy stream; PNG parity tests first; a rocprof trace
# of the new default to check the queues.
set -o pipefail
export TMPDIR=/tmp
T=r03n
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_headline_parity.py tests/test_gpu_alpha.py tests/test_gpu_png16.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
for v in "search:" "copy:" "search:128" "search:64"; do
  st=${v%%:*}; cu=${v##*:}
  tag=${T}_${st}${cu}
  env IK_FIND_STREAM=$st ${cu:+IK_FIND_CUS=$cu} timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { tail -5 gpurun_out/$tag.err; exit 1; }
  show gpurun_out/$tag.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -f csv -- python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo "PROFILE FAILED"; exit 1; }
show gpurun_out/${T}_prof.json
# the unfilter's per-segment clock (dev build with IK_UNF_PROF)
IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_exp/libimagekit_hip_unfprof.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_unfprof.json 2> gpurun_out/${T}_unfprof.err || { tail -5 gpurun_out/${T}_unfprof.err; exit 1; }
grep "unf-prof" gpurun_out/${T}_unfprof.err | tail -3

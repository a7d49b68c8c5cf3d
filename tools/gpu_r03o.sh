# round-3: the unfilter's per-segment clock (IK_UNF_PROF dev build), the unfilter
# word-at-a-time A/B, and SQ counter passes over one headline batch.
set -o pipefail
export TMPDIR=/tmp
T=r03o
mkdir -p gpurun_out
IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_exp/libimagekit_hip_unfprof.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_unfprof.json 2> gpurun_out/${T}_unfprof.err || { tail -5 gpurun_out/${T}_unfprof.err; exit 1; }
grep "unf-prof" gpurun_out/${T}_unfprof.err | tail -3
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['png_decode_stages_ms']; print(sys.argv[1], d['value'], d['ms_per_step'], 'find', s['find'], 'decode', s['decode'], 'expand', s['expand'], 'resolve', s['resolve'], 'unf', s['unfilter'], 'wall', s['kernel_stage_wall'])" $1; }
for sw in 1 0; do
  IK_PNG_UNF_SWAR=$sw timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/${T}_swar$sw.json 2> gpurun_out/${T}_swar$sw.err || { tail -5 gpurun_out/${T}_swar$sw.err; exit 1; }
  show gpurun_out/${T}_swar$sw.json
done
bash tools/gpu_r03m_pmc.sh

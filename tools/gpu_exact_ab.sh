# dev A/B of library variants in the headline pipeline with the exact coder: LIBS="name:path ..."
set -o pipefail
B="--webp-encoder ${ENC:-exact} --no-cpu-baseline --no-extras --no-pcie-leg --pageable-steps 0"
for v in $LIBS; do
  n=${v%%:*}; p=${v#*:}
  if [ -z "$NOALONE" ]; then IK_LIB_PATH=$p timeout -k 10 200 python -u tools/vp8x_timing.py --n 64 --iters 2 > gpurun_out/ab_t_$n.log 2>&1 || exit 1; else echo "{'gpu_exact_ms_per_batch': []}" > gpurun_out/ab_t_$n.log; fi
  IK_LIB_PATH=$p timeout -k 10 300 python -u bench.py $B > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit 1
  python3 -c "import json,ast; t=ast.literal_eval(open('gpurun_out/ab_t_$n.log').read().strip().splitlines()[-1]); d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]); p=d['png_decode_stages_ms']; print('$n ${ENC:-exact} alone', t['gpu_exact_ms_per_batch'], 'pipe', d['value'], d['ms_per_step'], 'kstage', p['kernel_stage_wall'], 'dec', p['decode'], 'exp', p['expand'], 'res', p['resolve'])"
done

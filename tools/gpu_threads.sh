# Dev: pipelined headline at several stated host-thread budgets
mkdir -p gpurun_out
for t in 32 16 24 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --threads $t > gpurun_out/thr_$t.json 2> gpurun_out/thr_$t.err || { tail -5 gpurun_out/thr_$t.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/thr_$t.json'));print($t, d['value'], d['ms_per_step'], d['png_decode_stages_ms']['upload_find'], d['png_decode_stages_ms']['decode_wall_ms'])"
done

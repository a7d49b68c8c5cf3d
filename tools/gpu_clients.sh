# Dev sweep: concurrent ik_transform_batch clients (bench --clients), PNG-in headline
mkdir -p gpurun_out
for c in ${CLIENTS:-1 2 3}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --no-extras --clients $c ${EXTRA:-} \
      > gpurun_out/clients_$c.json 2> gpurun_out/clients_$c.err || { echo "clients=$c failed"; tail -5 gpurun_out/clients_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/clients_$c.json'));print($c, d['value'], d['ms_per_step'], d['png_decode_stages_ms'])"
done

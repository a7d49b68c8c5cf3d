# Dev: staggered batch parts (upload gate only) vs one part, blocking steps
mkdir -p gpurun_out
for cfg in "1 3" "2 upload" "4 upload" "2 3"; do
  set -- $cfg
  if [ "$2" = 3 ]; then unset IK_BATCH_GATE; else export IK_BATCH_GATE=$2; fi
  timeout -k 10 300 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-extras --pipeline 0 --split $1 > gpurun_out/split_$1_$2.json 2> gpurun_out/split_$1_$2.err || { echo "split $cfg failed"; tail -5 gpurun_out/split_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/split_$1_$2.json'));print('$cfg', d['value'], d['ms_per_step'], d['png_decode_stages_ms']['decode_wall_ms'])"
done

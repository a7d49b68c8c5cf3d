#!/bin/bash
# bench headline at several batch splits (IK_BATCH_SPLIT), no extras / CPU leg
mkdir -p gpurun_out
for sp in ${SPLITS:-1 2 4}; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras --split $sp \
      > gpurun_out/split_$sp.json 2> gpurun_out/split_$sp.err || { tail -5 gpurun_out/split_$sp.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/split_$sp.json'));print('split $sp', d['value'], d['ms_per_step'], d['png_decode_stages_ms'])"
done

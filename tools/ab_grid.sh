#!/bin/bash
# A/B of the exact coder's resident grid (a fraction of the widest diagonal) on the headline bench
set -o pipefail
for g in 1.0 0.5 0.33 0.5 1.0 0.25; do
  IK_VP8X_GRID=$g timeout -k 10 300 python3 bench.py --steps 16 --warmup 3 --alt-steps 0 > gpurun_out/abg.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abg.json')); print('grid $g', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done

#!/bin/bash
# A/B of the host wait mode (IK_SYNC=spin vs the default blocking waits) on the
# headline bench and configs[2], alternating, one box: TAG=x bash tools/ab_sync.sh
set -o pipefail
TAG=${TAG:-absync}
mkdir -p gpurun_out
for r in 1 2; do
  for m in block spin; do
    echo "== $m $r $(date +%T)"
    if [ $m = spin ]; then export IK_SYNC=spin; else unset IK_SYNC; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --no-pcie-leg --steps 8 > gpurun_out/${TAG}_${m}${r}.json 2> gpurun_out/${TAG}_${m}${r}.err || { echo FAIL; tail -5 gpurun_out/${TAG}_${m}${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${m}${r}.json'));h=d.get('host_cpu',{});print(d['value'],d['ms_per_step'],h.get('per_rank_cores_busy'),h.get('host_coder_stage',{}).get('core_ms_per_image'),h.get('host_coder_stage',{}).get('cores_busy_per_gpu'))"
  done
done
for m in block spin; do
  echo "== c2 $m $(date +%T)"
  if [ $m = spin ]; then export IK_SYNC=spin; else unset IK_SYNC; fi
  timeout -k 10 600 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 4 --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_c2${m}.json 2> gpurun_out/${TAG}_c2${m}.err || { echo FAIL; tail -5 gpurun_out/${TAG}_c2${m}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c2${m}.json'));print(d['value'],d['ms_per_step'])"
done

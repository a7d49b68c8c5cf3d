set -o pipefail
mkdir -p gpurun_out
for v in base hv1 hv2 hv3; do
  timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib_ab/$v.so 3 256 >> gpurun_out/t6_rab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib_ab/$v.so 4 64 >> gpurun_out/t6_rab.txt 2>&1 || exit 1
done
grep '^{' gpurun_out/t6_rab.txt
C2="--source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 5 --warmup 1 --no-extras --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C2 > gpurun_out/t6_cur.json 2> gpurun_out/t6_cur.err || exit 1
IK_LIB_PATH=rust-image-transform_amd/lib_ab/prio.so timeout -k 10 300 python -u bench.py $C2 > gpurun_out/t6_prio.json 2> gpurun_out/t6_prio.err || exit 1
for f in cur prio; do python tools/bench_summary.py gpurun_out/t6_$f.json | head -1; done

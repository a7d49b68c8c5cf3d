set -o pipefail
mkdir -p gpurun_out
C2="--source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 4 --warmup 1 --no-extras --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C2 > gpurun_out/t4_new.json 2> gpurun_out/t4_new.err || exit 1
IK_LIB_PATH=rust-image-transform_amd/lib_ab/oldbits.so timeout -k 10 300 python -u bench.py $C2 > gpurun_out/t4_old.json 2> gpurun_out/t4_old.err || exit 1
IK_TIMING=1 timeout -k 10 300 python -u bench.py $C2 > gpurun_out/t4_tim.json 2> gpurun_out/t4_tim.err || exit 1
for f in new old tim; do python tools/bench_summary.py gpurun_out/t4_$f.json | head -1; done

set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-extras --steps 8"
timeout -k 10 300 python -u bench.py $B > gpurun_out/t10_cur.json 2> gpurun_out/t10_cur.err || exit 1
IK_TIMING=1 IK_LIB_PATH=rust-image-transform_amd/lib_ab/ch24.so timeout -k 10 300 python -u bench.py $B > gpurun_out/t10_ch24.json 2> gpurun_out/t10_ch24.err || exit 1
IK_TIMING=1 IK_LIB_PATH=rust-image-transform_amd/lib_ab/ch32.so timeout -k 10 300 python -u bench.py $B > gpurun_out/t10_ch32.json 2> gpurun_out/t10_ch32.err || exit 1
for f in cur ch24 ch32; do python tools/bench_summary.py gpurun_out/t10_$f.json | head -2; done

# round-3 dev experiment: the JPEG colour kernel's cost with the generic row-end path
# skipped (wrong pixels; timing only) vs the real kernel, configs[2] kernel stats
set -o pipefail
export TMPDIR=/tmp
T=r03aj
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_transform_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in real noedge; do
  if [ $v = noedge ]; then export IK_LIB_PATH=$PWD/rust-image-transform_amd/lib_exp/libimagekit_hip_noedge.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$v -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || { echo "FAILED $v"; tail -5 gpurun_out/${T}_$v.err; exit 1; }
  f=$(find gpurun_out/${T}_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_jpeg_color|k_jpeg_huff_batch|k_jpeg_idct" $f | cut -c1-150
done

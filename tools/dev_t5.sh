set -o pipefail
mkdir -p gpurun_out
for v in base hv1 hv2 hv3; do
  timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib_ab/$v.so 3 256 >> gpurun_out/t5_rab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/resize_ab.py rust-image-transform_amd/lib_ab/$v.so 4 64 >> gpurun_out/t5_rab.txt 2>&1 || exit 1
done
grep '^{' gpurun_out/t5_rab.txt

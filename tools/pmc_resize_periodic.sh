# PMC HBM traffic of the resize kernel alone (tools/resize_ab.py: 64 RGBA 4096^2 frames ->
# 512^2, 6 Triangle then 6 Lanczos3 launches), FETCH_SIZE / WRITE_SIZE in separate passes,
# FETCH_SIZE calibrated on tools/bw_probe pattern 0 -> gpurun_out/pmc_resize.json (copy to profiles/)
export TMPDIR=/tmp
mkdir -p gpurun_out && cp profiles/pmc_resize.json gpurun_out/pmc_resize.json
export IK_PMC_OUT=gpurun_out/pmc_resize.json IK_PMC_KERNEL=${IK_PMC_KERNEL:-k_resize_periodic}
L=rust-image-transform_amd/lib/libimagekit_hip.so
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rpF -o run -f csv -- python tools/resize_ab.py $L 4 64 > gpurun_out/rpF.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/rpW -o run -f csv -- python tools/resize_ab.py $L 4 64 > gpurun_out/rpW.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rpC -o run -f csv -- python tools/bw_probe.py 0 > gpurun_out/rpC.log 2>&1 && \
python tools/pmc_traffic.py gpurun_out/rpF gpurun_out/rpW gpurun_out/rpC triangle_4096_512_b64 64 4096 512 0 6 && \
python tools/pmc_traffic.py gpurun_out/rpF gpurun_out/rpW gpurun_out/rpC lanczos3_4096_512_b64 64 4096 512 6 6

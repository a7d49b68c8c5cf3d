# PMC HBM traffic of the fused resize kernel at the configs[4] geometry (8192^2 ->
# 1024^2, Lanczos3 main filter + triangle alt, batch 32).  The device kernels do
# not depend on the output format, so bench.py runs with --format jpeg (GPU
# entropy coding) to keep the host stage short.  Same counters and calibration as
# tools/pmc_traffic.sh; separate --pmc passes, each under its own time limit.
export TMPDIR=/tmp
mkdir -p gpurun_out && cp profiles/pmc_resize.json gpurun_out/pmc_resize.json
export IK_PMC_OUT=gpurun_out/pmc_resize.json
B=32
args="bench.py --no-cpu-baseline --no-alt-encoder --warmup 2 --steps 2 --batch $B --size 8192 --out 1024 --filter lanczos3 --format jpeg"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc4F -o run -f csv -- python $args > gpurun_out/pmc4F.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4W -o run -f csv -- python $args > gpurun_out/pmc4W.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc4C -o run -f csv -- python tools/bw_probe.py 0 > gpurun_out/pmc4C.log 2>&1 && \
python tools/pmc_traffic.py gpurun_out/pmc4F gpurun_out/pmc4W gpurun_out/pmc4C lanczos3_8192_1024_b$B $B 8192 1024 0 4 && \
python tools/pmc_traffic.py gpurun_out/pmc4F gpurun_out/pmc4W gpurun_out/pmc4C triangle_8192_1024_b$B $B 8192 1024 4 6

# PMC HBM traffic of the fused resize kernel under bench.py (FETCH_SIZE and WRITE_SIZE
# in separate passes, FETCH_SIZE calibrated on tools/bw_probe pattern 0) ->
# gpurun_out/pmc_resize.json (copy to profiles/) and raw CSVs under gpurun_out/.  bench.py --warmup 2
# --steps 2 launches the main filter (triangle) 4x, then the alt filter (lanczos3) 6x.
export TMPDIR=/tmp
# results land in gpurun_out/ (the only directory that comes back from the GPU box)
mkdir -p gpurun_out && cp profiles/pmc_resize.json gpurun_out/pmc_resize.json
export IK_PMC_OUT=gpurun_out/pmc_resize.json
B=${B:-32}
args="bench.py --no-cpu-baseline --no-alt-encoder --warmup 2 --steps 2 --batch $B"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF -o run -f csv -- python $args > gpurun_out/pmcF.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW -o run -f csv -- python $args > gpurun_out/pmcW.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcC -o run -f csv -- python tools/bw_probe.py 0 > gpurun_out/pmcC.log 2>&1 && \
python tools/pmc_traffic.py gpurun_out/pmcF gpurun_out/pmcW gpurun_out/pmcC triangle_4096_512_b$B $B 4096 512 0 4 && \
python tools/pmc_traffic.py gpurun_out/pmcF gpurun_out/pmcW gpurun_out/pmcC lanczos3_4096_512_b$B $B 4096 512 4 6

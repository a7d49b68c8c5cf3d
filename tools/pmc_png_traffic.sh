# PMC HBM traffic of the PNG decode kernels under bench.py (one 64-frame batch): FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM section), FETCH_SIZE doubled per the guide's
# gfx950 rule and also reported against the tools/bw_probe calibration -> gpurun_out/pmc_png.json
export TMPDIR=/tmp
mkdir -p gpurun_out
args="bench.py --no-cpu-baseline --no-extras --pipeline 0 --warmup 0 --steps 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcPF -o run -f csv -- python $args > gpurun_out/pmcPF.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcPW -o run -f csv -- python $args > gpurun_out/pmcPW.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcPC -o run -f csv -- python tools/bw_probe.py 0 > gpurun_out/pmcPC.log 2>&1 && \
python tools/pmc_png_traffic.py gpurun_out/pmcPF gpurun_out/pmcPW gpurun_out/pmcPC gpurun_out/pmc_png.json

# Instruction mix of the PNG kernels under bench.py (one 64-frame batch): one rocprofv3 --pmc pass of
# SQ counters (at most 8 per pass) -> gpurun_out/pmcI/ ; summary by tools/pmc_insts.py
export TMPDIR=/tmp
mkdir -p gpurun_out
args="bench.py --no-cpu-baseline --no-extras --no-pcie-leg --pipeline 0 --warmup 0 --steps 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmcI -o run -f csv -- python $args > gpurun_out/pmcI.log 2>&1 && \
python tools/pmc_insts.py gpurun_out/pmcI > gpurun_out/pmc_insts.txt

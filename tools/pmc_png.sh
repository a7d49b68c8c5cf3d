# Dev tool: PMC passes over the GPU PNG decode kernels (tools/png_decode_bench.py).
export TMPDIR=/tmp B=${B:-64} R=${R:-2}
T=${T:-P}
run() { tag=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc${T}_$tag -o run -f csv -- python tools/png_decode_bench.py > gpurun_out/pmc${T}_$tag.log 2>&1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc${T}_stats -o run -f csv -- python tools/png_decode_bench.py > gpurun_out/pmc${T}_stats.log 2>&1 && \
run a SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE SQ_WAVES && \
run b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA && \
run c SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_INSTS_SCRATCH_ST && \
run d TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr TD_BUSY_avr
echo done rc=$?

# Dev tool: PMC counter passes over the fused resize kernel (tools/sweep_resize.py).
# One rocprofv3 pass per counter set; the chain stops at the first failure.
export TMPDIR=/tmp FILTERS=${FILTERS:-1} B=${B:-32}
run() { tag=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$tag -o run -f csv -- python tools/sweep_resize.py > gpurun_out/pmc_$tag.log 2>&1; }
run e SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE SQ_WAVES && \
run f SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA && \
run g SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
echo done rc=$?

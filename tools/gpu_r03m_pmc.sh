# round-3: SQ counter passes over one headline batch (all PNG kernels of the step),
# one rocprofv3 pass per counter set, each under its own time limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmcq_$tag -o run -f csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras --no-pcie-leg > gpurun_out/pmcq_$tag.log 2>&1; }
run e SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE SQ_WAVES && \
run f SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA && \
run g SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
rc=$?
echo "pmc rc=$rc"
for k in k_png_decode k_png_expand4 k_png_resolve k_png_unfilter k_png_find; do python tools/pmc_summary.py $k gpurun_out/pmcq_e gpurun_out/pmcq_f gpurun_out/pmcq_g; done > gpurun_out/pmcq_summary.txt 2>&1; cat gpurun_out/pmcq_summary.txt
exit $rc

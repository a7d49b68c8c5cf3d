# Dev tool: PMC counter passes over the exact-mode Lanczos3 fused resize launch
# (64 x 4096^2 RGBA8 -> 512^2, tools/sweep_resize.py), one rocprofv3 pass per set,
# plus a kernel-trace --stats pass.  Outputs under gpurun_out/pmcL_<tag>/.
export TMPDIR=/tmp FILTERS=${FILTERS:-4} B=${B:-64}
TAGP=${TAGP:-L}
run() { tag=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc${TAGP}_$tag -o run -f csv -- python tools/sweep_resize.py > gpurun_out/pmc${TAGP}_$tag.log 2>&1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc${TAGP}_stats -o run -f csv -- python tools/sweep_resize.py > gpurun_out/pmc${TAGP}_stats.log 2>&1 && \
run a SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE SQ_WAVES && \
run b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA && \
run c SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
echo done rc=$?

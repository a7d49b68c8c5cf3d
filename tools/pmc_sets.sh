export TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$tag -o run -f csv -- python tools/sweep_resize.py > gpurun_out/pmc_$tag.log 2>&1 || return 1; timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmcp_$tag -o run -f csv -- python tools/bw_probe.py 0 > gpurun_out/pmcp_$tag.log 2>&1; }
export FILTERS=1 TARGETS=8192 B=16
run c SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES && \
run d TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum
echo done rc=$?

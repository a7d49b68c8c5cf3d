# Dev: HIP API + kernel + copy timeline of a short bench run (no counters)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d gpurun_out/trace -o run -f csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/trace_bench.json 2> gpurun_out/trace_bench.err
rc=$?
ls gpurun_out/trace/*/ 2>/dev/null | head; ls gpurun_out/trace | head
exit $rc

# The one GPU evidence script (run through gpurun from the repo root):
#   TAG=r04a STEPS="tests bench c2" bash tools/gpu_evidence.sh
# Steps (each under its own time limit; the script stops at the first failure):
#   tests     pytest -m gpu (every GPU parity test)
#   smoke     __graft_entry__.smoke()
#   bench     the default bench line (configs[1], the headline `value`)
#   prof      rocprofv3 --kernel-trace --stats of the headline bench command
#   c2        configs[2]: 256 x 4096^2 JPEG (RSTn) -> 512^2 Lanczos3 -> JPEG q85, CPU leg included
#   c2prof    rocprofv3 --kernel-trace --stats of the configs[2] command
#   c2norst   configs[2] with restart-free sources
#   lt        the loadtest mix (configs[3]), restart-free sources, 10,000 requests, CPU leg included
#   ltrst     the same with a restart marker per MCU row
#   jtests    the JPEG GPU parity tests only (decode, zune reconstruction, the configs[2] parity case)
#   ptime     the headline bench with IK_TIMING (host stage marks on stderr)
#   c4        configs[4] (8192^2 PNG -> 1024^2 Lanczos3 -> AVIF q60) under rocprofv3, kernel stats
#   pmc       PMC HBM traffic of the PNG kernels (tools/pmc_png_traffic.sh) -> ${TAG}_pmc_png.json
#   gtest     the GPU tests named in $GTESTS
# Outputs go to gpurun_out/${TAG}_*; copy what is judged into profiles/.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-dev}
STEPS=${STEPS:-"tests bench"}
mkdir -p gpurun_out
O=gpurun_out/${TAG}
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1 \
        || { echo "TESTS FAILED"; tail -40 ${O}_tests.log; exit 1; }
      tail -2 ${O}_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 \
        || { echo "SMOKE FAILED"; tail -20 ${O}_smoke.log; exit 1; }
      tail -2 ${O}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err \
        || { echo "BENCH FAILED"; tail -20 ${O}_bench.err; exit 1; }
      python tools/bench_summary.py ${O}_bench.json ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${O}_prof -o run -f csv -- python bench.py --no-cpu-baseline --no-extras --steps 8 > ${O}_prof.json 2> ${O}_prof.err \
        || { echo "PROFILE FAILED"; tail -20 ${O}_prof.err; exit 1; }
      python tools/bench_summary.py ${O}_prof.json
      find ${O}_prof -name "*kernel_stats.csv" -exec cp {} ${O}_kernel_stats.csv \; ;;
    c2)
      timeout -k 10 900 python -u bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 6 --warmup 1 --no-extras --cpu-seconds 10 > ${O}_c2.json 2> ${O}_c2.err \
        || { echo "C2 FAILED"; tail -20 ${O}_c2.err; exit 1; }
      python tools/bench_summary.py ${O}_c2.json ;;
    c2prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d ${O}_c2prof -o run -f csv -- python bench.py --source jpeg-rst --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 4 --warmup 1 --no-extras --no-cpu-baseline > ${O}_c2prof.json 2> ${O}_c2prof.err \
        || { echo "C2PROF FAILED"; tail -20 ${O}_c2prof.err; exit 1; }
      python tools/bench_summary.py ${O}_c2prof.json
      find ${O}_c2prof -name "*kernel_stats.csv" -exec cp {} ${O}_c2_kernel_stats.csv \; ;;
    c2norst)
      timeout -k 10 900 python -u bench.py --source jpeg --format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 4 --warmup 1 --no-extras --no-cpu-baseline > ${O}_c2norst.json 2> ${O}_c2norst.err \
        || { echo "C2NORST FAILED"; tail -20 ${O}_c2norst.err; exit 1; }
      python tools/bench_summary.py ${O}_c2norst.json ;;
    c4)
      # configs[4]: 32 x 8192^2 RGBA PNG (HBM) -> 1024^2 Lanczos3 -> AVIF q60, under rocprofv3 (kernel stats)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d ${O}_c4prof -o run -f csv -- python bench.py --size 8192 --out 1024 --filter lanczos3 --format avif --quality 60 --batch 32 --steps 3 --warmup 1 --no-extras --no-pcie-leg --cpu-seconds 10 > ${O}_c4.json 2> ${O}_c4.err \
        || { echo "C4 FAILED"; tail -20 ${O}_c4.err; exit 1; }
      python tools/bench_summary.py ${O}_c4.json
      find ${O}_c4prof -name "*kernel_stats.csv" -exec cp {} ${O}_c4_kernel_stats.csv \; ;;
    lt)
      timeout -k 10 900 python -u tools/loadtest.py --requests 10000 --batch 64 --threads 16 --cpu-seconds 15 > ${O}_lt.json 2> ${O}_lt.err \
        || { echo "LOADTEST FAILED"; tail -20 ${O}_lt.err; exit 1; }
      tail -c 600 ${O}_lt.json ;;
    ltrst)
      timeout -k 10 900 python -u tools/loadtest.py --requests 10000 --batch 64 --threads 16 --restart > ${O}_ltrst.json 2> ${O}_ltrst.err \
        || { echo "LOADTEST FAILED"; tail -20 ${O}_ltrst.err; exit 1; }
      tail -c 600 ${O}_ltrst.json ;;
    jtests)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg_zune.py tests/test_gpu_decode.py tests/test_gpu_headline_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_jtests.log 2>&1 \
        || { echo "JPEG TESTS FAILED"; tail -40 ${O}_jtests.log; exit 1; }
      tail -2 ${O}_jtests.log ;;
    ptime)
      IK_TIMING=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-extras --steps 6 > ${O}_ptime.json 2> ${O}_ptime.err \
        || { echo "PTIME FAILED"; tail -20 ${O}_ptime.err; exit 1; }
      python tools/bench_summary.py ${O}_ptime.json ;;
    pmc)
      # PMC HBM traffic of the PNG kernels on this code (FETCH_SIZE / WRITE_SIZE passes, each its own run)
      bash tools/pmc_png_traffic.sh > ${O}_pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 ${O}_pmc.log; exit 1; }
      cp gpurun_out/pmc_png.json ${O}_pmc_png.json
      python -c "import json;d=json.load(open('${O}_pmc_png.json'));print({k:v['hbm_bytes_per_batch'] for k,v in d.items() if isinstance(v,dict)}, d.get('code_sha16'))" ;;
    gtest)
      # the GPU tests named in GTESTS only
      timeout -k 10 600 python -u -m pytest ${GTESTS} -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_gtest.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -40 ${O}_gtest.log; exit 1; }
      tail -2 ${O}_gtest.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"

# round-3: PMC HBM traffic of the PNG decode kernels with this round's code
# (FETCH_SIZE and WRITE_SIZE passes, bw_probe calibration) -> gpurun_out/pmc_png.json
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_png_traffic.sh && python -c "import json; d=json.load(open('gpurun_out/pmc_png.json')); print(json.dumps(d, indent=1)[:3000])"

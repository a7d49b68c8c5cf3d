# Dev: resize kernel A/B over lib_ab/*.so variants (tools/resize_ab.py, RGBA 64 and RGB 256
# frames of 4096^2 -> 512^2), then PMC passes over the base variant's launches.
# usage: bash tools/resize_abl.sh "base nohorz ..." [pmc]
export TMPDIR=/tmp
L=rust-image-transform_amd/lib_ab
for v in $1; do
  timeout -k 10 120 python tools/resize_ab.py $L/$v.so 4 64 || exit 1
  timeout -k 10 120 python tools/resize_ab.py $L/$v.so 3 256 || exit 1
done
if [ "$2" = pmc ]; then
  p() { t=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/rpmc_$t -o run -f csv -- python tools/resize_ab.py $L/base.so 4 64 > gpurun_out/rpmc_$t.log 2>&1 || exit 1; }
  p a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  p b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
  echo pmc done
fi

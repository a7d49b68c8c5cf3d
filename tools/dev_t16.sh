set -o pipefail
mkdir -p gpurun_out
C2="--format jpeg --quality 85 --filter lanczos3 --batch 256 --steps 5 --warmup 1 --no-extras --no-cpu-baseline"
for v in cur w512 w2048; do
  L=""; [ $v != cur ] && L="IK_LIB_PATH=rust-image-transform_amd/lib_ab/$v.so"
  for src in jpeg-rst jpeg; do
    env $L timeout -k 10 300 python -u bench.py --source $src $C2 > gpurun_out/t16_${v}_$src.json 2> gpurun_out/t16_${v}_$src.err || exit 1
    echo "$v $src $(python tools/bench_summary.py gpurun_out/t16_${v}_$src.json | head -1)"
  done
done

# Bench sweep on the GPU box: streaming vs sync, both WebP encoders, batch sizes.
# Every step time-limited; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
    tag=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-alt-encoder --steps 8 "$@" > gpurun_out/sw_$tag.json 2> gpurun_out/sw_$tag.err || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/sw_$tag.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/sw_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['vp8_kernel_ms'], d['host_stage_ms'])"
}
for spec in "$@"; do
    tag=${spec%%:*}; a=${spec#*:}
    run $tag $a || exit 1
done

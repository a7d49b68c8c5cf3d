# round-3: where the restart-free loadtest batch spends its time (IK_JPEG_TIMING
# per-image phase lines of the self-synchronising path)
set -o pipefail
export TMPDIR=/tmp
T=r03ah
mkdir -p gpurun_out
IK_JPEG_TIMING=1 timeout -k 10 300 python tools/loadtest.py --requests 512 --batch 64 --threads 16 > gpurun_out/${T}_lt_norst.json 2> gpurun_out/${T}_lt_norst.err || { tail -5 gpurun_out/${T}_lt_norst.err; exit 1; }
python - <<'P'
import re, statistics
L=open('gpurun_out/r03ah_lt_norst.err').read().splitlines()
seq=[l for l in L if l.startswith('[jpeg seq]')]
img=[l for l in L if l.startswith('[jpeg] ')]
print(len(seq), 'seq lines;', len(img), 'image lines')
for l in seq[:3]+img[:3]: print(l)
def col(lines, key):
    v=[float(m.group(1)) for l in lines for m in [re.search(key+r' ([0-9.]+)', l)] if m]
    return (statistics.mean(v), max(v)) if v else None
print('parse', col(img,'parse'), 'alloc', col(img,'alloc'), 'entropy/upload', col(img,'entropy/upload'), 'reconstruct', col(img,'reconstruct'))
P

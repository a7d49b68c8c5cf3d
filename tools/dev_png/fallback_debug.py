"""Which PNG streams of a set fall back to the host decoder, decoded one at a
time and as a batch (IK_PNG_TIMING=1 prints the GPU path's per-batch line)."""
import ctypes
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "rust-image-transform_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..", "tests")]
import ikutil  # noqa: E402
import test_gpu_png as T  # noqa: E402
from imagekit import _lib, decode_image, decode_image_batch  # noqa: E402

lib = _lib.load()
assert lib.ik_init(0) == 0
lib.ik_set_png_gpu_min(0)


def counters():
    c = (ctypes.c_ulonglong * 2)()
    lib.ik_png_counters(c)
    return c[0], c[1]


shapes = [(300, 2500, 4), (517, 1100, 3), (64, 4100, 1), (1000, 1090, 4), (211, 3333, 2), (90, 2049, 4)]
imgs = [ikutil.synth(w, h, c, seed=50 + k, pattern="N" if k % 2 else "S") for k, (w, h, c) in enumerate(shapes)]
datas = [T.own_png(im, idat_size=65536) for im in imgs]
for k, d in enumerate(datas):
    g0, h0 = counters()
    decode_image(d)
    g1, h1 = counters()
    print(shapes[k], len(d), "gpu", g1 - g0, "host", h1 - h0, flush=True)
g0, h0 = counters()
decode_image_batch(datas)
g1, h1 = counters()
print("batch gpu", g1 - g0, "host", h1 - h0, flush=True)

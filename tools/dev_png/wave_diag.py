"""Dev diagnostic (GPU): decode PNGs through the library with IK_TIMING, print why
a stream fell back to the host decoder, and compare pixels with Pillow."""
import io, os, sys
os.environ.setdefault("IK_TIMING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import ctypes
import numpy as np
from PIL import Image
import ikutil
from imagekit import _lib
from imagekit.transform import decode_image
lib = _lib.load()
assert lib.ik_init(0) == 0
def counters():
    c = (ctypes.c_ulonglong * 2)(); lib.ik_png_counters(c); return c[0], c[1]
for (w, h, c, pat, seed) in [(1024, 1024, 4, "S", 8), (640, 480, 3, "S", 1), (2048, 2048, 4, "S", 3)]:
    img = ikutil.synth(w, h, c, seed=seed, pattern=pat)
    b = io.BytesIO(); Image.fromarray(img, "RGBA" if c == 4 else "RGB").save(b, format="PNG")
    g0, h0 = counters()
    d = decode_image(b.getvalue())
    g1, h1 = counters()
    px = d[0].to_numpy() if hasattr(d[0], "to_numpy") else None
    print(w, h, c, "gpu", g1 - g0, "host", h1 - h0, flush=True)

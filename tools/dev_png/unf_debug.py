"""Unfilter debugging: decode a few PNGs on the GPU and report the first
mismatching rows against the source pixels."""
import io
import os
import sys

import numpy as np
from PIL import Image

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "rust-image-transform_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..", "tests")]
import ikutil  # noqa: E402
from imagekit import _lib, decode_image  # noqa: E402

lib = _lib.load()
assert lib.ik_init(0) == 0
for (w, h, c, pat) in [(640, 480, 4, "S"), (1500, 700, 4, "N"), (1500, 700, 3, "N"), (333, 222, 1, "N"), (4096, 4096, 4, "S")]:
    img = ikutil.synth(w, h, c, seed=3, pattern=pat)
    buf = io.BytesIO()
    Image.fromarray(img if c != 1 else img[..., 0] if img.ndim == 3 else img).save(buf, format="PNG")
    try:
        out, _ = decode_image(buf.getvalue())
        px = out.to_array()
    except Exception as e:  # noqa: BLE001
        print(w, h, c, pat, "ERROR", e, flush=True)
        break
    px = px.reshape(img.shape)
    bad = np.nonzero((px != img).reshape(h, -1).any(axis=1))[0]
    print(w, h, c, pat, "bad rows", len(bad), bad[:10], flush=True)
    if len(bad):
        y = bad[0]
        cols = np.nonzero((px[y] != img[y]).reshape(-1))[0]
        print("  row", y, "first bad byte", cols[:8], flush=True)

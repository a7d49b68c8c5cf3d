"""Where the GPU zune-mode JPEG decode differs from the oracle restatement."""
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
o = ikutil.Oracle()
for (w, h, sub, q) in [(640, 480, 0, 50), (64, 64, 0, 50), (64, 64, 2, 90)]:
    buf = io.BytesIO()
    Image.fromarray(ikutil.synth(w, h, 3, seed=w + q)).save(buf, format="JPEG", quality=q, subsampling=sub)
    b = buf.getvalue()
    got = decode_image(b)[0].to_array().astype(int)
    want = o.jpeg_decode(b, 1).astype(int)
    d = got - want
    bad = np.argwhere(d != 0)
    print((w, h, sub, q), "mismatch", len(bad), "of", d.size, flush=True)
    if len(bad):
        ys, xs = bad[:, 0], bad[:, 1]
        print("  by channel", [int((d[..., c] != 0).sum()) for c in range(3)])
        print("  y%8 hist", np.bincount(ys % 8, minlength=8), "x%8 hist", np.bincount(xs % 8, minlength=8))
        for (y, x, c) in bad[:12]:
            print("  ", y, x, c, "got", got[y, x], "want", want[y, x])
        lj = o.jpeg_decode(b, 0).astype(int)
        print("  got==libjpeg frac", float((got == lj).mean()))

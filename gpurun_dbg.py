import sys, numpy as np
sys.path[:0] = ["tests", "rust-image-transform_amd", "."]
import ikutil
from imagekit import DynamicImage, FilterType, _lib
lib = _lib.load(); lib.ik_init(0)
o = ikutil.Oracle()
for (W, H, nw, nh) in [(300, 7, 5, 300), (300, 7, 5, 299), (100, 7, 5, 300), (300, 300, 5, 5), (7, 300, 300, 5)]:
    for f in range(5):
        for c in (1, 3, 4):
            src = ikutil.synth(W, H, c, seed=W * 7 + H + c, pattern="N")
            got = DynamicImage.from_array(src).resize(nw, nh, FilterType(f)).to_array()
            want = o.resize(src, nw, nh, f)
            bad = np.argwhere(got != want)
            if len(bad):
                rows = sorted(set(bad[:, 0].tolist())); cols = sorted(set(bad[:, 1].tolist()))
                print(W, H, nw, nh, "f", f, "c", c, "nbad", len(bad), "rows", rows[:5], rows[-3:], "cols", cols)
print("done")

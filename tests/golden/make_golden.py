"""Generate tests/golden/resize_golden.npz -- small known-answer vectors for the
resampler (TEST INFRASTRUCTURE).

Inputs: deterministic SplitMix64 images (tests/ikutil.synth).  Expected outputs:
the C oracle (oracle/resize.c, image 0.25.8 imageops::resize restated), each one
cross-checked bit for bit against the independent numpy restatement
(tests/oracle_np.py) before it is written.  No reference code is executed or
copied (the reference is Rust and cannot be built here); these vectors pin the
restatement against regressions and are what the GPU path is compared with.

Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import ikutil  # noqa: E402
import oracle_np  # noqa: E402

CASES = [  # (W, H, nw, nh, C, filter, pattern, seed)
    (64, 48, 17, 13, 4, 4, "N", 0), (64, 48, 17, 13, 3, 1, "N", 1), (97, 61, 32, 20, 4, 4, "S", 2),
    (256, 256, 32, 32, 4, 1, "S", 3), (256, 256, 32, 32, 4, 4, "S", 3), (256, 256, 32, 32, 4, 0, "N", 4),
    (33, 1, 7, 1, 3, 4, "N", 5), (2, 2, 200, 200, 3, 4, "N", 6), (40, 30, 40, 7, 1, 2, "N", 7),
    (50, 50, 51, 49, 2, 3, "N", 8), (800, 600, 400, 300, 3, 4, "S", 9), (160, 90, 64, 36, 4, 1, "S", 10),
]


def main():
    orc = ikutil.Oracle()
    out = {}
    for i, (W, H, nw, nh, C, f, pat, seed) in enumerate(CASES):
        src = ikutil.synth(W, H, C, seed=seed, pattern=pat)
        got = orc.resize(src, nw, nh, f)
        ref = oracle_np.resize(src, nw, nh, f)
        assert np.array_equal(got, ref), f"C oracle and numpy restatement disagree on case {i}"
        out[f"case{i}_meta"] = np.array([W, H, nw, nh, C, f, seed, 0 if pat == "S" else 1], np.int64)
        out[f"case{i}_out"] = got
    np.savez_compressed(os.path.join(HERE, "resize_golden.npz"), **out)
    print(f"wrote {len(CASES)} cases")


if __name__ == "__main__":
    main()

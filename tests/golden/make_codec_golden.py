"""Generate tests/golden/codec_golden.npz -- encoded-byte known answers for the
encode_image branches (TEST INFRASTRUCTURE).

- webp_*: WebPEncodeRGB of this container's system libwebp (1.2.2) through
  ctypes -- the simple-API call webp 0.3.1's Encoder::from_rgb(..).encode(q)
  makes (reference src/transform.rs:131-136).  Labelled a "libwebp-1.2.2 proxy":
  the libwebp vendored by libwebp-sys 0.9.6 cannot be checked offline.
- jpeg_*: the oracle restatement of image 0.25.8's JpegEncoder (oracle/jpeg_enc.c),
  checked to decode in libjpeg-turbo (Pillow) within 30 dB of its input.
Inputs are deterministic SplitMix64 images (tests/ikutil.synth); only outputs and
the input recipe are stored.  No reference code is executed or copied.

Run: python tests/golden/make_codec_golden.py
"""
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.dirname(HERE)]
import ikutil  # noqa: E402

CASES = [  # (name, W, H, pattern, seed, q)
    ("a", 64, 48, "S", 0, 80), ("b", 64, 48, "N", 1, 80), ("c", 37, 23, "S", 2, 10), ("d", 128, 96, "S", 3, 95),
]


def psnr(a, b):
    m = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if m == 0 else 10 * np.log10(255.0 ** 2 / m)


def main():
    from PIL import Image
    orc = ikutil.Oracle()
    out = {}
    for name, W, H, pat, seed, q in CASES:
        rgb = ikutil.synth(W, H, 3, seed=seed, pattern=pat)
        w = orc.webp_encode_rgb(rgb, float(q))
        j = orc.jpeg_encode_rgb(rgb, q)
        assert np.asarray(Image.open(io.BytesIO(w))).shape == (H, W, 3)
        assert psnr(np.asarray(Image.open(io.BytesIO(j)).convert("RGB")), rgb) > (30 if pat == "S" and q >= 80 else 5)
        out[f"{name}_meta"] = np.array([W, H, 0 if pat == "S" else 1, seed, q], np.int64)
        out[f"{name}_webp"] = np.frombuffer(w, np.uint8)
        out[f"{name}_jpeg"] = np.frombuffer(j, np.uint8)
    np.savez_compressed(os.path.join(HERE, "codec_golden.npz"), **out)
    print(f"wrote {len(CASES)} cases")


if __name__ == "__main__":
    main()

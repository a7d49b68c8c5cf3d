"""Encoded-byte known answers (tests/golden/codec_golden.npz, made by
tests/golden/make_codec_golden.py).

CPU: the oracle reproduces them (libwebp 1.2.2 WebPEncodeRGB proxy; the JPEG
restatement).  GPU (marked): encode_image reproduces the same bytes with both WebP
coders (libwebp, and the exact GPU coder)."""
import os

import numpy as np
import pytest

import ikutil

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "codec_golden.npz"))
NAMES = sorted({k.split("_")[0] for k in G.files})


def _case(name):
    W, H, pat, seed, q = (int(x) for x in G[f"{name}_meta"])
    return ikutil.synth(W, H, 3, seed=seed, pattern="S" if pat == 0 else "N"), q


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_codec_golden(oracle, name):
    rgb, q = _case(name)
    assert oracle.webp_encode_rgb(rgb, float(q)) == G[f"{name}_webp"].tobytes()
    assert oracle.jpeg_encode_rgb(rgb, q) == G[f"{name}_jpeg"].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_encoders_reproduce_codec_golden(ik, oracle, name):
    import ctypes
    from imagekit import DynamicImage, ImageFormat, _lib, encode_image
    rgb, q = _case(name)
    d = DynamicImage.from_array(rgb)
    assert encode_image(d, ImageFormat.webp, q) == G[f"{name}_webp"].tobytes()
    assert encode_image(d, ImageFormat.jpeg, q) == G[f"{name}_jpeg"].tobytes()
    prev = ik.ik_get_webp_encoder()
    got = {}
    try:
        for enc in (0, 2):  # libwebp, the exact GPU coder (the default AUTO picks libwebp for one image)
            assert ik.ik_set_webp_encoder(enc) == 0
            got[enc] = encode_image(d, ImageFormat.webp, q)
    finally:
        assert ik.ik_set_webp_encoder(prev) == 0
    assert got[0] == G[f"{name}_webp"].tobytes() and got[2] == G[f"{name}_webp"].tobytes()
    assert ik.ik_set_webp_encoder(1) != 0  # the retired non-exact encoder is refused

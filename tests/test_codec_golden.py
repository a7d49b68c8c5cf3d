"""Encoded-byte known answers (tests/golden/codec_golden.npz, made by
tests/golden/make_codec_golden.py).

CPU: the oracle reproduces them (libwebp 1.2.2 WebPEncodeRGB proxy; the JPEG
restatement; the scalar VP8 restatement).  GPU (marked): encode_image / the GPU
VP8 encoder reproduce the same bytes."""
import os
import sys

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


@pytest.mark.parametrize("name", NAMES)
def test_scalar_vp8_reproduces_golden(oracle, name):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    vp8 = pytest.importorskip("vp8_cpu_check")
    rgb, q = _case(name)
    Y, U, V = oracle.webp_yuv420(rgb)
    assert vp8.encode(Y, U, V, float(q), -1)[0] == G[f"{name}_vp8"].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_encoders_reproduce_codec_golden(ik, oracle, name):
    import ctypes
    from imagekit import DynamicImage, ImageFormat, _lib, encode_image
    rgb, q = _case(name)
    d = DynamicImage.from_array(rgb)
    assert encode_image(d, ImageFormat.webp, q) == G[f"{name}_webp"].tobytes()
    assert encode_image(d, ImageFormat.jpeg, q) == G[f"{name}_jpeg"].tobytes()
    assert ik.ik_set_webp_encoder(1) == 0
    try:
        got = encode_image(d, ImageFormat.webp, q)
    finally:
        assert ik.ik_set_webp_encoder(0) == 0
    assert got == G[f"{name}_vp8"].tobytes()

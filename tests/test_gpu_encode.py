"""GPU parity for encode_image's device front ends (reference src/transform.rs:113-150).

WebP: the device YUV420 planes must equal libwebp 1.2.2's own import (and the
oracle restatement); the WebP bytes must equal WebPEncodeRGB(to_rgb8(img), q)
byte for byte -- i.e. webp 0.3.1 Encoder::from_rgb(..).encode(q) on the same
libwebp.  JPEG: device coefficients and bytes must equal the image 0.25.8
JpegEncoder restatement byte for byte.  AVIF: rav1e (the reference's AV1 encoder)
is absent, the build codes AV1 with libavif/aom: parity unpinned, checked as a
decoded-PSNR bound (Pillow/dav1d), dimensions, alpha handling and q-monotone size."""
import ctypes
import io

import numpy as np
import pytest

import ikutil
from imagekit import DynamicImage, ImageFormat, encode_image

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (2, 3), (7, 5), (64, 48), (65, 49), (100, 100), (320, 240), (511, 257), (512, 512)]


def _dev_yuv(ik, img: np.ndarray):
    h, w, c = img.shape
    d = DynamicImage.from_array(img)
    uw, uh = (w + 1) // 2, (h + 1) // 2
    n = w * h + 2 * uw * uh
    dy = ctypes.c_void_p()
    assert ik.ik_dev_alloc(n, ctypes.byref(dy)) == 0
    try:
        # the image handle's device pointer/pitch are private: go through a fresh upload
        from imagekit import _lib
        pitch = ((w * c + 255) // 256) * 256
        ds = ctypes.c_void_p()
        assert ik.ik_dev_alloc(pitch * h + 16, ctypes.byref(ds)) == 0
        buf = np.zeros((h, pitch), np.uint8)
        buf[:, :w * c] = img.reshape(h, w * c)
        assert ik.ik_memcpy_h2d(ds, buf.ctypes.data, buf.nbytes) == 0
        assert ik.ik_webp_yuv420_device(ds, w, h, c, pitch, dy, None) == 0, _lib.last_error()
        assert ik.ik_dev_synchronize() == 0
        out = np.zeros(n, np.uint8)
        assert ik.ik_memcpy_d2h(out.ctypes.data, dy, n) == 0
        ik.ik_dev_free(ds)
    finally:
        ik.ik_dev_free(dy)
    del d
    return out[:w * h].reshape(h, w), out[w * h:w * h + uw * uh].reshape(uh, uw), \
        out[w * h + uw * uh:].reshape(uh, uw)


@pytest.mark.parametrize("wh", SIZES)
@pytest.mark.parametrize("c", [1, 3, 4])
def test_webp_yuv420_planes(ik, oracle, wh, c):
    w, h = wh
    img = ikutil.synth(w, h, c, seed=w + h, pattern="N")
    rgb = oracle.to_rgb8(img)
    gy, gu, gv = _dev_yuv(ik, img)
    ly, lu, lv = oracle.libwebp_import_yuv(rgb)
    np.testing.assert_array_equal(gy, ly)
    np.testing.assert_array_equal(gu, lu)
    np.testing.assert_array_equal(gv, lv)


@pytest.mark.parametrize("wh", [(1, 1), (7, 5), (64, 48), (320, 240), (512, 512)])
@pytest.mark.parametrize("q", [1, 10, 75, 80, 100])
def test_webp_bytes_match_libwebp(ik, oracle, wh, q):
    w, h = wh
    img = ikutil.synth(w, h, 4, seed=q, pattern="S")
    got = encode_image(DynamicImage.from_array(img), ImageFormat.webp, q)
    assert got == oracle.webp_encode_rgb(oracle.to_rgb8(img), float(q))


@pytest.mark.parametrize("wh", SIZES)
@pytest.mark.parametrize("q", [1, 10, 50, 85, 100])
def test_jpeg_bytes_match_oracle(ik, oracle, wh, q):
    w, h = wh
    img = ikutil.synth(w, h, 3, seed=q + w, pattern="S")
    got = encode_image(DynamicImage.from_array(img), ImageFormat.jpeg, q)
    assert got == oracle.jpeg_encode_rgb(img, q)


@pytest.mark.parametrize("c", [1, 2, 4])
def test_jpeg_to_rgb8_channels(ik, oracle, c):
    img = ikutil.synth(37, 23, c, seed=c, pattern="N")
    got = encode_image(DynamicImage.from_array(img), ImageFormat.jpeg, 85)
    assert got == oracle.jpeg_encode_rgb(oracle.to_rgb8(img), 85)


def test_quality_clamp(ik, oracle):
    img = ikutil.synth(40, 30, 3, seed=1)
    d = DynamicImage.from_array(img)
    assert encode_image(d, ImageFormat.jpeg, 0) == oracle.jpeg_encode_rgb(img, 1)
    assert encode_image(d, ImageFormat.jpeg, 101) == oracle.jpeg_encode_rgb(img, 100)
    assert encode_image(d, ImageFormat.webp, 0) == oracle.webp_encode_rgb(img, 1.0)


# ---- AVIF (image AvifEncoder -> ravif/rav1e in the reference; libavif/aom here) ----
def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


@pytest.mark.parametrize("wh", [(1, 1), (17, 9), (320, 240), (512, 512)])
def test_avif_encode_decodes_close_to_source(ik, wh):
    from PIL import Image
    w, h = wh
    src = ikutil.synth(w, h, 4, seed=w + h, pattern="S")
    b = encode_image(DynamicImage.from_array(src), ImageFormat.avif, 80)
    assert b[4:12] == b"ftypavif"
    im = Image.open(io.BytesIO(b))
    assert im.size == (w, h) and im.mode == "RGB"  # opaque source: no alpha plane
    if w * h >= 64:
        assert _psnr(np.asarray(im), src[..., :3]) > 30.0


def test_avif_alpha_and_gray(ik):
    from PIL import Image
    src = ikutil.synth(96, 64, 4, seed=3, pattern="S").copy()
    src[..., 3] = np.linspace(0, 255, 96, dtype=np.uint8)[None, :]
    im = Image.open(io.BytesIO(encode_image(DynamicImage.from_array(src), ImageFormat.avif, 90)))
    assert im.mode == "RGBA"
    a = np.asarray(im)
    assert np.abs(a[..., 3].astype(int) - src[..., 3]).max() <= 8
    g = ikutil.synth(40, 30, 1, seed=4, pattern="S")
    im = Image.open(io.BytesIO(encode_image(DynamicImage.from_array(g), ImageFormat.avif, 90)))
    rgb = np.asarray(im.convert("RGB")).astype(int)
    assert np.abs(rgb - g.repeat(3, axis=2)).mean() < 3.0


def test_avif_quality_orders_size(ik):
    img = DynamicImage.from_array(ikutil.synth(256, 256, 3, seed=9, pattern="N"))
    assert len(encode_image(img, ImageFormat.avif, 10)) < len(encode_image(img, ImageFormat.avif, 95))

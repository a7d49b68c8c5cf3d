"""CPU: pin the oracle (TEST INFRASTRUCTURE) before trusting it.

- C oracle (oracle/resize.c) == independent numpy restatement (tests/oracle_np.py),
  bit for bit, every filter / channel count / geometry class.
- Output geometry == the reference's own known answers (tests/transform.rs).
- WebP colour conversion restatement == libwebp 1.2.2's own WebPPictureImportRGB.
- WebP bytes == WebPEncodeRGB (the call webp 0.3.1 makes, src/transform.rs:134-136).
- JPEG restatement: decodable, JFIF/SOI/EOI framing, quality monotone as the
  reference tests require (tests/transform.rs:175-186, :275-287).
- Golden vectors in tests/golden/ reproduce.
"""
import io
import os

import numpy as np
import pytest

import ikutil
import oracle_np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resize_golden.npz")


@pytest.mark.parametrize("geom", [((64, 48), (17, 13)), ((97, 61), (32, 20)), ((33, 1), (7, 1)),
                                  ((2, 2), (20, 20)), ((40, 30), (40, 7)), ((50, 50), (51, 49)),
                                  ((9, 200), (3, 25)), ((1, 1), (4, 4))])
@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("f", range(5))
def test_c_oracle_matches_numpy_restatement(oracle, geom, c, f):
    (W, H), (nw, nh) = geom
    src = ikutil.synth(W, H, c, seed=W + H + c + f, pattern="N")
    np.testing.assert_array_equal(oracle.resize(src, nw, nh, f), oracle_np.resize(src, nw, nh, f))


# tests/transform.rs dimension known-answers (:10-96, :224-269)
KATS = [((800, 600), (400, None), (400, 300)), ((800, 600), (None, 300), (400, 300)),
        ((800, 600), (400, 300), (400, 300)), ((1920, 1080), (960, None), (960, 540)),
        ((800, 600), (None, None), (800, 600)), ((100, 100), (200, 200), (200, 200)),
        ((800, 600), (1, 1), (1, 1)), ((2, 2), (200, 200), (200, 200)),
        ((1920, 1080), (640, 480), (640, 360)), ((1000, 1000), (100, 100), (100, 100))]


@pytest.mark.parametrize("src,wh,want", KATS)
def test_reference_dimension_kats(oracle, src, wh, want):
    assert oracle.resize_image_dims(*src, *wh) == want
    assert oracle_np.resize_image_dims(*src, *wh) == want


def test_resize_of_constant_image_is_constant(oracle):
    src = np.full((48, 64, 4), 200, np.uint8)
    for f in range(5):
        assert (oracle.resize(src, 17, 13, f) == 200).all()


def test_golden_vectors(oracle):
    g = np.load(GOLDEN)
    n = len([k for k in g.files if k.endswith("_meta")])
    assert n >= 10
    for i in range(n):
        W, H, nw, nh, C, f, seed, pat = (int(x) for x in g[f"case{i}_meta"])
        src = ikutil.synth(W, H, C, seed=seed, pattern="N" if pat else "S")
        np.testing.assert_array_equal(oracle.resize(src, nw, nh, f), g[f"case{i}_out"])


@pytest.mark.parametrize("wh", [(1, 1), (2, 3), (7, 5), (64, 48), (65, 49), (320, 240)])
def test_webp_yuv_restatement_matches_libwebp(oracle, wh):
    w, h = wh
    rgb = ikutil.synth(w, h, 3, seed=w * h, pattern="N")
    for a, b in zip(oracle.webp_yuv420(rgb), oracle.libwebp_import_yuv(rgb)):
        np.testing.assert_array_equal(a, b)


def test_webp_encode_is_webpencodergb(oracle):
    rgb = ikutil.synth(50, 50, 3, seed=1)
    b = oracle.webp_encode_rgb(rgb, 80.0)
    assert b[:4] == b"RIFF" and b[8:12] == b"WEBP"


def test_jpeg_restatement_framing_and_decodability(oracle):
    from PIL import Image
    rgb = ikutil.synth(100, 75, 3, seed=2)
    b = oracle.jpeg_encode_rgb(rgb, 80)
    assert b[:2] == b"\xff\xd8" and b[-2:] == b"\xff\xd9"
    assert b[2:4] == b"\xff\xe0" and b[6:11] == b"JFIF\x00"
    im = np.asarray(Image.open(io.BytesIO(b)).convert("RGB")).astype(float)
    psnr = 10 * np.log10(255 ** 2 / ((im - rgb) ** 2).mean())
    assert psnr > 30


def test_jpeg_quality_monotone_like_reference(oracle):
    z = np.zeros((500, 500, 3), np.uint8)  # DynamicImage::new_rgb8(500, 500)
    assert len(oracle.jpeg_encode_rgb(z, 95)) > len(oracle.jpeg_encode_rgb(z, 10))
    big = np.zeros((1000, 1000, 3), np.uint8)
    assert len(oracle.jpeg_encode_rgb(big[:100, :100], 80)) < len(oracle.jpeg_encode_rgb(big, 80))


def test_transform_cpu_path(oracle):
    img = ikutil.synth(640, 480, 3, seed=0)
    b, dims = oracle.transform(img, 320, None, 4, 1, 80)  # config 1 shape: w=320, webp q80
    assert dims == (320, 240) and b[:4] == b"RIFF"

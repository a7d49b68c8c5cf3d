"""GPU parity with translucent alpha.

image 0.25.8's resize (reference src/transform.rs:85-89) resamples every channel
of Rgba8 / LumaA8 independently: it does NOT premultiply by alpha, so colour
under alpha = 0 bleeds into neighbours exactly as the weights say.  The device
resampler restates that ("alpha"): these tests hold it bit-exact
against the oracle with random and hard-edged alpha, for C = 2 and C = 4, every
filter, and through the pipeline: JPEG / WebP drop alpha in to_rgb8
(src/transform.rs:123-137), AVIF keeps it (to_rgba8, :140-145; parity with rav1e
unpinned, the decoded alpha is checked against the resized alpha)."""
import ctypes
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

import ikutil
from imagekit import DynamicImage, FilterType, ImageFormat, _lib, decode_image, encode_image

pytestmark = pytest.mark.gpu

FILTERS = [FilterType.Nearest, FilterType.Triangle, FilterType.CatmullRom, FilterType.Gaussian,
           FilterType.Lanczos3]
GEOMS = [((97, 61), (32, 20)), ((64, 48), (129, 97)), ((333, 200), (100, 61)), ((1024, 768), (256, 192))]


@pytest.mark.parametrize("alpha", ["random", "edge"])
@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: f"{g[0][0]}x{g[0][1]}-{g[1][0]}x{g[1][1]}")
@pytest.mark.parametrize("c", [2, 4])
@pytest.mark.parametrize("f", FILTERS, ids=lambda f: f.name)
def test_resize_translucent_matches_oracle(ik, oracle, f, c, geom, alpha):
    (W, H), (nw, nh) = geom
    src = ikutil.synth(W, H, c, seed=W + c, pattern="N" if alpha == "random" else "S", alpha=alpha)
    assert src[..., -1].min() < 255
    got = DynamicImage.from_array(src).resize(nw, nh, f).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, nw, nh, int(f)))


def test_no_premultiply_colour_bleeds_from_transparent_pixels(ik, oracle):
    """The stated assumption, visibly: red under alpha 0 on the left, blue opaque on
    the right; after a Triangle downscale the seam's colour mixes red in (a
    premultiplying resampler would give pure blue there)."""
    src = np.zeros((8, 16, 4), np.uint8)
    src[:, :8] = (255, 0, 0, 0)
    src[:, 8:] = (0, 0, 255, 255)
    got = DynamicImage.from_array(src).resize(4, 2, FilterType.Triangle).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, 4, 2, int(FilterType.Triangle)))
    seam = got[0, 2]
    assert seam[0] > 0 and 0 < seam[3] < 255


def _pipeline(ik, imgs, nw, nh, filt, fmt, q):
    H, W, C = imgs[0].shape
    n = len(imgs)
    pitch = (W * C + 255) // 256 * 256
    src = np.zeros((n, H, pitch), np.uint8)
    for i, im in enumerate(imgs):
        src[i, :, :W * C] = im.reshape(H, W * C)
    d = ctypes.c_void_p()
    assert ik.ik_dev_alloc(src.nbytes, ctypes.byref(d)) == 0
    p = ctypes.c_void_p()
    try:
        assert ik.ik_memcpy_h2d(d, src.ctypes.data, src.nbytes) == 0
        assert ik.ik_pipeline_create(W, H, C, nw, nh, filt, fmt, q, n, 2, ctypes.byref(p)) == 0, _lib.last_error()
        cap = n * (nw * nh * 4 + 65536)
        out = np.zeros(cap, np.uint8)
        sizes = (ctypes.c_size_t * n)()
        assert ik.ik_pipeline_run(p, d, pitch, H * pitch, n, out.ctypes.data, cap, sizes) == 0, _lib.last_error()
    finally:
        if p:
            ik.ik_pipeline_destroy(p)
        ik.ik_dev_free(d)
    res, off = [], 0
    for i in range(n):
        res.append(bytes(out[off:off + sizes[i]]))
        off += sizes[i]
    return res


@pytest.mark.parametrize("c", [2, 4])
@pytest.mark.parametrize("fmt", [0, 1], ids=["jpeg", "webp"])
def test_pipeline_translucent_drops_alpha_like_to_rgb8(ik, oracle, c, fmt):
    imgs = [ikutil.synth(301, 203, c, seed=40 + s, pattern="N", alpha="random") for s in range(3)]
    got = _pipeline(ik, imgs, 97, 61, 4, fmt, 80)
    for im, b in zip(imgs, got):
        rgb = oracle.to_rgb8(oracle.resize(im, 97, 61, 4))
        want = oracle.jpeg_encode_rgb(rgb, 80) if fmt == 0 else oracle.webp_encode_rgb(rgb, 80.0)
        assert b == want


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


@pytest.mark.parametrize("c", [2, 4])
def test_avif_translucent_alpha_plane(ik, oracle, c):
    """AVIF keeps alpha: the pipeline's bytes equal encode_image of the oracle-resized
    pixels, and the decoded alpha plane is close to the resized alpha."""
    imgs = [ikutil.synth(200, 150, c, seed=60 + s, pattern="S", alpha="edge" if s else "random") for s in range(2)]
    got = _pipeline(ik, imgs, 100, 75, 4, 2, 80)
    for im, b in zip(imgs, got):
        ref = oracle.resize(im, 100, 75, 4)
        assert b[4:12] == b"ftypavif"
        assert b == encode_image(DynamicImage.from_array(ref), ImageFormat.avif, 80)
        dec = np.asarray(Image.open(io.BytesIO(b)).convert("RGBA"))
        assert dec.shape == (75, 100, 4)
        assert _psnr(dec[..., 3], ref[..., -1]) > 30


def _png(img):
    b = io.BytesIO()
    Image.fromarray(img, "LA" if img.shape[2] == 2 else "RGBA").save(b, format="PNG")
    return b.getvalue()


@pytest.mark.parametrize("c", [2, 4])
def test_gpu_png_decode_translucent(ik, c):
    """Random alpha through the GPU PNG decoder: bit-exact, and decoded on the GPU."""
    img = ikutil.synth(777, 333, c, seed=5, pattern="N", alpha="random")
    cnt0 = (ctypes.c_ulonglong * 2)()
    cnt1 = (ctypes.c_ulonglong * 2)()
    assert ik.ik_set_png_gpu_min(0) == 0
    try:
        ik.ik_png_counters(cnt0)
        dec, fmt = decode_image(_png(img))
        ik.ik_png_counters(cnt1)
    finally:
        ik.ik_set_png_gpu_min(256 << 10)
    np.testing.assert_array_equal(dec.to_array(), img)
    assert cnt1[0] == cnt0[0] + 1 and cnt1[1] == cnt0[1]


@pytest.mark.parametrize("c", [2, 4])
def test_transform_from_translucent_png(ik, oracle, c):
    """decode (GPU PNG) -> resize Lanczos3 -> WebP: bytes equal the oracle's
    transform of the same pixels (alpha dropped by to_rgb8 after resizing)."""
    from imagekit.transform import transform
    img = ikutil.synth(640, 480, c, seed=6, pattern="S", alpha="random")
    assert ik.ik_set_png_gpu_min(0) == 0
    try:
        got = transform(_png(img), 160, 120, ImageFormat.webp, 75, filter=4)
    finally:
        ik.ik_set_png_gpu_min(256 << 10)
    want, dims = oracle.transform(img, 160, 120, 4, 1, 75)
    assert dims == (160, 120) and got == want

"""GPU parity: the gfx950 resampler vs the CPU oracle (image 0.25.8 imageops::resize
as used by reference src/transform.rs:85-89).  Bar: bit-exact for every filter
(the device uses the reference's f32 op order, no FMA, host-computed weights)."""
import ctypes

import numpy as np
import pytest

import ikutil
from imagekit import DynamicImage, FilterType, resize_image

pytestmark = pytest.mark.gpu

FILTERS = [FilterType.Nearest, FilterType.Triangle, FilterType.CatmullRom, FilterType.Gaussian,
           FilterType.Lanczos3]

SMALL = [((64, 48), (17, 13)), ((97, 61), (32, 20)), ((256, 256), (32, 32)), ((33, 1), (7, 1)),
         ((2, 2), (200, 200)), ((40, 30), (40, 7)), ((50, 50), (51, 49)), ((1, 1), (3, 5)),
         ((300, 7), (5, 300)), ((129, 257), (64, 128))]


@pytest.mark.parametrize("geom", SMALL, ids=lambda g: f"{g[0][0]}x{g[0][1]}-{g[1][0]}x{g[1][1]}")
@pytest.mark.parametrize("c", [1, 2, 3, 4])
@pytest.mark.parametrize("f", FILTERS, ids=lambda f: f.name)
def test_resize_exact_small(ik, oracle, geom, c, f):
    (W, H), (nw, nh) = geom
    src = ikutil.synth(W, H, c, seed=W * 7 + H + c, pattern="N")
    got = DynamicImage.from_array(src).resize(nw, nh, f).to_array()
    want = oracle.resize(src, nw, nh, int(f))
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("geom,c,f", [
    (((800, 600), (400, 300)), 3, FilterType.Lanczos3),
    (((1920, 1080), (640, 360)), 3, FilterType.Lanczos3),
    (((1000, 1000), (100, 100)), 4, FilterType.Triangle),
    (((2000, 2000), (431, 431)), 3, FilterType.Lanczos3),
    (((640, 480), (320, 240)), 3, FilterType.Lanczos3),
    (((1024, 768), (1023, 767)), 4, FilterType.Lanczos3),
    (((333, 222), (1000, 666)), 3, FilterType.Lanczos3),
    (((123, 45), (1230, 450)), 4, FilterType.Triangle),
    (((800, 600), (1, 1)), 3, FilterType.Lanczos3),
    (((5000, 8), (3, 2)), 4, FilterType.Lanczos3),
])
def test_resize_exact_medium(ik, oracle, geom, c, f):
    (W, H), (nw, nh) = geom
    src = ikutil.synth(W, H, c, seed=3, pattern="S")
    got = DynamicImage.from_array(src).resize(nw, nh, f).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, nw, nh, int(f)))


@pytest.mark.parametrize("f", [FilterType.Triangle, FilterType.Lanczos3, FilterType.Nearest])
def test_resize_full_size_4096_rgba(ik, oracle, f):
    """BASELINE configs[1]/[2] geometry: 4096^2 RGBA8 -> 512^2, bit-exact."""
    src = ikutil.synth(4096, 4096, 4, seed=11, pattern="S")
    got = DynamicImage.from_array(src).resize(512, 512, f).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, 512, 512, int(f)))


def test_resize_batch_device(ik, oracle):
    """Batched launch over device-resident images (the pipeline's resize)."""
    W, H, C, n, nw, nh = 1000, 700, 4, 3, 125, 88
    imgs = [ikutil.synth(W, H, C, seed=s, pattern="N" if s % 2 else "S") for s in range(n)]
    pitch, opitch = 4096, 512
    src = np.zeros((n, H, pitch), np.uint8)
    for i, im in enumerate(imgs):
        src[i, :, :W * C] = im.reshape(H, W * C)
    d_src, d_dst = ctypes.c_void_p(), ctypes.c_void_p()
    assert ik.ik_dev_alloc(src.nbytes, ctypes.byref(d_src)) == 0
    assert ik.ik_dev_alloc(n * nh * opitch, ctypes.byref(d_dst)) == 0
    try:
        assert ik.ik_memcpy_h2d(d_src, src.ctypes.data, src.nbytes) == 0
        assert ik.ik_resize_batch_device(d_src, W, H, C, pitch, H * pitch, n, nw, nh,
                                         int(FilterType.Lanczos3), d_dst, opitch, nh * opitch,
                                         None) == 0
        assert ik.ik_dev_synchronize() == 0
        out = np.zeros((n, nh, opitch), np.uint8)
        assert ik.ik_memcpy_d2h(out.ctypes.data, d_dst, out.nbytes) == 0
    finally:
        ik.ik_dev_free(d_src)
        ik.ik_dev_free(d_dst)
    for i, im in enumerate(imgs):
        want = oracle.resize(im, nw, nh, LANCZOS3)
        np.testing.assert_array_equal(out[i, :, :nw * C].reshape(nh, nw, C), want)


LANCZOS3 = int(FilterType.Lanczos3)


@pytest.mark.parametrize("wh", [(400, None), (None, 300), (400, 300), (640, 480), (None, None),
                                (1, 1), (0, None), (200, 200), (800, 10000)])
def test_resize_image_dims_and_pixels(ik, oracle, wh):
    """resize_image (src/transform.rs:62-90): target dims + aspect fit + pixels."""
    w, h = wh
    src = ikutil.synth(800, 600, 3, seed=5)
    img = DynamicImage.from_array(src)
    out = resize_image(img, w, h)
    ow, oh = oracle.resize_image_dims(800, 600, w, h)
    assert out.dimensions() == (ow, oh)
    want = src if (ow, oh) == (800, 600) else oracle.resize(src, ow, oh, LANCZOS3)
    np.testing.assert_array_equal(out.to_array(), want)


# Integer vertical ratios take the periodic kernel (k_resize_periodic: A rotating
# accumulators, zero-weight taps outside each output's window); the rest of the
# geometries above keep k_resize_fused.  Both must be bit-exact.
PERIODIC = [((2048, 1024), (256, 128)), ((1024, 1024), (256, 256)), ((640, 480), (160, 120)),
            ((96, 64), (48, 32)), ((512, 4096), (64, 512)), ((3000, 2000), (375, 250)),
            ((37, 64), (37, 8)), ((4096, 256), (512, 32)), ((300, 900), (7, 450)), ((64, 2048), (64, 256)),
            ((8, 8), (4, 4)), ((3, 16), (3, 2)), ((5, 12), (5, 3)), ((10, 6), (5, 3)), ((7, 64), (9, 16))]


@pytest.mark.parametrize("geom", PERIODIC, ids=lambda g: f"{g[0][0]}x{g[0][1]}-{g[1][0]}x{g[1][1]}")
@pytest.mark.parametrize("c", [1, 3, 4])
@pytest.mark.parametrize("f", FILTERS, ids=lambda f: f.name)
def test_resize_exact_periodic(ik, oracle, geom, c, f):
    (W, H), (nw, nh) = geom
    src = ikutil.synth(W, H, c, seed=W + 3 * H + c, pattern="N" if (W + c) % 2 else "S")
    got = DynamicImage.from_array(src).resize(nw, nh, f).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, nw, nh, int(f)))


@pytest.mark.parametrize("periodic", ["1", "0"])
def test_resize_batch_device_periodic(ik, oracle, monkeypatch, periodic):
    """A batched launch at an 8x vertical ratio, on the periodic kernel and with it
    switched off (IK_RESIZE_PERIODIC=0): both bit-exact."""
    monkeypatch.setenv("IK_RESIZE_PERIODIC", periodic)
    W, H, C, n, nw, nh = 1000, 704, 4, 3, 125, 88
    imgs = [ikutil.synth(W, H, C, seed=20 + s, pattern="N" if s % 2 else "S") for s in range(n)]
    pitch, opitch = 4096, 512
    src = np.zeros((n, H, pitch), np.uint8)
    for i, im in enumerate(imgs):
        src[i, :, :W * C] = im.reshape(H, W * C)
    d_src, d_dst = ctypes.c_void_p(), ctypes.c_void_p()
    assert ik.ik_dev_alloc(src.nbytes, ctypes.byref(d_src)) == 0
    assert ik.ik_dev_alloc(n * nh * opitch, ctypes.byref(d_dst)) == 0
    try:
        assert ik.ik_memcpy_h2d(d_src, src.ctypes.data, src.nbytes) == 0
        for f in (FilterType.Lanczos3, FilterType.Triangle, FilterType.CatmullRom):
            assert ik.ik_resize_batch_device(d_src, W, H, C, pitch, H * pitch, n, nw, nh, int(f), d_dst, opitch,
                                             nh * opitch, None) == 0
            assert ik.ik_dev_synchronize() == 0
            out = np.zeros((n, nh, opitch), np.uint8)
            assert ik.ik_memcpy_d2h(out.ctypes.data, d_dst, out.nbytes) == 0
            for i, im in enumerate(imgs):
                np.testing.assert_array_equal(out[i, :, :nw * C].reshape(nh, nw, C), oracle.resize(im, nw, nh, int(f)))
    finally:
        ik.ik_dev_free(d_src)
        ik.ik_dev_free(d_dst)


def test_resize_kernel_name(ik, monkeypatch):
    """ik_resize_kernel_name reports the kernel launch_resize picks."""
    name = lambda *g: ik.ik_resize_kernel_name(*g).decode()  # noqa: E731
    assert name(4096, 4096, 4, 512, 512, LANCZOS3) == "k_resize_periodic"
    assert name(4096, 4096, 3, 512, 512, int(FilterType.Triangle)) == "k_resize_periodic"
    assert name(2000, 2000, 3, 431, 431, LANCZOS3) == "k_resize_fused"
    assert name(4096, 4096, 4, 512, 512, int(FilterType.Nearest)) == "k_resize_fused"
    monkeypatch.setenv("IK_RESIZE_PERIODIC", "0")
    assert name(4096, 4096, 4, 512, 512, LANCZOS3) == "k_resize_fused"
    assert ik.ik_resize_kernel_name(0, 1, 4, 1, 1, 1) is None

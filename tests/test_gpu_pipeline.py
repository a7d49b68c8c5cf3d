"""GPU: the batched pipeline (ik_pipeline_*) end to end against the oracle -- the
/img handler's decode -> resize_image -> encode_image chain (reference
src/lib.rs:175-191, src/transform.rs:62-150) over device-resident frames.

Bars: JPEG bytes == the oracle's restatement of image 0.25.8's JpegEncoder on
the oracle-resized pixels (the pipeline codes them with k_jpeg_huff_enc on the
GPU); WebP bytes == libwebp WebPEncodeRGB on the oracle-resized pixels (default
encoder).  Includes a configs[2]-shaped case: 4096^2 -> 512^2 Lanczos3, JPEG q85."""
import ctypes

import numpy as np
import pytest

import ikutil
from imagekit import _lib

pytestmark = pytest.mark.gpu
IK_JPEG, IK_WEBP = 0, 1


def _run(ik, imgs, nw, nh, filt, fmt, q, threads=3):
    H, W, C = imgs[0].shape
    n = len(imgs)
    pitch = (W * C + 255) // 256 * 256  # the pipeline wants 8-byte aligned rows; pad like a pitched allocation
    src = np.zeros((n, H, pitch), np.uint8)
    for i, im in enumerate(imgs):
        src[i, :, :W * C] = im.reshape(H, W * C)
    d = ctypes.c_void_p()
    assert ik.ik_dev_alloc(src.nbytes, ctypes.byref(d)) == 0
    p = ctypes.c_void_p()
    try:
        assert ik.ik_memcpy_h2d(d, src.ctypes.data, src.nbytes) == 0
        assert ik.ik_pipeline_create(W, H, C, nw, nh, filt, fmt, q, n, threads, ctypes.byref(p)) == 0, _lib.last_error()
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


@pytest.mark.parametrize("c", [3, 4])
@pytest.mark.parametrize("filt", [1, 4])
@pytest.mark.parametrize("q", [10, 85, 100])
def test_pipeline_jpeg_bytes_match_oracle(ik, oracle, c, filt, q):
    imgs = [ikutil.synth(301, 203, c, seed=s + q, pattern="S" if s % 2 else "N") for s in range(3)]
    got = _run(ik, imgs, 97, 61, filt, IK_JPEG, q)
    for im, b in zip(imgs, got):
        assert b == oracle.jpeg_encode_rgb(oracle.to_rgb8(oracle.resize(im, 97, 61, filt)), q)


@pytest.mark.parametrize("q", [50, 80])
def test_pipeline_webp_bytes_match_libwebp(ik, oracle, q):
    imgs = [ikutil.synth(256, 192, 4, seed=s, pattern="S") for s in range(2)]
    got = _run(ik, imgs, 64, 48, 1, IK_WEBP, q)
    for im, b in zip(imgs, got):
        assert b == oracle.webp_encode_rgb(oracle.to_rgb8(oracle.resize(im, 64, 48, 1)), float(q))


def test_pipeline_config2_shape(ik, oracle):
    """configs[2]: 4096^2 RGBA -> 512^2 Lanczos3 -> JPEG q85 (two frames)."""
    imgs = [ikutil.synth(4096, 4096, 4, seed=70 + s, pattern="S") for s in range(2)]
    got = _run(ik, imgs, 512, 512, 4, IK_JPEG, 85, threads=2)
    for im, b in zip(imgs, got):
        assert b[:2] == b"\xff\xd8" and b[-2:] == b"\xff\xd9"
        assert b == oracle.jpeg_encode_rgb(oracle.to_rgb8(oracle.resize(im, 512, 512, 4)), 85)

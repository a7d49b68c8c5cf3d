"""GPU: the exact WebP coder (ik_webp_encode_exact_device: libwebp method 4's segment
analysis and macroblock decisions on the GPU -- ik_vp8_analysis.hip, ik_vp8x.hip --
and its bitstream on the host, ik_vp8x_host.cpp).  The reference codes WebP with libwebp
(reference src/transform.rs:129-137 -> webp 0.3.1 Encoder::from_rgb(..).encode(q)).

Bar: the file is byte-identical to WebPEncodeRGB(to_rgb8(img), q) -- on the committed
golden WebP bytes, ragged sizes, smooth and noise content, qualities 1 ... 100 (chroma
error diffusion on at <= 98), batches, and 512x512 frames made the bench's way."""
import ctypes
import os

import numpy as np
import pytest

import ikutil
from imagekit import DynamicImage, FilterType, _lib
from test_gpu_vp8_analysis import _device_yuv_batch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "codec_golden.npz")


def encode_exact(ik, imgs, q):
    h, w, _ = imgs[0].shape
    dy, stride = _device_yuv_batch(ik, imgs)
    n = len(imgs)
    outs = (_lib.u8p * n)()
    lens = (ctypes.c_size_t * n)()
    try:
        assert ik.ik_webp_encode_exact_device(dy, stride, n, w, h, int(q), ctypes.cast(outs, ctypes.c_void_p),
                                              ctypes.cast(lens, ctypes.c_void_p)) == 0, _lib.last_error()
    finally:
        ik.ik_dev_free(dy)
    files = []
    for i in range(n):
        files.append(ctypes.string_at(outs[i], lens[i]))
        ik.ik_buf_free(outs[i])
    return files


def first_diff(a, b):
    return next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))


def test_golden_webp_bytes(ik):
    g = np.load(GOLD)
    for name in ("a", "b", "c", "d"):
        W, H, pat, seed, q = (int(v) for v in g[f"{name}_meta"])
        rgb = ikutil.synth(W, H, 3, seed=seed, pattern="SN"[pat])
        got = encode_exact(ik, [rgb], q)[0]
        want = bytes(g[f"{name}_webp"])
        assert got == want, f"{name}: differs at byte {first_diff(got, want)} ({len(got)} vs {len(want)} bytes)"


@pytest.mark.parametrize("wh", [(1, 1), (7, 5), (16, 16), (17, 31), (64, 48), (333, 222), (512, 512)])
@pytest.mark.parametrize("pat", ["S", "N"])
@pytest.mark.parametrize("q", [1, 50, 80, 100])
def test_equals_webpencodergb(ik, oracle, wh, pat, q):
    w, h = wh
    img = ikutil.synth(w, h, 4, seed=w + 5 * h, pattern=pat)
    got = encode_exact(ik, [img], q)[0]
    want = oracle.webp_encode_rgb(oracle.to_rgb8(img), float(q))
    assert got == want, f"{w}x{h} {pat} q{q}: differs at byte {first_diff(got, want)} ({len(got)} vs {len(want)})"


# frames above 1,024 MBs: epochs of more than 96 MBs (M = mb_count / 8), many diagonals
# per epoch, and statistics folds in raster order (an epoch over 163 MBs can reach
# libwebp's 65,534 halving point, so k_vp8x_run folds it serially)
@pytest.mark.parametrize("w,h,pat,q", [(799, 799, "S", 80), (1024, 1024, "S", 80), (1000, 600, "N", 80),
                                       (1000, 600, "S", 95), (1920, 1080, "S", 80)])
def test_large_frames(ik, oracle, w, h, pat, q):
    img = ikutil.synth(w, h, 3, seed=w ^ h, pattern=pat)
    got = encode_exact(ik, [img], q)[0]
    want = oracle.webp_encode_rgb(img, float(q))
    assert got == want, f"{w}x{h} {pat} q{q}: differs at byte {first_diff(got, want)} ({len(got)} vs {len(want)})"


def test_counters_past_the_halving_point(ik, oracle):
    # 1920x1080 noise at q95: 8,160 MBs of 25 coded blocks each -- a coefficient slot's
    # record count passes 65,534 within the frame, so libwebp halves it mid-frame and
    # the fold's raster order decides the probabilities
    img = ikutil.synth(1920, 1080, 3, seed=7, pattern="N")
    got = encode_exact(ik, [img], 95)[0]
    want = oracle.webp_encode_rgb(img, 95.0)
    assert got == want, f"differs at byte {first_diff(got, want)} ({len(got)} vs {len(want)})"


def test_work_area_growth(ik, oracle):
    # one thread's calls: small, large (the work area and pinned buffers grow), small
    # again on the grown area, and a batch of two large frames
    shapes = [(64, 48), (1280, 720), (96, 80)]
    for k, (w, h) in enumerate(shapes):
        img = ikutil.synth(w, h, 3, seed=11 + k, pattern="S")
        assert encode_exact(ik, [img], 80)[0] == oracle.webp_encode_rgb(img, 80.0), f"{w}x{h}"
    imgs = [ikutil.synth(1280, 720, 3, seed=s, pattern="SN"[s]) for s in range(2)]
    for i, (got, img) in enumerate(zip(encode_exact(ik, imgs, 80), imgs)):
        assert got == oracle.webp_encode_rgb(img, 80.0), f"batch image {i}"


def test_batch(ik, oracle):
    imgs = [ikutil.synth(512, 512, 3, seed=s, pattern="SSNS"[s]) for s in range(4)]
    for i, (got, img) in enumerate(zip(encode_exact(ik, imgs, 80), imgs)):
        assert got == oracle.webp_encode_rgb(img, 80.0), f"batch image {i}"


def test_bench_frames(ik, oracle):
    smalls = [DynamicImage.from_array(ikutil.synth(4096, 4096, 4, seed=s, pattern="S")).resize(
        512, 512, FilterType.Triangle).to_array() for s in range(2)]
    for i, (got, img) in enumerate(zip(encode_exact(ik, smalls, 80), smalls)):
        assert got == oracle.webp_encode_rgb(oracle.to_rgb8(img), 80.0), f"bench frame {i}"


def test_transform_batch_with_the_exact_coder(ik):
    # encode_image's WebP branch through the batch path (same-geometry groups and a
    # single request) with IK_WEBP_EXACT: the bytes equal the libwebp coder's (the
    # default) for the same requests
    import io
    from PIL import Image
    from imagekit import ImageFormat, transform_batch
    datas = []
    for s in range(3):
        b = io.BytesIO()
        Image.fromarray(ikutil.synth(1024, 768, 4, seed=s, pattern="S"), "RGBA").save(b, format="PNG")
        datas.append(b.getvalue())
    datas.append(datas[0])
    sizes = [(512, None)] * 3 + [(300, 200)]
    fmts = [ImageFormat.webp] * 4
    qs = [80, 80, 80, 50]
    prev = ik.ik_get_webp_encoder()
    try:
        assert ik.ik_set_webp_encoder(0) == 0
        ref = transform_batch(datas, sizes, fmts, qs, FilterType.Triangle)
        assert ik.ik_set_webp_encoder(2) == 0
        got = transform_batch(datas, sizes, fmts, qs, FilterType.Triangle)
    finally:
        ik.ik_set_webp_encoder(prev)
    assert got == ref

"""GPU: libwebp's method-4 segment analysis on the device (ik_vp8_analyze_device:
k_vp8_analyze + k_vp8_kmeans in ik_vp8_analysis.hip, the header arithmetic in
ik_webp_gpu.cpp) -- the first stage of a byte-exact GPU WebP coder (reference
src/transform.rs:129-137 -> webp 0.3.1 -> libwebp).

Bar: for every frame, the segment map, segment quantisers, base quantiser, chroma
quantiser deltas and segment-tree probabilities equal the ones libwebp wrote into
its own bytes for the same pixels (WebPEncodeRGB, read back by tests/vp8_parse.py),
on the committed golden WebP bytes, on ragged sizes, at several qualities, in
batches, and on 512x512 frames made the bench's way (4096x4096 synthetic frames,
resized on the GPU)."""
import ctypes
import os

import numpy as np
import pytest

import ikutil
import vp8_parse
from imagekit import DynamicImage, FilterType, _lib

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "codec_golden.npz")


class SegHeader(ctypes.Structure):
    _fields_ = [("num_segments", ctypes.c_int32), ("update_map", ctypes.c_int32), ("quant", ctypes.c_int32 * 4),
                ("fstrength", ctypes.c_int32 * 4), ("base_quant", ctypes.c_int32), ("dq_uv_dc", ctypes.c_int32),
                ("dq_uv_ac", ctypes.c_int32), ("probs", ctypes.c_int32 * 3), ("alpha", ctypes.c_int32),
                ("uv_alpha", ctypes.c_int32)]


def _device_yuv_batch(ik, imgs):
    """Every image through the product's device colour conversion (to_rgb8 + libwebp's
    RGB->YUV420, ik_webp_yuv420_device) into one buffer, images `stride` apart."""
    h, w, _ = imgs[0].shape
    n1 = w * h + 2 * ((w + 1) // 2) * ((h + 1) // 2)
    stride = (n1 + 255) // 256 * 256
    dy = ctypes.c_void_p()
    assert ik.ik_dev_alloc(stride * len(imgs), ctypes.byref(dy)) == 0
    for i, img in enumerate(imgs):
        c = img.shape[2]
        pitch = ((w * c + 255) // 256) * 256
        ds = ctypes.c_void_p()
        assert ik.ik_dev_alloc(pitch * h + 16, ctypes.byref(ds)) == 0
        buf = np.zeros((h, pitch), np.uint8)
        buf[:, :w * c] = img.reshape(h, w * c)
        assert ik.ik_memcpy_h2d(ds, buf.ctypes.data, buf.nbytes) == 0
        assert ik.ik_webp_yuv420_device(ds, w, h, c, pitch, ctypes.c_void_p(dy.value + i * stride), None) == 0, \
            _lib.last_error()
        assert ik.ik_dev_synchronize() == 0
        ik.ik_dev_free(ds)
    return dy, stride


def analyze(ik, imgs, q):
    h, w, _ = imgs[0].shape
    dy, stride = _device_yuv_batch(ik, imgs)
    nmb = ((w + 15) // 16) * ((h + 15) // 16)
    seg = np.zeros(nmb * len(imgs), np.uint8)
    hdr = (SegHeader * len(imgs))()
    try:
        assert ik.ik_vp8_analyze_device(dy, stride, len(imgs), w, h, ctypes.c_float(q), seg.ctypes.data,
                                        ctypes.cast(hdr, ctypes.c_void_p)) == 0, _lib.last_error()
    finally:
        ik.ik_dev_free(dy)
    return [{"segments": seg[i * nmb:(i + 1) * nmb], "num_segments": hdr[i].num_segments,
             "update_map": hdr[i].update_map, "quant": list(hdr[i].quant), "base_quant": hdr[i].base_quant,
             "uv_dc": hdr[i].dq_uv_dc, "uv_ac": hdr[i].dq_uv_ac, "probs": list(hdr[i].probs)} for i in range(len(imgs))]


def check(got, r, where):
    from test_vp8_analysis import check_against_bitstream
    check_against_bitstream(got, r, where)


def test_golden_webp_bytes(ik):
    g = np.load(GOLD)
    for name in ("a", "b", "c", "d"):
        W, H, pat, seed, q = (int(v) for v in g[f"{name}_meta"])
        rgb = ikutil.synth(W, H, 3, seed=seed, pattern="SN"[pat])
        check(analyze(ik, [rgb], float(q))[0], vp8_parse.parse(bytes(g[f"{name}_webp"])), name)


@pytest.mark.parametrize("wh", [(1, 1), (7, 5), (16, 16), (17, 31), (64, 48), (65, 49), (100, 70), (333, 222),
                                (511, 257), (512, 512), (1000, 600)])
@pytest.mark.parametrize("pat", ["S", "N"])
@pytest.mark.parametrize("q", [10.0, 80.0, 95.0])
def test_equals_libwebp(ik, oracle, wh, pat, q):
    w, h = wh
    img = ikutil.synth(w, h, 4, seed=w + 7 * h, pattern=pat)
    r = vp8_parse.parse(oracle.webp_encode_rgb(oracle.to_rgb8(img), q))
    check(analyze(ik, [img], q)[0], r, f"{w}x{h} {pat} q{q}")


def test_batch_of_images(ik, oracle):
    imgs = [ikutil.synth(512, 512, 3, seed=s, pattern="SSNS"[s]) for s in range(4)]
    got = analyze(ik, imgs, 80.0)
    for i, img in enumerate(imgs):
        check(got[i], vp8_parse.parse(oracle.webp_encode_rgb(img, 80.0)), f"batch image {i}")


@pytest.mark.parametrize("seed", [0, 1])
def test_bench_frames(ik, oracle, seed):
    # bench.py's headline frame: 4096x4096 RGBA8 synthetic, Triangle-resized to 512x512
    small = DynamicImage.from_array(ikutil.synth(4096, 4096, 4, seed=seed, pattern="S")).resize(
        512, 512, FilterType.Triangle).to_array()
    got = analyze(ik, [small], 80.0)[0]
    r = vp8_parse.parse(oracle.webp_encode_rgb(oracle.to_rgb8(small), 80.0))
    assert r["segment"]["update_map"]  # these frames do use 4 segments
    check(got, r, f"bench frame {seed}")

"""GPU: decode_image's WebP branch on the device (ik_vp8d_host.cpp + ik_vp8d.hip) -- the
reference decodes with load_from_memory_with_format (src/transform.rs:31); this path is
pinned to libwebp's WebPDecodeRGB (fancy upsampling, libwebp's YUV -> RGB).

Bar: pixels identical to WebPDecodeRGB (tests/webp_tool.py, the system libwebp 1.2.2)
on the committed golden WebP bytes, on files of the default encoder and of advanced
configurations (one to four segments, no / simple / normal loop filter, sharpness,
several token partitions, methods 0..6, qualities 0..100), ragged sizes, large
frames, VP8X containers without alpha, and the files the exact GPU coder writes.
IK_WEBP_DECODE=gpu makes a file the GPU path would leave to libwebp an error, so
these tests prove the device decoded them.  Files it leaves to libwebp on purpose
(alpha, lossless, truncated token data) keep libwebp's answer."""
import io
import os

import numpy as np
import pytest

import ikutil
import webp_tool as wt
from imagekit import DynamicImage, FilterType, ImageFormat, TransformError, decode_image, encode_image

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "codec_golden.npz")


@pytest.fixture
def gpu_only(monkeypatch):
    monkeypatch.setenv("IK_WEBP_DECODE", "gpu")


def gpu_decode(data: bytes) -> np.ndarray:
    img, fmt = decode_image(data)
    assert fmt is ImageFormat.webp
    return img.to_array()


def check(data: bytes, what=""):
    want = wt.decode_rgb(data)
    got = gpu_decode(data)
    assert got.shape == want.shape, what
    if not np.array_equal(got, want):
        bad = np.argwhere(np.any(got != want, axis=-1))
        y, x = bad[0]
        raise AssertionError(f"{what}: {len(bad)} pixels differ, first at ({x}, {y}): {got[y, x]} vs {want[y, x]}")


def test_golden_webp_bytes(ik, gpu_only):
    g = np.load(GOLD)
    for name in ("a", "b", "c", "d"):
        check(bytes(g[f"{name}_webp"]), name)


@pytest.mark.parametrize("wh", [(1, 1), (7, 5), (16, 16), (17, 31), (33, 21), (100, 75), (333, 222), (512, 512)])
@pytest.mark.parametrize("pat", ["S", "N"])
@pytest.mark.parametrize("q", [0, 50, 80, 100])
def test_default_encoder(ik, gpu_only, wh, pat, q):
    w, h = wh
    img = ikutil.synth(w, h, 3, seed=w * 7 + h, pattern=pat)
    check(wt.encode(img, q), f"{w}x{h} {pat} q{q}")


CONFIGS = [
    dict(segments=1, sns_strength=0),
    dict(segments=2),
    dict(segments=4, sns_strength=100),
    dict(filter_strength=0),
    dict(filter_type=0, filter_strength=60),
    dict(filter_type=0, filter_strength=100, filter_sharpness=5),
    dict(filter_strength=100, filter_sharpness=7),
    dict(filter_strength=40, filter_sharpness=2),
    dict(method=0, partitions=1),
    dict(method=0, partitions=2),
    dict(method=1, partitions=3, filter_type=0, filter_strength=50),
    dict(method=2, partitions=3, segments=4),
    dict(method=6),
    dict(method=3, autofilter=1),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[",".join(f"{k}={v}" for k, v in c.items()) for c in CONFIGS])
@pytest.mark.parametrize("q", [10, 75, 95])
def test_encoder_configurations(ik, gpu_only, cfg, q):
    for k, (w, h, pat) in enumerate([(301, 257, "S"), (130, 66, "N")]):
        img = ikutil.synth(w, h, 3, seed=13 + k, pattern=pat)
        check(wt.encode(img, q, **cfg), f"{w}x{h} {pat} q{q} {cfg}")


def test_configurations_cover_the_bitstream_features(ik):
    img = ikutil.synth(301, 257, 3, seed=13, pattern="S")
    infos = [wt.vp8_frame_info(wt.encode(img, 75, **c)) for c in CONFIGS]
    assert {i["partitions"] for i in infos} >= {1, 2, 4, 8}
    assert any(i["simple"] and i["level"] for i in infos) and any(not i["simple"] and i["level"] for i in infos)
    assert any(i["level"] == 0 for i in infos) and any(i["sharpness"] >= 5 for i in infos)
    assert any(not i["segments"] for i in infos) and any(i["update_map"] for i in infos)


@pytest.mark.parametrize("w,h,pat,q", [(1920, 1080, "S", 80), (1023, 769, "N", 60), (4096, 64, "S", 90),
                                       (64, 2049, "S", 30)])
def test_large_frames(ik, gpu_only, w, h, pat, q):
    img = ikutil.synth(w, h, 3, seed=w ^ h, pattern=pat)
    check(wt.encode(img, q), f"{w}x{h} {pat} q{q}")


def test_files_of_the_exact_coder(ik, gpu_only):
    # encode_image's own WebP output (the reference's transform output) decoded again
    for k, (w, h) in enumerate([(320, 240), (97, 61)]):
        img = DynamicImage.from_array(ikutil.synth(w, h, 4, seed=k, pattern="S"))
        for q in (30, 80):
            check(encode_image(img, ImageFormat.webp, q), f"{w}x{h} q{q}")


def test_vp8x_without_alpha(ik, gpu_only):
    # an extended container (EXIF + ICC chunks around the "VP8 " frame), no alpha
    from PIL import Image
    px = ikutil.synth(150, 99, 3, seed=21, pattern="S")
    b = io.BytesIO()
    Image.fromarray(px).save(b, format="WEBP", quality=70, exif=b"Exif\x00\x00MM\x00*\x00\x00\x00\x08\x00\x00",
                             icc_profile=b"\x00" * 128)
    data = b.getvalue()
    assert data[12:16] == b"VP8X"
    check(data, "VP8X")


def test_alpha_and_lossless_stay_on_libwebp(ik, monkeypatch):
    from PIL import Image
    px = ikutil.synth(40, 30, 4, seed=2, alpha="random")
    for kw in (dict(quality=80), dict(lossless=True, exact=True)):
        b = io.BytesIO()
        Image.fromarray(px).save(b, format="WEBP", **kw)
        data = b.getvalue()
        monkeypatch.setenv("IK_WEBP_DECODE", "gpu")
        with pytest.raises(TransformError):
            decode_image(data)
        monkeypatch.setenv("IK_WEBP_DECODE", "auto")
        img, _ = decode_image(data)
        assert img.channels == 4


def _truncate_tokens(data: bytes, keep: float) -> bytes:
    # cut the token partition short and rewrite the chunk and RIFF sizes, so that
    # the container is consistent and only the token data runs out
    f = bytearray(data[20:])
    part0 = (f[0] | f[1] << 8 | f[2] << 16) >> 5
    start = 10 + part0
    cut = start + max(1, int((len(f) - start) * keep))
    f = bytes(f[:cut])
    if len(f) & 1:
        f += b"\x00"
    body = b"WEBP" + b"VP8 " + len(f).to_bytes(4, "little") + f
    return b"RIFF" + len(body).to_bytes(4, "little") + body


def test_token_data_running_out(ik, monkeypatch):
    img = ikutil.synth(200, 150, 3, seed=8, pattern="N")
    data = _truncate_tokens(wt.encode(img, 90), 0.5)
    with pytest.raises(ValueError):
        wt.decode_rgb(data)  # libwebp: premature end of file
    monkeypatch.setenv("IK_WEBP_DECODE", "gpu")
    with pytest.raises(TransformError):
        decode_image(data)  # the GPU path hands it back
    monkeypatch.setenv("IK_WEBP_DECODE", "auto")
    with pytest.raises(TransformError):
        decode_image(data)  # and libwebp's verdict is the answer


def test_transform_batch_webp_inputs(ik, gpu_only):
    # WebP inputs through the batch path (decode_batch_dev -> the device decoder per
    # item, in parallel) -> resize -> JPEG: the same bytes as the one-request path
    from imagekit import transform_batch
    from imagekit.transform import transform
    datas = [wt.encode(ikutil.synth(640 + 16 * s, 480, 3, seed=s, pattern="S"), 80) for s in range(5)]
    sizes = [(320, None)] * 5
    fmts = [ImageFormat.jpeg] * 5
    qs = [85] * 5
    got = transform_batch(datas, sizes, fmts, qs, FilterType.Triangle)
    for i, d in enumerate(datas):
        assert got[i] == transform(d, 320, None, ImageFormat.jpeg, 85, FilterType.Triangle), i


def test_auto_policy(ik, monkeypatch):
    # default (auto): frames from 3 MPix on take the device path, smaller ones libwebp;
    # either way the pixels are WebPDecodeRGB's
    monkeypatch.delenv("IK_WEBP_DECODE", raising=False)
    for w, h in [(2048, 1536), (640, 480)]:
        img = ikutil.synth(w, h, 3, seed=w, pattern="S")
        check(wt.encode(img, 80), f"auto {w}x{h}")

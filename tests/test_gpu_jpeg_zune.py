"""GPU: decode_image on a JPEG in the default reconstruction mode -- zune-jpeg
0.4.21's (reference src/transform.rs:31 -> image 0.25.8 -> zune-jpeg,
Cargo.lock:3106-3109).

Bar: the GPU's pixels equal the oracle's zune-jpeg restatement
(oracle/jpeg_dec.c IKO_JPEG_ZUNE: stb_image-derived IDCT with the DC-only
shortcut, separable +2 >> 2 upsampling over the MCU-padded rows, i16 YCbCr->RGB)
bit for bit, across baseline / progressive, 4:4:4 / 4:2:2 / 4:2:0, gray, restart
intervals (GPU entropy decoding), restart-free scans (self-synchronising GPU
decoding), batches, CMYK.  libjpeg-turbo (Pillow) is kept as a sanity bound
only: the two reconstructions differ by rounding, not by content.  Parity with
zune-jpeg itself is unpinned (no crate sources or outputs in this environment).
"""
import io

import numpy as np
import pytest
from PIL import Image, ImageFile

import ikutil
from imagekit import ImageFormat, decode_image, decode_image_batch, encode_image, resize_image

pytestmark = pytest.mark.gpu

ZUNE = 1


def _jpeg(img, mode=None, **kw):
    ImageFile.MAXBLOCK = max(ImageFile.MAXBLOCK, 1 << 24)
    buf = io.BytesIO()
    Image.fromarray(img, mode).save(buf, format="JPEG", **kw)
    return buf.getvalue()


def _bound(got, b):
    """sanity bound against libjpeg-turbo: rounding-level differences only"""
    pil = np.asarray(Image.open(io.BytesIO(b)).convert("RGB" if got.shape[-1] == 3 else "L"))
    d = np.abs(got.astype(np.int32) - pil.reshape(got.shape).astype(np.int32))
    assert np.percentile(d, 99.9) <= 16 and (d.mean() < 1.5 if d.size >= 768 else d.max() <= 8), (d.mean(), d.max())


@pytest.fixture(autouse=True)
def zune_mode(ik):
    assert ik.ik_get_jpeg_reconstruction() == ZUNE  # the default


@pytest.mark.parametrize("wh", [(640, 480), (17, 9), (1, 1), (33, 65), (2000, 1000)])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("q", [50, 90])
def test_baseline_equals_zune_restatement(oracle, wh, sub, q):
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + q), quality=q, subsampling=sub)
    img, fmt = decode_image(b)
    assert fmt is ImageFormat.jpeg
    got = img.to_array()
    np.testing.assert_array_equal(got, oracle.jpeg_decode(b, ZUNE))
    _bound(got, b)


@pytest.mark.parametrize("wh", [(64, 64), (37, 19), (641, 479)])
@pytest.mark.parametrize("sub", [0, 2])
@pytest.mark.parametrize("q", [30, 95])
def test_progressive_equals_zune_restatement(oracle, wh, sub, q):
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w * h + q, pattern="N" if q == 95 else "S"), quality=q, subsampling=sub,
              progressive=True)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE))


def test_gray_restarts_and_self_sync(oracle):
    g = ikutil.synth(123, 77, 1, seed=3)[..., 0]
    b = _jpeg(g, quality=80)
    img, _ = decode_image(b)
    assert img.channels == 1
    np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE))
    for kw in ({"restart_marker_rows": 1}, {"restart_marker_blocks": 5}, {}):
        b = _jpeg(ikutil.synth(1500, 900, 3, seed=1, pattern="S"), quality=90, subsampling=2, **kw)
        img, _ = decode_image(b)
        np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE))


def test_dc_only_blocks_take_the_shortcut(oracle):
    """Flat 8x8 areas: every AC coefficient zero -> zune-jpeg writes (dc >> 3) + 128,
    which is not always what the full IDCT rounds to (libjpeg differs there)."""
    levels = np.arange(100, 164, dtype=np.uint8).reshape(8, 8)
    img = np.repeat(np.repeat(levels, 8, 0), 8, 1)[..., None].repeat(3, 2)  # flat 8x8 blocks, 64 gray levels
    b = _jpeg(img, quality=90, subsampling=0)  # DC step 3: off the multiples of 8
    got, _ = decode_image(b)
    np.testing.assert_array_equal(got.to_array(), oracle.jpeg_decode(b, ZUNE))


@pytest.mark.parametrize("q", [60, 92])
def test_cmyk_decodes_to_rgb(ik, oracle, q):
    """4-component Adobe CMYK (Pillow writes it inverted) -> RGB8, as Pillow's
    cmyk2rgb: equal to Pillow in the libjpeg mode, to the restatement by default."""
    c = ikutil.synth(160, 90, 4, seed=q)
    b = _jpeg(c, "CMYK", quality=q)
    img, fmt = decode_image(b)
    assert fmt is ImageFormat.jpeg and img.channels == 3
    np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE))
    assert ik.ik_set_jpeg_reconstruction(0) == 0
    try:
        lj, _ = decode_image(b)
        np.testing.assert_array_equal(lj.to_array(), np.asarray(Image.open(io.BytesIO(b)).convert("RGB")))
    finally:
        assert ik.ik_set_jpeg_reconstruction(ZUNE) == 0


def test_batch_equals_restatement(oracle):
    blobs = [_jpeg(ikutil.synth(w, h, 3, seed=k), quality=88, subsampling=s, **kw)
             for k, (w, h, s, kw) in enumerate([(320, 240, 2, {"restart_marker_rows": 1}), (1000, 700, 1, {}),
                                                (333, 222, 0, {"progressive": True}), (2048, 1536, 2, {})])]
    out = decode_image_batch(blobs)
    for (img, fmt), b in zip(out, blobs):
        assert fmt is ImageFormat.jpeg
        np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE))


def test_config1_jpeg_to_webp_equals_oracle(oracle):
    """configs[1]-style request: JPEG in -> resize_image -> WebP out, byte for byte
    the oracle's transform of the oracle's zune-jpeg decode."""
    b = _jpeg(ikutil.synth(640, 480, 3, seed=11, pattern="S"), quality=90)
    img, _ = decode_image(b)
    out = resize_image(img, 320, None)
    want, dims = oracle.transform(oracle.jpeg_decode(b, ZUNE), 320, None, 4, 1, 80)
    assert dims == (320, 240)
    assert encode_image(out, ImageFormat.webp, 80) == want


@pytest.mark.parametrize("sub", [1, 2])
def test_batch_colour_edges_equal_restatement(oracle, sub):
    """The batched colour kernels (ik_jpeg.hip k_jpeg_color_fast_b: eight pixels by
    16 rows per thread, interior groups only; k_jpeg_color_ends_b: the row ends)
    over images whose widths and heights fall on and off the group, MCU and band
    boundaries, mixed in one batch so that the grid is sized by the widest."""
    sizes = [(48, 48), (49, 50), (57, 41), (63, 64), (65, 33), (100, 61), (257, 129), (1023, 77), (4001, 24),
             (520, 9), (16, 300), (24, 17)]
    blobs = [_jpeg(ikutil.synth(w, h, 3, seed=40 + k, pattern="N"), quality=95, subsampling=sub,
                   **({"restart_marker_rows": 1} if k % 3 == 0 else {}))
             for k, (w, h) in enumerate(sizes)]
    out = decode_image_batch(blobs)
    for (img, fmt), b, wh in zip(out, blobs, sizes):
        assert fmt is ImageFormat.jpeg
        np.testing.assert_array_equal(img.to_array(), oracle.jpeg_decode(b, ZUNE), err_msg=str(wh))

"""CPU: the oracle's JPEG decoder (oracle/jpeg_dec.c), pinned.

Its libjpeg-turbo reconstruction must equal Pillow's decoder (libjpeg-turbo
3.1.4) bit for bit on every stream shape the GPU tests use -- baseline and
progressive, 4:4:4 / 4:2:2 / 4:2:0, gray, restart intervals, CMYK -- which pins
the entropy decoder both reconstructions share.  The zune-jpeg 0.4.21
restatement (the reference's decoder; parity unpinned) must stay within a
rounding-level bound of it, and take zune-jpeg's DC-only shortcut."""
import io

import numpy as np
import pytest
from PIL import Image, ImageFile

import ikutil

LIBJPEG, ZUNE = 0, 1


def _jpeg(img, mode=None, **kw):
    ImageFile.MAXBLOCK = max(ImageFile.MAXBLOCK, 1 << 24)
    buf = io.BytesIO()
    Image.fromarray(img, mode).save(buf, format="JPEG", **kw)
    return buf.getvalue()


CASES = [
    ((640, 480), 2, 90, {}), ((17, 9), 1, 50, {}), ((1, 1), 0, 90, {}), ((33, 65), 2, 50, {}),
    ((321, 243), 0, 95, {}), ((500, 301), 2, 50, {"progressive": True}),
    ((97, 61), 1, 80, {"progressive": True, "restart_marker_blocks": 3}), ((257, 129), 2, 85, {"restart_marker_rows": 1}),
]


@pytest.mark.parametrize("wh,sub,q,kw", CASES)
def test_libjpeg_mode_equals_pillow(oracle, wh, sub, q, kw):
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + q, pattern="N" if q == 95 else "S"), quality=q, subsampling=sub, **kw)
    pil = np.asarray(Image.open(io.BytesIO(b)))
    np.testing.assert_array_equal(oracle.jpeg_decode(b, LIBJPEG), pil)
    zu = oracle.jpeg_decode(b, ZUNE)
    d = np.abs(zu.astype(np.int32) - pil.astype(np.int32))
    # rounding-level: zune's colour constants (45/32 ... ) and DC shortcut move a
    # sample by a few levels at most; one pixel's "mean" is its own difference
    assert np.percentile(d, 99.9) <= 16 and (d.mean() < 1.5 if d.size >= 768 else d.max() <= 8)


def test_gray_and_cmyk_equal_pillow(oracle):
    g = ikutil.synth(200, 100, 1, seed=1)[..., 0]
    b = _jpeg(g, "L", quality=85)
    np.testing.assert_array_equal(oracle.jpeg_decode(b, LIBJPEG)[..., 0], np.asarray(Image.open(io.BytesIO(b))))
    c = ikutil.synth(160, 90, 4, seed=3)
    b = _jpeg(c, "CMYK", quality=90)
    im = Image.open(io.BytesIO(b))
    assert im.mode == "CMYK"
    np.testing.assert_array_equal(oracle.jpeg_decode(b, LIBJPEG), np.asarray(im.convert("RGB")))


def test_zune_dc_only_shortcut(oracle):
    """A flat block: zune-jpeg's (dc >> 3) + 128 truncates where the full IDCT
    (and libjpeg) round, so some flat levels come out one lower."""
    levels = np.arange(100, 160, dtype=np.uint8)
    img = np.repeat(np.repeat(levels[None, :, None], 8, 0), 8, 1)  # 8 x (60*8) gray, one level per block
    b = _jpeg(img[..., 0], "L", quality=90)  # DC step 3: dequantised DCs off the multiples of 8
    zu = oracle.jpeg_decode(b, ZUNE)[..., 0]
    lj = oracle.jpeg_decode(b, LIBJPEG)[..., 0]
    assert (zu <= lj).all() and (zu < lj).any()
    assert (lj.astype(int) - zu.astype(int)).max() == 1

"""GPU: ik_transform_batch -- the /img handler (reference src/lib.rs:175-191) for
many requests at once, loadtest-style mixed inputs, sizes and formats
(loadtest/src/main.rs:59-60,84-85).  Bar: every request's bytes equal
ik_transform on the same request (itself pinned against the oracle by the
decode/resize/encode parity tests), except AVIF, whose encoder is not
deterministic across threads: decodable, right size."""
import ctypes
import io

import numpy as np
import pytest
from PIL import Image

import ikutil
from imagekit import ImageFormat, TransformError, _lib, transform_batch

pytestmark = pytest.mark.gpu


def _single(ik, b, w, h, fmt, q, filt=4):
    out, n = _lib.u8p(), ctypes.c_size_t()
    assert ik.ik_transform(b, len(b), -1 if w is None else w, -1 if h is None else h, fmt.value, q, filt,
                           ctypes.byref(out), ctypes.byref(n)) == 0, _lib.last_error()
    r = ctypes.string_at(out, n.value)
    ik.ik_buf_free(out)
    return r


def _inputs():
    blobs = []
    for k, (w, h) in enumerate([(640, 480), (1000, 700), (333, 222), (800, 600)]):
        buf = io.BytesIO()
        Image.fromarray(ikutil.synth(w, h, 3, seed=k, pattern="S")).save(
            buf, format="JPEG", quality=90, subsampling=2, **({"restart_marker_rows": 1} if k % 2 == 0 else {}))
        blobs.append(buf.getvalue())
    buf = io.BytesIO()
    Image.fromarray(ikutil.synth(300, 200, 4, seed=9)).save(buf, format="PNG")
    blobs.append(buf.getvalue())
    buf = io.BytesIO()
    Image.fromarray(ikutil.synth(256, 256, 3, seed=10)).save(buf, format="WEBP", quality=90)
    blobs.append(buf.getvalue())
    return blobs


def test_transform_batch_equals_single_requests(ik):
    blobs = _inputs()
    sizes = [(320, None), (None, 240), (None, None), (400, 400), (150, 100), (512, None)]
    fmts = [ImageFormat.webp, ImageFormat.jpeg, ImageFormat.webp, ImageFormat.jpeg, ImageFormat.webp, ImageFormat.jpeg]
    qs = [80, 85, 75, 90, 80, 80]
    got = transform_batch(blobs, sizes, fmts, qs, threads=4)
    for b, (w, h), f, q, g in zip(blobs, sizes, fmts, qs, got):
        assert g == _single(ik, b, w, h, f, q)


def test_transform_batch_avif_and_errors(ik):
    blobs = _inputs()[:2]
    got = transform_batch(blobs, [(160, None), (None, 120)], [ImageFormat.avif, ImageFormat.avif], [60, 60])
    for g, (w, h) in zip(got, [(160, 120), (171, 120)]):
        im = Image.open(io.BytesIO(g))
        assert im.size == (w, h)
    with pytest.raises(TransformError):
        transform_batch([blobs[0], b"not an image"], [(10, None), (10, None)], [ImageFormat.jpeg] * 2, [80, 80])

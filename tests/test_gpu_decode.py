"""GPU: decode_image (reference src/transform.rs:27-43) through ik_decode.

JPEG, in the libjpeg-turbo reconstruction mode (ik_set_jpeg_reconstruction(
IK_JPEG_RECON_LIBJPEG): islow IDCT, fancy upsampling, fixed-point YCbCr) for the
whole module: must equal libjpeg-turbo (Pillow) bit for bit, which pins the
entropy decoding the default zune-jpeg mode shares (that mode:
tests/test_gpu_jpeg_zune.py).  PNG: decoding is specified exactly; checked
against Pillow/libpng and against the source pixels, across colour types, bit
depths, the five filter types and Adam7 (a small PNG writer below produces those).
"""
import ctypes
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image, ImageFile

import ikutil
from imagekit import ImageFormat, TransformError, decode_image

pytestmark = pytest.mark.gpu

IK_JPEG_RECON_LIBJPEG, IK_JPEG_RECON_ZUNE = 0, 1


@pytest.fixture(autouse=True, scope="module")
def libjpeg_reconstruction(ik):
    assert ik.ik_set_jpeg_reconstruction(IK_JPEG_RECON_LIBJPEG) == 0
    yield
    assert ik.ik_set_jpeg_reconstruction(IK_JPEG_RECON_ZUNE) == 0


def _jpeg(img, **kw):
    ImageFile.MAXBLOCK = max(ImageFile.MAXBLOCK, 1 << 24)  # progressive noise needs a big buffer
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", **kw)
    return buf.getvalue()


@pytest.mark.parametrize("wh", [(640, 480), (17, 9), (1, 1), (33, 65), (2000, 1000)])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("q", [50, 90])
def test_jpeg_decode_matches_libjpeg_turbo(ik, wh, sub, q):
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + q), quality=q, subsampling=sub)
    img, fmt = decode_image(b)
    assert fmt is ImageFormat.jpeg
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_gray_and_restart_markers(ik):
    g = ikutil.synth(123, 77, 1, seed=3)[..., 0]
    b = _jpeg(g, quality=80)
    img, _ = decode_image(b)
    assert img.channels == 1
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b))))
    b = _jpeg(ikutil.synth(300, 200, 3, seed=1), quality=90, subsampling=2, restart_marker_rows=1)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


@pytest.mark.parametrize("wh", [(64, 64), (1, 1), (37, 19), (641, 479)])
@pytest.mark.parametrize("sub", [0, 2])
@pytest.mark.parametrize("q", [30, 95])
def test_jpeg_progressive_matches_libjpeg_turbo(ik, wh, sub, q):
    # SOF2: DC first + refine, spectral-selection AC first, successive-approximation
    # AC refine with EOB runs (libjpeg's default progression script)
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w * h + q, pattern="N" if q == 95 else "S"), quality=q,
              subsampling=sub, progressive=True)
    assert b"\xff\xc2" in b
    img, fmt = decode_image(b)
    assert fmt is ImageFormat.jpeg
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_progressive_gray_and_restarts(ik):
    g = ikutil.synth(129, 70, 1, seed=5)[..., 0]
    b = _jpeg(g, quality=75, progressive=True)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b))))
    b = _jpeg(ikutil.synth(200, 150, 3, seed=6), quality=85, subsampling=1, progressive=True,
              restart_marker_blocks=3)
    assert b"\xff\xdd" in b
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def _jpeg_counts(ik):
    import ctypes
    c = (ctypes.c_ulonglong * 2)()
    assert ik.ik_jpeg_counters(c) == 0
    return c[0], c[1]


@pytest.mark.parametrize("wh,sub,q,rst", [
    ((640, 480), 2, 90, {"restart_marker_rows": 1}),
    ((333, 211), 0, 75, {"restart_marker_blocks": 5}),
    ((1000, 700), 1, 95, {"restart_marker_rows": 2}),
    ((64, 64), 2, 30, {"restart_marker_blocks": 1}),
    ((17, 9), 0, 50, {"restart_marker_blocks": 2}),
    ((2048, 1536), 2, 85, {"restart_marker_rows": 1}),
])
def test_jpeg_progressive_restarts_entropy_decoded_on_the_gpu(ik, wh, sub, q, rst):
    """Progressive scans with restart intervals (DC first/refine, AC first with EOB
    runs, AC refine) go through k_jpeg_prog, one lane per interval, scan after scan:
    equal to libjpeg-turbo, and the stream counted as GPU-decoded, not host."""
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + h + q, pattern="N" if q == 95 else "S"), quality=q, subsampling=sub,
              progressive=True, **rst)
    assert b"\xff\xc2" in b and b"\xff\xdd" in b
    g0, h0 = _jpeg_counts(ik)
    img, fmt = decode_image(b)
    g1, h1 = _jpeg_counts(ik)
    assert fmt is ImageFormat.jpeg
    assert (g1 - g0, h1 - h0) == (1, 0)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_progressive_restarts_gray_on_the_gpu(ik):
    g = ikutil.synth(257, 131, 1, seed=9)[..., 0]
    b = _jpeg(g, quality=88, progressive=True, restart_marker_blocks=4)
    g0, h0 = _jpeg_counts(ik)
    img, _ = decode_image(b)
    g1, h1 = _jpeg_counts(ik)
    assert (g1 - g0, h1 - h0) == (1, 0)
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_progressive_without_restarts_stays_on_the_host(ik):
    # a restart-free progressive scan is one serial bitstream: the host decoder
    b = _jpeg(ikutil.synth(120, 80, 3, seed=11), quality=80, progressive=True)
    g0, h0 = _jpeg_counts(ik)
    img, _ = decode_image(b)
    g1, h1 = _jpeg_counts(ik)
    assert (g1 - g0, h1 - h0) == (0, 1)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_progressive_restarts_corrupt_interval_gives_the_host_answer(ik):
    # a bad code in one interval: the GPU flags it and the host decoder decides
    b = bytearray(_jpeg(ikutil.synth(320, 240, 3, seed=12), quality=85, progressive=True,
                        restart_marker_rows=1))
    sos = [i for i in range(len(b) - 1) if b[i] == 0xFF and b[i + 1] == 0xDA]
    k = sos[len(sos) // 2] + 40  # inside a middle scan's data
    for j in range(k, k + 8):
        if b[j] != 0xFF and b[j - 1] != 0xFF:
            b[j] ^= 0x5A
    b = bytes(b)
    try:
        ref = np.asarray(Image.open(io.BytesIO(b)))
    except OSError:
        ref = None
    try:
        img, _ = decode_image(b)
        if ref is not None:
            assert img.to_array().shape == ref.shape
    except TransformError as e:
        assert "Jpeg" in str(e) or "jpeg" in str(e)


def test_jpeg_truncated_progressive_is_an_error_or_partial(ik):
    # a stream cut inside its entropy data decodes like libjpeg (missing bits read as
    # zeros) or fails with the reference's error string, never crashes
    b = _jpeg(ikutil.synth(96, 96, 3, seed=7), quality=80, progressive=True)
    for cut in (len(b) // 2, len(b) - 3):
        try:
            img, _ = decode_image(b[:cut])
            assert img.dimensions() == (96, 96)
        except TransformError as e:
            assert "Jpeg" in str(e) or "jpeg" in str(e)


# ---- PNG writer for the test (all filter types, Adam7, any colour type) ------
def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _filter_row(row, prev, bpp, ft):
    out = bytearray(len(row))
    for i in range(len(row)):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        if ft == 0: p = 0
        elif ft == 1: p = a
        elif ft == 2: p = b
        elif ft == 3: p = (a + b) >> 1
        else:
            pp = a + b - c
            pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
            p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
        out[i] = (row[i] - p) & 255
    return bytes([ft]) + bytes(out)


def _pack_rows(samples, depth):
    # samples: (h, w*spp) uint8 values < 2**depth
    if depth == 8:
        return [bytes(r) for r in samples]
    rows = []
    for r in samples:
        bits = "".join(format(int(v), f"0{depth}b") for v in r)
        bits += "0" * (-len(bits) % 8)
        rows.append(int(bits, 2).to_bytes(len(bits) // 8, "big") if bits else b"")
    return rows


def make_png(samples, w, h, ctype, depth=8, interlace=False, plte=None, trns=None):
    spp = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bpp = max(1, spp * depth // 8)
    raw = b""
    passes = ([(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
              if interlace else [(0, 0, 1, 1)])
    ft = 0
    for (x0, y0, dx, dy) in passes:
        sub = samples.reshape(h, w, spp)[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        rows = _pack_rows(sub.reshape(sub.shape[0], -1), depth)
        prev = None
        for r in rows:
            raw += _filter_row(r, prev, bpp, ft % 5)
            ft += 1
            prev = r
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if plte is not None:
        out += _chunk(b"PLTE", bytes(plte))
    if trns is not None:
        out += _chunk(b"tRNS", bytes(trns))
    out += _chunk(b"IDAT", zlib.compress(raw, 6)) + _chunk(b"IEND", b"")
    return out


@pytest.mark.parametrize("ctype,spp", [(0, 1), (2, 3), (4, 2), (6, 4)])
@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("wh", [(1, 1), (7, 5), (64, 48), (129, 33)])
def test_png_8bit_exact(ik, ctype, spp, interlace, wh):
    w, h = wh
    px = ikutil.synth(w, h, 4, seed=w * h + ctype, pattern="N")[..., :spp]
    b = make_png(np.ascontiguousarray(px), w, h, ctype, interlace=interlace)
    img, fmt = decode_image(b)
    assert fmt is None
    np.testing.assert_array_equal(img.to_array(), px.reshape(h, w, spp))


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_png_low_bit_gray_expands(ik, depth):
    w, h = 37, 11
    rng = np.random.default_rng(depth)
    v = rng.integers(0, 1 << depth, (h, w), dtype=np.uint8)
    b = make_png(v, w, h, 0, depth=depth)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array()[..., 0], v * (255 // ((1 << depth) - 1)))
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b)).convert("L")))


def test_png_palette_and_trns(ik):
    w, h = 40, 30
    rng = np.random.default_rng(7)
    idx = rng.integers(0, 16, (h, w), dtype=np.uint8)
    pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
    b = make_png(idx, w, h, 3, plte=pal.flatten())
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), pal[idx])
    alpha = np.arange(16, dtype=np.uint8) * 16
    b = make_png(idx, w, h, 3, plte=pal.flatten(), trns=alpha[:10])
    img, _ = decode_image(b)
    a = np.concatenate([alpha[:10], np.full(6, 255, np.uint8)])
    want = np.concatenate([pal[idx], a[idx][..., None]], -1)
    np.testing.assert_array_equal(img.to_array(), want)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b)).convert("RGBA")))


def test_png_rgb_trns_adds_alpha(ik):
    px = np.zeros((4, 5, 3), np.uint8)
    px[1, 2] = (10, 20, 30)
    b = make_png(px, 5, 4, 2, trns=[0, 10, 0, 20, 0, 30])
    img, _ = decode_image(b)
    out = img.to_array()
    assert out.shape == (4, 5, 4) and out[1, 2, 3] == 0 and (out[..., 3].sum() == 255 * 19)


def test_png_corruption_is_an_error(ik):
    b = bytearray(make_png(np.zeros((8, 8, 3), np.uint8), 8, 8, 2))
    b[40] ^= 0xFF  # inside IDAT -> CRC mismatch
    with pytest.raises(TransformError):
        decode_image(bytes(b))
    with pytest.raises(TransformError):
        decode_image(b[:30])


def _png_from_stream(w, h, stream, split=1):
    """RGB8 PNG whose IDAT data is `stream` (a zlib stream), cut into `split` chunks."""
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    step = -(-len(stream) // split)
    for i in range(0, len(stream), step):
        out += _chunk(b"IDAT", stream[i:i + step])
    return out + _chunk(b"IEND", b"")


def test_png_inflate_paths(ik):
    """The one-shot inflate (libdeflate) and the zlib path agree on what is an image:
    many IDAT chunks; extra data after the image rows (accepted, as the zlib path
    does); a short stream (an error)."""
    w, h = 300, 97
    px = ikutil.synth(w, h, 3, seed=5, pattern="S")
    raw = b"".join(_filter_row(px[y].tobytes(), px[y - 1].tobytes() if y else None, 3, 2 if y % 3 else 4)
                   for y in range(h))
    for split in (1, 7, 64):
        img, _ = decode_image(_png_from_stream(w, h, zlib.compress(raw, 9), split))
        np.testing.assert_array_equal(img.to_array(), px)
    img, _ = decode_image(_png_from_stream(w, h, zlib.compress(raw + bytes(50), 6)))
    np.testing.assert_array_equal(img.to_array(), px)
    with pytest.raises(TransformError):
        decode_image(_png_from_stream(w, h, zlib.compress(raw[:-10], 6)))


@pytest.mark.parametrize("blob", [b"GIF89a" + bytes(20), b"BM" + bytes(40),
                                  b"\x00\x00\x00\x1cftypavif" + bytes(20), bytes(100), b""])
def test_unsupported_or_unknown_formats(ik, blob):
    with pytest.raises(TransformError):
        decode_image(blob)


def test_webp_decode_and_format(ik):
    buf = io.BytesIO()
    Image.fromarray(ikutil.synth(33, 21, 3, seed=4)).save(buf, format="WEBP", quality=80)
    img, fmt = decode_image(buf.getvalue())
    assert fmt is ImageFormat.webp and img.dimensions() == (33, 21) and img.channels == 3
    # lossless with real alpha -> Rgba8 (an all-opaque lossless file has alpha_is_used = 0 -> Rgb8)
    px = ikutil.synth(33, 21, 4, seed=4)
    px[..., 3] = np.arange(33 * 21, dtype=np.uint32).reshape(21, 33) % 256
    buf = io.BytesIO()
    Image.fromarray(px).save(buf, format="WEBP", lossless=True, exact=True)
    img, fmt = decode_image(buf.getvalue())
    assert img.channels == 4
    np.testing.assert_array_equal(img.to_array(), px)


def test_config1_jpeg_to_webp(ik, oracle):
    """BASELINE configs[0]: 640x480 JPEG -> w=320 webp q80 through the device path,
    byte-identical to the CPU restatement fed the same decoded pixels."""
    from imagekit import encode_image, resize_image
    b = _jpeg(ikutil.synth(640, 480, 3, seed=0), quality=90)
    img, _ = decode_image(b)
    out = resize_image(img, 320, None)
    assert out.dimensions() == (320, 240)
    want, dims = oracle.transform(np.asarray(Image.open(io.BytesIO(b))), 320, None, 4, 1, 80)
    assert encode_image(out, ImageFormat.webp, 80) == want


# ---- GPU entropy decoding (the self-synchronising ik_jsync.hip path): baseline scans with restart intervals ----
@pytest.mark.parametrize("wh", [(16, 16), (300, 200), (1023, 767), (17, 9)])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("rst", [("rows", 1), ("rows", 3), ("blocks", 1), ("blocks", 7)])
def test_jpeg_restart_intervals_gpu_entropy(ik, wh, sub, rst):
    """Restart-marked baseline scans through the self-synchronising GPU decoder (ik_jsync.hip: lanes of
    1,024 bits, interval starts from the unstuffing pass); pixels equal libjpeg-turbo's."""
    w, h = wh
    kw = {"restart_marker_rows" if rst[0] == "rows" else "restart_marker_blocks": rst[1]}
    pat = "N" if (w * h) % 2 else "S"
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + h + sub, pattern=pat), quality=85, subsampling=sub, **kw)
    img, fmt = decode_image(b)
    assert fmt is ImageFormat.jpeg
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


@pytest.mark.parametrize("q", [10, 100])
def test_jpeg_restart_gray_and_extreme_quality(ik, q):
    g = ikutil.synth(257, 131, 1, seed=q, pattern="N")[..., 0]
    b = _jpeg(g, quality=q, restart_marker_blocks=5)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_restart_large_4096(ik):
    """A configs[2]-sized frame (4096 x 4096, 4:2:0, one restart per MCU row)."""
    b = _jpeg(ikutil.synth(4096, 4096, 3, seed=9, pattern="S"), quality=90, subsampling=2, restart_marker_rows=1)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_restart_corrupt_interval_is_handled_like_the_host(ik):
    """A bad code inside one interval: the GPU flags it and the host decoder
    decides (an error, or libjpeg-style tolerant output) -- never a crash."""
    b = bytearray(_jpeg(ikutil.synth(320, 240, 3, seed=4, pattern="N"), quality=90, restart_marker_rows=1))
    sos = b.index(b"\xff\xda")
    mid = sos + (len(b) - sos) // 2
    for i in range(mid, mid + 64):
        if b[i] not in (0xFF, 0x00) and b[i - 1] != 0xFF:
            b[i] = 0xFF ^ b[i] if b[i] != 0xFF else b[i]
    try:
        img, _ = decode_image(bytes(b))
        assert img.to_array().shape == (240, 320, 3)
    except TransformError:
        pass


def test_decode_batch_one_launch_matches_libjpeg_turbo(ik):
    """ik_decode_batch: restart JPEGs of mixed geometry/subsampling entropy-decoded
    in one GPU launch, plus inputs that take the single-image paths (no restarts,
    progressive, PNG); every result equals its own decoder's answer."""
    from imagekit import decode_image_batch
    blobs, want = [], []
    for k, (w, h, sub) in enumerate([(640, 480, 2), (333, 211, 0), (96, 64, 1), (1024, 768, 2), (17, 9, 2)]):
        b = _jpeg(ikutil.synth(w, h, 3, seed=50 + k, pattern="S" if k % 2 else "N"), quality=80 + k,
                  subsampling=sub, restart_marker_rows=1 + k % 2)
        blobs.append(b)
        want.append(np.asarray(Image.open(io.BytesIO(b))))
    b = _jpeg(ikutil.synth(200, 100, 3, seed=60), quality=75)  # no restart markers: host entropy path
    blobs.append(b)
    want.append(np.asarray(Image.open(io.BytesIO(b))))
    b = _jpeg(ikutil.synth(120, 90, 3, seed=61), quality=75, progressive=True, restart_marker_blocks=2)
    blobs.append(b)
    want.append(np.asarray(Image.open(io.BytesIO(b))))
    px = ikutil.synth(40, 30, 4, seed=62)
    buf = io.BytesIO()
    Image.fromarray(px).save(buf, format="PNG")
    blobs.append(buf.getvalue())
    want.append(px)
    out = decode_image_batch(blobs)
    assert len(out) == len(blobs)
    for (img, fmt), w_ in zip(out, want):
        a = img.to_array()
        np.testing.assert_array_equal(a.reshape(w_.shape), w_)
    assert [f for _, f in out][:7] == [ImageFormat.jpeg] * 7 and out[7][1] is None


def test_decode_batch_reports_failures(ik):
    from imagekit import decode_image_batch
    good = _jpeg(ikutil.synth(64, 48, 3, seed=1), quality=80, restart_marker_rows=1)
    with pytest.raises(TransformError):
        decode_image_batch([good, b"\x00" * 10, good])


def test_jpeg_small_scans_counted_where_decoded(ik):
    """Baseline scans of 4 KiB and up go to the self-synchronising GPU decoder
    (counted GPU), smaller ones to the host entropy decoder (counted host): pixels
    equal libjpeg-turbo's either way."""
    c0 = (ctypes.c_ulonglong * 2)()
    ik.ik_jpeg_counters(c0)
    small = _jpeg(ikutil.synth(40, 30, 3, seed=3, pattern="S"), quality=85)
    big = _jpeg(ikutil.synth(700, 500, 3, seed=4, pattern="S"), quality=85)
    assert len(small) < 4096 < len(big)
    for b in (small, big):
        img, _ = decode_image(b)
        np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))
    c1 = (ctypes.c_ulonglong * 2)()
    ik.ik_jpeg_counters(c1)
    assert (c1[0] - c0[0], c1[1] - c0[1]) == (1, 1)


@pytest.mark.parametrize("wh", [(1500, 1100), (2048, 1536), (1001, 999)])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("pat", ["S", "N"])
def test_jpeg_no_restart_self_sync_gpu(ik, wh, sub, pat):
    """Restart-free baseline scans go through the self-synchronising GPU decoder
    (sync pass with warm-up, fix rounds, bases, decode pass -- all on the GPU):
    pixels equal libjpeg-turbo's."""
    w, h = wh
    b = _jpeg(ikutil.synth(w, h, 3, seed=w + sub, pattern=pat), quality=92 if pat == "S" else 60, subsampling=sub)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array(), np.asarray(Image.open(io.BytesIO(b))))


def test_jpeg_no_restart_gray_self_sync(ik):
    g = ikutil.synth(1800, 1200, 1, seed=4, pattern="N")[..., 0]
    b = _jpeg(g, quality=75)
    img, _ = decode_image(b)
    np.testing.assert_array_equal(img.to_array()[..., 0], np.asarray(Image.open(io.BytesIO(b))))

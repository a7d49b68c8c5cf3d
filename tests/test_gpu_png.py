"""GPU: decode_image on PNG through the GPU inflate + unfilter path (ik_png.hip).

Reference: src/transform.rs:31 (image 0.25.8 -> png 0.18, EXPAND).  Bar: the
decoded pixels are identical to Pillow's decoder (libpng + zlib) and to this
library's host decoder, for every colour type the GPU path covers, every filter
type, zlib levels and strategies, multi-IDAT streams, odd sizes, and the 4096^2
RGBA frames of configs[1]; a batch decodes in one set of launches; corrupt
streams give the host decoder's png error."""
import ctypes
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

import ikutil
from imagekit import TransformError, _lib, decode_image, decode_image_batch

pytestmark = pytest.mark.gpu

MODES = {1: "L", 2: "LA", 3: "RGB", 4: "RGBA"}
CTYPE = {1: 0, 2: 4, 3: 2, 4: 6}


def png_counters(ik):
    c = (ctypes.c_ulonglong * 2)()
    assert ik.ik_png_counters(c) == 0
    return c[0], c[1]


@pytest.fixture(scope="module")
def gpu_png(ik):
    assert ik.ik_set_png_gpu_min(0) == 0  # every PNG through the GPU path
    yield ik
    ik.ik_set_png_gpu_min(256 << 10)


@pytest.fixture
def on_gpu(gpu_png):
    """The test's valid PNGs must all be decoded by the GPU path, none by the
    host decoder's fallback (a GPU decoder that rejects a stream still gives
    right pixels through the fallback, so pixel equality alone cannot tell)."""
    g0, h0 = png_counters(gpu_png)
    yield gpu_png
    g1, h1 = png_counters(gpu_png)
    assert g1 > g0, "no PNG stream went through the GPU path"
    assert h1 == h0, f"{h1 - h0} PNG stream(s) fell back to the host decoder"


def pil_png(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img if img.shape[2] > 1 else img[..., 0], MODES[img.shape[2]]).save(b, format="PNG", **kw)
    return b.getvalue()


def chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def own_png(img, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, filters=None, idat_size=None):
    """A PNG with chosen row filters and zlib settings (the encoder side of the test)."""
    h, w, c = img.shape
    rows = []
    prev = np.zeros(w * c, np.int32)
    for y in range(h):
        cur = img[y].reshape(-1).astype(np.int32)
        ft = (y % 5) if filters is None else filters if isinstance(filters, int) else int(filters[y])
        a = np.concatenate([np.zeros(c, np.int32), cur[:-c]])
        b = prev
        cc = np.concatenate([np.zeros(c, np.int32), prev[:-c]])
        if ft == 0:
            f = cur
        elif ft == 1:
            f = cur - a
        elif ft == 2:
            f = cur - b
        elif ft == 3:
            f = cur - ((a + b) >> 1)
        else:
            p = a + b - cc
            pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - cc)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, cc))
            f = cur - pred
        rows.append(bytes([ft]) + (f & 255).astype(np.uint8).tobytes())
        prev = cur
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = co.compress(b"".join(rows)) + co.flush()
    ihdr = struct.pack(">IIBBBBB", w, h, 8, CTYPE[c], 0, 0, 0)
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr)
    step = idat_size or len(z)
    for i in range(0, len(z), step):
        out += chunk(b"IDAT", z[i:i + step])
    return out + chunk(b"IEND", b"")


def decode_px(data):
    img, fmt = decode_image(data)
    assert fmt is None
    return img.to_array()


def pil_px(data):
    im = Image.open(io.BytesIO(data))
    a = np.asarray(im)
    return a[..., None] if a.ndim == 2 else a


@pytest.mark.parametrize("c", [1, 2, 3, 4])
@pytest.mark.parametrize("w,h", [(1, 1), (17, 9), (640, 480), (1001, 333)])
def test_pillow_pngs(on_gpu, c, w, h):
    img = ikutil.synth(w, h, c, seed=w * 7 + c)
    data = pil_png(img)
    np.testing.assert_array_equal(decode_px(data), img)


@pytest.mark.parametrize("level,strategy", [(1, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_DEFAULT_STRATEGY),
                                            (9, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FILTERED),
                                            (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE), (6, zlib.Z_FIXED),
                                            (0, zlib.Z_DEFAULT_STRATEGY)])
def test_all_filters_levels_strategies(on_gpu, level, strategy):
    img = ikutil.synth(777, 401, 4, seed=level * 10 + strategy)
    data = own_png(img, level=level, strategy=strategy, idat_size=8192)
    np.testing.assert_array_equal(decode_px(data), img)
    np.testing.assert_array_equal(pil_px(data), img)


@pytest.mark.parametrize("ft", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("c", [1, 3, 4])
def test_each_filter_type(on_gpu, ft, c):
    img = ikutil.synth(333, 130, c, seed=ft + 10 * c, pattern="N" if ft == 4 else "S")
    data = own_png(img, filters=ft)
    np.testing.assert_array_equal(decode_px(data), img)


def test_noise_and_host_decoder_agree(gpu_png):
    img = ikutil.synth(1500, 700, 4, seed=3, pattern="N")
    data = pil_png(img)
    gpu = decode_px(data)
    gpu_png.ik_set_png_gpu_min(-1)
    try:
        host = decode_px(data)
    finally:
        gpu_png.ik_set_png_gpu_min(0)
    np.testing.assert_array_equal(gpu, img)
    np.testing.assert_array_equal(host, img)


def test_configs1_frame_4096(on_gpu):
    """configs[1]: a 4096x4096 RGBA8 synthetic frame as PNG (35 MB, ~2,000 decoder lanes)."""
    img = ikutil.synth(4096, 4096, 4, seed=1)
    data = pil_png(img)
    np.testing.assert_array_equal(decode_px(data), img)


def test_batch_tall_band_groups(on_gpu):
    """Unfilter across workgroups: images taller than one 16-band group (1,024
    rows), so band 16k waits on band 16k-1 of another workgroup; every filter
    type (rows cycle through 0-4), several bytes-per-pixel classes in one batch,
    heights off the 64-row band grid."""
    shapes = [(300, 2500, 4), (517, 1100, 3), (64, 4100, 1), (1000, 1090, 4), (211, 3333, 2), (90, 2049, 4)]
    imgs = [ikutil.synth(w, h, c, seed=50 + k, pattern="N" if k % 2 else "S") for k, (w, h, c) in enumerate(shapes)]
    datas = [own_png(im, idat_size=65536) for im in imgs]
    out = decode_image_batch(datas)
    for (d, fmt), im in zip(out, imgs):
        np.testing.assert_array_equal(d.to_array().reshape(im.shape), im)


def test_unfilter_scan_path_batch(on_gpu):
    """k_png_unfilter_su (RGBA8 images of None / Sub / Up rows: segments of a None
    or Sub row and the Up rows under it) beside the diagonal kernel in one batch:
    Up runs crossing the workgroups' row slices, an image that is one segment (Up
    from row 0), Sub-only and None-only images, the widest scan-path row (4,096
    pixels: 1,024 chunks) and one pixel wider, and images with Average /
    Paeth rows (diagonal); rows of 4,097 ... 8,192 pixels take the wide scan kernel
    (8 chunks per thread), 8,193 the diagonal one."""
    rnd = np.random.default_rng(5)
    cases = [
        ((4096, 300, 4), rnd.choice([1, 2, 2, 2, 2, 2, 2, 0], 300)),
        ((1000, 2000, 4), np.where(rnd.random(2000) < 0.02, 1, 2)),
        ((777, 1500, 4), np.full(1500, 2)),
        ((512, 700, 4), np.full(700, 1)),
        ((333, 257, 4), np.full(257, 0)),
        ((4097, 64, 4), rnd.choice([1, 2], 64)),
        ((640, 900, 4), rnd.choice([1, 2, 3, 4], 900)),
        ((901, 333, 3), rnd.choice([1, 2], 333)),
        ((1234, 1111, 4), np.concatenate([np.full(1110, 2), [4]])),
        ((8192, 40, 4), rnd.choice([1, 2, 2, 2, 0], 40)),   # the wide scan-path kernel (2,048 chunks)
        ((6000, 33, 4), np.where(np.arange(33) % 11 == 0, 1, 2)),
        ((8193, 9, 4), rnd.choice([1, 2], 9)),               # one pixel wider: diagonal
    ]
    imgs = [ikutil.synth(w, h, c, seed=70 + k, pattern="N" if k % 2 else "S") for k, ((w, h, c), _) in enumerate(cases)]
    datas = [own_png(im, filters=f, idat_size=65536) for im, (_, f) in zip(imgs, cases)]
    out = decode_image_batch(datas)
    for (d, fmt), im in zip(out, imgs):
        np.testing.assert_array_equal(d.to_array().reshape(im.shape), im)


def test_flat_images_markers_through_every_unit(on_gpu):
    """A flat image is runs of copies across every unit boundary: window markers fill
    its rows (chains through every earlier unit) -- beside a normal frame.  (With
    IK_PNG_DIRECT=1 the direct-rows expand's marker list overflows here and the batch
    takes the resolve pass after all; tests/test_gpu_png_direct.py runs that.)"""
    flat = np.zeros((2048, 2048, 4), np.uint8)
    flat[..., 0] = 200
    flat[..., 3] = 255
    img = ikutil.synth(1024, 768, 4, seed=91, pattern="S")
    datas = [own_png(flat, filters=0, idat_size=65536), pil_png(img), own_png(flat[:300], filters=2)]
    out = decode_image_batch(datas)
    for (d, fmt), im in zip(out, [flat, img, flat[:300]]):
        np.testing.assert_array_equal(d.to_array().reshape(im.shape), im)


def test_batch_mixed(on_gpu):
    imgs = [ikutil.synth(w, h, c, seed=k) for k, (w, h, c) in
            enumerate([(640, 480, 4), (1024, 768, 3), (333, 222, 1), (2048, 1024, 4), (100, 3000, 2)])]
    datas = [pil_png(im) for im in imgs] + [own_png(imgs[0], level=9, idat_size=1000)]
    out = decode_image_batch(datas)
    for (d, fmt), im in zip(out, imgs + [imgs[0]]):
        assert fmt is None
        np.testing.assert_array_equal(d.to_array(), im)


def test_corrupt_png_errors(gpu_png):
    img = ikutil.synth(640, 480, 4, seed=4)
    data = bytearray(pil_png(img))
    data[len(data) // 2] ^= 0x40  # inside IDAT: CRC mismatch
    with pytest.raises(TransformError) as ei:
        decode_image(bytes(data))
    assert "Png" in str(ei.value) or "CRC" in str(ei.value)
    # consistent CRC, corrupt deflate data: the GPU rejects it, the host decoder reports it
    good = own_png(img, level=6)
    pos = good.index(b"IDAT")
    ln = struct.unpack(">I", good[pos - 4:pos])[0]
    z = bytearray(good[pos + 4:pos + 4 + ln])
    z[len(z) // 3] ^= 0xFF
    bad = good[:pos - 4] + chunk(b"IDAT", bytes(z)) + chunk(b"IEND", b"")
    try:
        got = decode_px(bad)
    except TransformError:
        return
    with pytest.raises(Exception):  # if anything decoded, it must not claim to be the original
        np.testing.assert_array_equal(got, img)


def test_transform_from_png_bytes(on_gpu, oracle):
    """decode (GPU PNG) -> resize_image -> encode_image: bytes equal the oracle's
    transform of the same pixels (configs[1] shape, reduced size)."""
    from imagekit import ImageFormat
    from imagekit.transform import transform
    img = ikutil.synth(1024, 1024, 4, seed=8)
    data = pil_png(img)
    got = transform(data, 128, 128, ImageFormat.webp, 80, filter=1)
    want, dims = oracle.transform(img, 128, 128, 1, 1, 80)
    assert dims == (128, 128) and got == want


def test_gpu_crc_check_in_batch(gpu_png):
    """The upload's GPU gather pass checks every IDAT CRC (png 0.18 verifies them):
    in one batch, a payload byte flipped in the second IDAT chunk and a stored CRC
    flipped in the last one each give png's CRC error for that stream only (the
    host decoder reports it); the intact streams decode on the GPU."""
    imgs = [ikutil.synth(700, 300 + 50 * k, 4, seed=70 + k, pattern="N" if k % 2 else "S") for k in range(4)]
    datas = [own_png(im, idat_size=20000) for im in imgs]
    bad_payload = bytearray(datas[1])
    p = bad_payload.index(b"IDAT")
    p = bad_payload.index(b"IDAT", p + 4)  # the second IDAT chunk
    bad_payload[p + 4 + 777] ^= 0x01
    bad_crc = bytearray(datas[3])
    q = bad_crc.rindex(b"IDAT")
    ln = struct.unpack(">I", bad_crc[q - 4:q])[0]
    bad_crc[q + 4 + ln + 1] ^= 0x80
    batch = [datas[0], bytes(bad_payload), datas[2], bytes(bad_crc)]
    lib = _lib.load()
    n = len(batch)
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in batch])
    lens = (ctypes.c_size_t * n)(*[len(b) for b in batch])
    outs = (ctypes.c_void_p * n)()
    fmts = (ctypes.c_int * n)()
    status = (ctypes.c_int * n)()
    g0, h0 = png_counters(gpu_png)
    rc = lib.ik_decode_batch(ptrs, lens, n, outs, fmts, status)
    g1, h1 = png_counters(gpu_png)
    assert rc != 0 and "crc" in _lib.last_error().lower()
    assert [status[i] != 0 for i in range(n)] == [False, True, False, True]
    assert (g1 - g0, h1 - h0) == (2, 2)
    from imagekit.transform import DynamicImage
    for i in (0, 2):
        np.testing.assert_array_equal(DynamicImage(outs[i]).to_array(), imgs[i])


def test_pinned_inputs_equal_pageable(on_gpu):
    """Inputs in page-locked memory (ik_host_alloc, DMAed in place) and in
    ordinary memory (staged) give the same bytes through transform_batch."""
    from imagekit import ImageFormat, PinnedBytes, transform_batch
    imgs = [ikutil.synth(1200, 900, c, seed=90 + c) for c in (3, 4)]
    datas = [pil_png(im) for im in imgs]
    pinned = [PinnedBytes(d) for d in datas]
    assert [p.tobytes() for p in pinned] == datas
    sizes, fmts, qs = [(300, None)] * 2, [ImageFormat.webp, ImageFormat.jpeg], [80, 85]
    a = transform_batch(datas, sizes, fmts, qs, filter=1)
    b = transform_batch(pinned, sizes, fmts, qs, filter=1)
    c = transform_batch([pinned[0], datas[1]], sizes, fmts, qs, filter=1)
    assert a == b == c


def _pack_rows(samples, depth):
    """(h, w) samples < 2^depth -> packed PNG rows (MSB first), filter byte 0 or 1..4 cycling."""
    h, w = samples.shape
    per = 8 // depth
    rows = []
    for y in range(h):
        v = samples[y].astype(np.int64)
        if depth < 8:
            pad = (-w) % per
            v = np.concatenate([v, np.zeros(pad, np.int64)]).reshape(-1, per)
            shifts = np.array([8 - depth * (k + 1) for k in range(per)])
            row = (v << shifts).sum(1).astype(np.uint8)
        else:
            row = v.astype(np.uint8)
        rows.append(row)
    return rows


def expand_png(samples, depth, ctype, plte=None, trns=None, level=6):
    """A PNG of gray / palette / RGB samples at `depth` bits with optional PLTE / tRNS;
    rows cycle through the five filter types (bpp = 1 byte below 8 bits)."""
    if ctype == 2:
        h, w, _ = samples.shape
        raw_rows = [samples[y].reshape(-1).astype(np.uint8) for y in range(h)]
        bpp = 3
    else:
        h, w = samples.shape
        raw_rows = _pack_rows(samples, depth)
        bpp = 1
    out_rows, prev = [], np.zeros(len(raw_rows[0]), np.int32)
    for y, r in enumerate(raw_rows):
        cur = r.astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        ft = y % 5
        if ft == 0:
            f = cur
        elif ft == 1:
            f = cur - a
        elif ft == 2:
            f = cur - prev
        elif ft == 3:
            f = cur - ((a + prev) >> 1)
        else:
            p = a + prev - c
            pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - c)
            f = cur - np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
        out_rows.append(bytes([ft]) + (f & 255).astype(np.uint8).tobytes())
        prev = cur
    z = zlib.compress(b"".join(out_rows), level)
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    if plte is not None:
        out += chunk(b"PLTE", plte)
    if trns is not None:
        out += chunk(b"tRNS", trns)
    for i in range(0, len(z), 30000):
        out += chunk(b"IDAT", z[i:i + 30000])
    return out + chunk(b"IEND", b"")


EXPAND_CASES = [("P", 8, False), ("P", 8, True), ("P", 4, False), ("P", 4, True), ("P", 2, True), ("P", 1, False),
                ("L", 1, False), ("L", 2, False), ("L", 4, False), ("L", 8, True), ("L", 4, True), ("L", 1, True),
                ("RGB", 8, True)]


@pytest.mark.parametrize("kind,depth,with_trns", EXPAND_CASES)
@pytest.mark.parametrize("w,h", [(333, 77), (1001, 300)])
def test_expand_on_gpu(gpu_png, kind, depth, with_trns, w, h):
    """png's EXPAND on the GPU path (k_png_px): palette -> RGB / RGBA, gray below 8
    bits -> 8 bits, tRNS -> alpha; pixels equal the EXPAND rule and the host decoder."""
    rng = np.random.default_rng(w * 131 + depth * 7 + with_trns)
    if kind == "P":
        npal = min(1 << depth, 200 if depth == 8 else 1 << depth)
        pal = rng.integers(0, 256, (npal, 3), dtype=np.uint8)
        idx = rng.integers(0, min(1 << depth, npal + 3), (h, w)).astype(np.uint8)  # a few indices past the palette
        trns = rng.integers(0, 256, max(1, npal // 2), dtype=np.uint8) if with_trns else None
        data = expand_png(idx, depth, 3, plte=pal.tobytes(), trns=None if trns is None else trns.tobytes())
        big = np.zeros((256, 3), np.uint8)
        big[:npal] = pal
        want = big[idx]
        if trns is not None:
            alpha = np.full(256, 255, np.uint8)
            alpha[:len(trns)] = trns
            want = np.concatenate([want, alpha[idx][..., None]], -1)
    elif kind == "L":
        v = rng.integers(0, 1 << depth, (h, w)).astype(np.uint8)
        key = int(v[3, 5])
        data = expand_png(v, depth, 0, trns=struct.pack(">H", key) if with_trns else None)
        g = (v.astype(np.int32) * {1: 255, 2: 85, 4: 17, 8: 1}[depth]).astype(np.uint8)
        want = g[..., None]
        if with_trns:
            want = np.concatenate([want, np.where(v == key, 0, 255).astype(np.uint8)[..., None]], -1)
    else:
        px = rng.integers(0, 4, (h, w, 3)).astype(np.uint8) * 60  # few colours: the key hits often
        key = px[2, 2]
        data = expand_png(px, 8, 2, trns=struct.pack(">HHH", *[int(k) for k in key]))
        want = np.concatenate([px, np.where((px == key).all(-1), 0, 255).astype(np.uint8)[..., None]], -1)
    g0, h0 = png_counters(gpu_png)
    got = decode_px(data)
    g1, h1 = png_counters(gpu_png)
    assert (g1 - g0, h1 - h0) == (1, 0), "the stream must decode on the GPU path"
    np.testing.assert_array_equal(got, want)
    gpu_png.ik_set_png_gpu_min(-1)
    try:
        host = decode_px(data)
    finally:
        gpu_png.ik_set_png_gpu_min(0)
    np.testing.assert_array_equal(host, want)


def test_pillow_palette_pngs(on_gpu):
    """Pillow's own palette PNGs (P mode, with and without transparency) through the GPU path."""
    rng = np.random.default_rng(5)
    idx = rng.integers(0, 60, (480, 640)).astype(np.uint8)
    im = Image.fromarray(idx, "P")
    im.putpalette(rng.integers(0, 256, 768, dtype=np.uint8).tobytes())
    for kw in ({}, {"transparency": 7}, {"transparency": bytes(range(0, 240, 4))}):
        b = io.BytesIO()
        im.save(b, format="PNG", **kw)
        data = b.getvalue()
        want = np.asarray(Image.open(io.BytesIO(data)).convert("RGBA" if kw else "RGB"))
        np.testing.assert_array_equal(decode_px(data), want)

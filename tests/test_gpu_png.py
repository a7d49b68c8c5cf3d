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
        ft = (y % 5) if filters is None else filters
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

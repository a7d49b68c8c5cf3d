"""GPU: 16-bit PNG.  png 0.18 + image 0.25.8 decode 16-bit
streams to Rgb16 / Rgba16 / L16 / La16 (EXPAND adds tRNS alpha, keeps 16 bits);
resize_image resamples the u16 samples with the u8 path's f32 sequence, clamped
to 65535 (reference src/transform.rs:31,85-89); encode_image's to_rgb8 / to_rgba8
rescale to 8 bits first (:123,131,140) -- here (v + 128) / 257, image's rounding
u16 -> u8 conversion as restated (parity unpinned).  Limits are
decoded BYTES (image's max_alloc, 512 MiB): a 16-bit image counts twice."""
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

import ikutil
import oracle_np
from imagekit import DynamicImage, FilterType, ImageFormat, TransformError, decode_image, encode_image

pytestmark = pytest.mark.gpu
CTYPE = {1: 0, 2: 4, 3: 2, 4: 6}


def chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def png16(img, trns=None, filt=None):
    """A 16-bit PNG of an (H, W, C) uint16 array; row filters cycle through 0..4."""
    h, w, c = img.shape
    be = img.astype(">u2").view(np.uint8).reshape(h, w * c * 2).astype(np.int32)
    rows, prev, bpp = [], np.zeros(w * c * 2, np.int32), 2 * c
    for y in range(h):
        cur = be[y]
        ft = (y % 5) if filt is None else filt
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        b = prev
        cc = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
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
            f = cur - np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, cc))
        rows.append(bytes([ft]) + (f & 255).astype(np.uint8).tobytes())
        prev = cur
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, CTYPE[c], 0, 0, 0))
    if trns is not None:
        out += chunk(b"tRNS", struct.pack(">" + "H" * len(trns), *trns))
    return out + chunk(b"IDAT", zlib.compress(b"".join(rows), 6)) + chunk(b"IEND", b"")


def synth16(w, h, c, seed):
    r = ikutil.splitmix64(0x16B17 + seed, w * h * c).reshape(h, w, c)
    return (r & np.uint64(0xFFFF)).astype(np.uint16)


@pytest.mark.parametrize("c", [1, 2, 3, 4])
@pytest.mark.parametrize("w,h", [(1, 1), (37, 19), (640, 480)])
def test_decode_16bit(ik, c, w, h):
    img = synth16(w, h, c, seed=w + c)
    d, fmt = decode_image(png16(img))
    assert fmt is None and d.depth == 2 and d.color() == {1: "L16", 2: "La16", 3: "Rgb16", 4: "Rgba16"}[c]
    np.testing.assert_array_equal(d.to_array(), img)


def test_decode_16bit_pillow_gray(ik):
    """A 16-bit gray PNG written by Pillow ("I;16"), decoded to L16."""
    img = synth16(301, 77, 1, seed=9)[..., 0]
    b = io.BytesIO()
    Image.fromarray(img, "I;16").save(b, format="PNG")
    d, _ = decode_image(b.getvalue())
    np.testing.assert_array_equal(d.to_array()[..., 0], img)


@pytest.mark.parametrize("c", [1, 3])
def test_decode_16bit_trns_expands_alpha(ik, c):
    img = synth16(64, 40, c, seed=3)
    key = tuple(int(v) for v in img[5, 7])
    img[20, :] = key  # a row of the transparent colour
    d, _ = decode_image(png16(img, trns=key))
    got = d.to_array()
    assert got.shape == (40, 64, c + 1)
    np.testing.assert_array_equal(got[..., :c], img)
    want_a = np.where((img == np.array(key, np.uint16)).all(-1), 0, 65535)
    np.testing.assert_array_equal(got[..., c], want_a)


@pytest.mark.parametrize("c", [1, 2, 3, 4])
@pytest.mark.parametrize("f", [FilterType.Nearest, FilterType.Triangle, FilterType.Lanczos3], ids=lambda f: f.name)
@pytest.mark.parametrize("geom", [((97, 61), (32, 20)), ((40, 30), (123, 77)), ((640, 480), (200, 150))],
                         ids=lambda g: f"{g[0][0]}x{g[0][1]}-{g[1][0]}x{g[1][1]}")
def test_resize_16bit_matches_restatement(ik, c, f, geom):
    (W, H), (nw, nh) = geom
    src = synth16(W, H, c, seed=W + int(f))
    got = DynamicImage.from_array(src).resize(nw, nh, f)
    assert got.depth == 2
    np.testing.assert_array_equal(got.to_array(), oracle_np.resize(src, nw, nh, int(f)))


def _to8(a):
    return ((a.astype(np.uint32) + 128) // 257).astype(np.uint8)


@pytest.mark.parametrize("c", [3, 4])
def test_encode_16bit_rescales_like_to_rgb8(ik, oracle, c):
    src = synth16(96, 64, c, seed=11)
    d = DynamicImage.from_array(src)
    for fmt, enc in ((ImageFormat.webp, lambda rgb: oracle.webp_encode_rgb(rgb, 80.0)),
                     (ImageFormat.jpeg, lambda rgb: oracle.jpeg_encode_rgb(rgb, 80))):
        assert encode_image(d, fmt, 80) == enc(oracle.to_rgb8(_to8(src)))


def test_transform_from_16bit_png(ik, oracle):
    """16-bit PNG -> resize_image (u16) -> WebP: bytes equal the restated chain."""
    from imagekit.transform import transform
    src = synth16(320, 240, 4, seed=12)
    got = transform(png16(src), 160, None, ImageFormat.webp, 75, filter=4)
    small = oracle_np.resize(src, 160, 120, 4)
    assert got == oracle.webp_encode_rgb(oracle.to_rgb8(_to8(small)), 75.0)


def test_limits_count_decoded_bytes(ik):
    """max_alloc is bytes: 16-bit RGBA at 8 bytes per pixel over 512 MiB fails with
    image's Limits error, while the same pixel count fits at 8 bits."""
    w, h = 16384, 4200  # 68.8 M pixels: 550 MB as Rgba16, 275 MB as Rgba8
    hdr16 = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, 6, 0, 0, 0))
    bad = hdr16 + chunk(b"IDAT", zlib.compress(b"\x00" * 64)) + chunk(b"IEND", b"")
    with pytest.raises(TransformError, match="Limits"):
        decode_image(bad)


@pytest.mark.parametrize("c,trns", [(1, None), (2, None), (3, None), (4, None), (1, "key"), (3, "key")])
def test_16bit_decodes_on_the_gpu(ik, c, trns):
    """16-bit streams above the GPU threshold go through the GPU inflate + unfilter
    and k_png_px (byte order, tRNS alpha), not the host decoder."""
    import ctypes
    img = synth16(640, 480, c, seed=40 + c)
    key = None
    if trns:
        key = tuple(int(v) for v in img[7, 9])
        img[100:140, :] = key
    c0 = (ctypes.c_ulonglong * 2)()
    ik.ik_png_counters(c0)
    d, _ = decode_image(png16(img, trns=key))
    c1 = (ctypes.c_ulonglong * 2)()
    ik.ik_png_counters(c1)
    assert (c1[0] - c0[0], c1[1] - c0[1]) == (1, 0), "the 16-bit stream must decode on the GPU"
    got = d.to_array()
    assert d.depth == 2
    np.testing.assert_array_equal(got[..., :c], img)
    if key is not None:
        want_a = np.where((img == np.array(key, np.uint16)).all(-1), 0, 65535)
        np.testing.assert_array_equal(got[..., c], want_a)

"""CPU: the GPU PNG decoder's parallel-inflate algorithm, run by its CPU model
(rust-image-transform_amd/lib/libik_pngmodel.so: the same ik_inflate.h decoder
core and ik_png_plan.h chain check the GPU path uses), against zlib.

decode_image on a PNG (reference src/transform.rs:31 -> png 0.18) inflates the
IDAT zlib stream; the GPU path decodes it from block-start candidates in
parallel.  Bar: bytes identical to zlib.decompress for every stream shape zlib
produces (dynamic, fixed and stored blocks; all levels and strategies), plus a
stream with a planted false candidate that the chain check must drop."""
import ctypes
import io
import os
import struct
import zlib

import numpy as np
import pytest

import ikutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = os.path.join(ROOT, "rust-image-transform_amd", "lib", "libik_pngmodel.so")


@pytest.fixture(scope="module")
def model():
    if not os.path.exists(MODEL):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "rust-image-transform_amd"), "lib/libik_pngmodel.so"],
                       check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(MODEL)
    L.ikm_inflate_chunked.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]
    L.ikm_plausible_dynamic.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]
    return L


def inflate(model, z, raw_len, chunk):
    out = np.zeros(raw_len + 16, np.uint8)
    n = ctypes.c_uint64()
    st = (ctypes.c_int * 10)()
    rc = model.ikm_inflate_chunked(z, len(z), chunk, out.ctypes.data, raw_len, ctypes.byref(n), st)
    return rc, bytes(out[:n.value]), list(st)


def filtered(img):
    h = img.shape[0]
    ft = np.arange(h) % 5  # all five filter types, raw bytes left unfiltered (still a valid zlib payload)
    return b"".join(bytes([int(ft[y])]) + img[y].tobytes() for y in range(h))


CASES = [
    (256, 256, 4, "S", 6, zlib.Z_DEFAULT_STRATEGY),
    (640, 480, 3, "S", 6, zlib.Z_DEFAULT_STRATEGY),
    (300, 200, 4, "N", 6, zlib.Z_DEFAULT_STRATEGY),   # noise: stored blocks mixed in
    (512, 384, 4, "S", 9, zlib.Z_DEFAULT_STRATEGY),
    (777, 333, 1, "S", 1, zlib.Z_DEFAULT_STRATEGY),
    (500, 300, 2, "S", 6, zlib.Z_FILTERED),
    (500, 300, 4, "S", 6, zlib.Z_HUFFMAN_ONLY),
    (500, 300, 4, "S", 6, zlib.Z_RLE),
    (400, 300, 3, "S", 6, zlib.Z_FIXED),              # fixed-code blocks: no candidates, one lane
    (600, 400, 4, "S", 0, zlib.Z_DEFAULT_STRATEGY),   # stored only
]


@pytest.mark.parametrize("w,h,c,pat,level,strategy", CASES)
@pytest.mark.parametrize("chunk", [4096, 16384])
def test_chunked_inflate_equals_zlib(model, w, h, c, pat, level, strategy, chunk):
    raw = filtered(ikutil.synth(w, h, c, seed=w + h, pattern=pat))
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = co.compress(raw) + co.flush()
    rc, out, st = inflate(model, z, len(raw), chunk)
    assert rc == 0, st
    assert out == raw


def _idat(png):
    pos, out = 8, b""
    while pos < len(png):
        ln = struct.unpack(">I", png[pos:pos + 4])[0]
        if png[pos + 4:pos + 8] == b"IDAT":
            out += png[pos + 8:pos + 8 + ln]
        pos += 12 + ln
    return out


@pytest.mark.parametrize("mode,c", [("RGBA", 4), ("RGB", 3), ("L", 1), ("LA", 2)])
def test_pillow_png_streams(model, mode, c):
    from PIL import Image
    img = ikutil.synth(1024, 512, c, seed=5)
    b = io.BytesIO()
    Image.fromarray(img if c > 1 else img[..., 0], mode).save(b, format="PNG")
    z = _idat(b.getvalue())
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw
    chunks, cands, lanes, rounds = st[:4]
    assert lanes >= 8 and rounds == 1  # many parallel decoders, no false candidate on real data


def test_false_candidate_is_dropped(model):
    """A stored block whose payload is a valid-looking dynamic block header: the
    finder takes it as a block start, the chain check must discard it and the
    predecessor must decode through it."""
    base = zlib.compressobj(6, zlib.DEFLATED, -15)
    hdr_src = base.compress(ikutil.synth(64, 64, 4, seed=1).tobytes()) + base.flush()
    # hdr_src begins with a genuine dynamic block header (BFINAL=1): use its first 200 bytes as bait
    bait = hdr_src[:200]
    assert model.ikm_plausible_dynamic(bait, len(bait), 0) == 1
    payload = bait * 40 + bytes(range(256)) * 64
    co = zlib.compressobj(0, zlib.DEFLATED, 15)  # stored blocks only: the bait sits verbatim in the stream
    z = co.compress(payload) + co.flush()
    # prepend a dynamic-coded part so that the stream has real candidates too
    co2 = zlib.compressobj(6, zlib.DEFLATED, 15)
    mixed_raw = ikutil.synth(200, 200, 4, seed=2).tobytes() + payload
    z2 = co2.compress(ikutil.synth(200, 200, 4, seed=2).tobytes()) + co2.flush(zlib.Z_FULL_FLUSH)
    co3 = zlib.compressobj(0, zlib.DEFLATED, -15)
    z2 = z2 + co3.compress(payload) + co3.flush()
    for stream, raw in ((z, payload), (z2, mixed_raw)):
        rc, out, st = inflate(model, stream, len(raw), 4096)
        assert rc == 0 and out == raw, st
    assert st[5] >= 1  # at least one candidate dropped by the chain check


def test_corrupt_stream_is_rejected(model):
    raw = filtered(ikutil.synth(256, 256, 4, seed=3))
    z = bytearray(zlib.compress(raw, 6))
    z[len(z) // 2] ^= 0x5A
    rc, out, st = inflate(model, bytes(z), len(raw), 4096)
    assert rc != 0 or out != raw  # never a silent "success" with the original bytes
    if rc == 0:
        with pytest.raises(zlib.error):
            zlib.decompress(bytes(z))


def test_deep_marker_chain(model):
    """A smooth RGBA image with row filters cycling 0-4: long matches carry bytes
    back through the window of every earlier decoder, so resolving a byte can
    take more hops than any fixed bound (a byte hops at most once per decoder).
    It once fell to the host decoder at 64 hops; the bound is now the lane count."""
    from test_gpu_png import own_png
    img = ikutil.synth(300, 2500, 4, seed=50, pattern="S")
    z = _idat(own_png(img, idat_size=65536))
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    assert st[2] > 64  # more decoders than the old hop bound


def test_unfilter_word_equals_bytewise_definition():
    """ik_unfilter.h's word-at-a-time row filters (the GPU unfilter for 4- and
    8-byte pixels) against png's byte-wise Sub / Up / Average / Paeth, over every
    (a, b, c) byte triple and every filter type."""
    L = ctypes.CDLL(MODEL)
    L.ikm_unfilter_word_check.restype = ctypes.c_long
    assert L.ikm_unfilter_word_check() == 0


def test_block_search_kraft_sum_equals_definition():
    """cl_kraft_top (k_png_find's Kraft test, absent lengths shifted out) equals the
    plain sum of 2^(7 - len) over a header's ncode code-length-code lengths."""
    L = ctypes.CDLL(MODEL)
    L.ikm_cl_kraft_check.restype = ctypes.c_long
    L.ikm_cl_kraft_check.argtypes = [ctypes.c_long]
    assert L.ikm_cl_kraft_check(200000) == 0


"""CPU: the GPU PNG upload's gather pass (ik_png.hip k_png_gather + k_png_crc_check),
run by its CPU model (libik_pngmodel.so: the same ik_png_gather.h plan and ik_crc.h
CRC algebra the kernels use), against zlib.

decode_image on a PNG (reference src/transform.rs:31 -> png 0.18) verifies every
chunk's CRC-32 and inflates the concatenated IDAT payloads.  The upload DMAs whole
files and the GPU assembles the zlib stream and checks the IDAT CRCs, so the
bar is: the assembled stream equals the concatenated payloads (zlib inflates
it to the image's filtered rows), every CRC of an intact file passes, and a
flipped byte in any IDAT payload or stored CRC fails exactly that chunk."""
import ctypes
import io
import os
import struct
import zlib

import numpy as np
import pytest
from PIL import Image, ImageFile

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
    L.ikm_gather_check.restype = ctypes.c_int
    L.ikm_gather_check.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.ikm_crc32_joined.restype = ctypes.c_uint32
    L.ikm_crc32_joined.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t]
    return L


def _chunks(png: bytes):
    out, pos = [], 8
    while pos + 12 <= len(png):
        n = struct.unpack(">I", png[pos:pos + 4])[0]
        out.append((png[pos + 4:pos + 8], pos + 8, n))
        pos += 12 + n
    return out


def _png_multi_idat(px, chunk):
    """A PNG whose zlib stream is cut into IDAT chunks of `chunk` bytes (libpng-style)."""
    b = io.BytesIO()
    Image.fromarray(px).save(b, format="PNG")
    src = b.getvalue()
    ch = _chunks(src)
    z = b"".join(src[o:o + n] for t, o, n in ch if t == b"IDAT")
    out = bytearray(src[:8])
    for t, o, n in ch:
        if t == b"IDAT":
            continue
        if t == b"IEND":
            for k in range(0, len(z), chunk):
                part = z[k:k + chunk]
                out += struct.pack(">I", len(part)) + b"IDAT" + part + struct.pack(">I", zlib.crc32(b"IDAT" + part))
        out += src[o - 8:o + n + 4]
    return bytes(out), z


def _run(model, png, z_off=0, tail=0):
    zlen = sum(n for t, o, n in _chunks(png) if t == b"IDAT")
    cap = z_off + zlen + tail + 64
    buf = np.full(cap, 0xAB, np.uint8)
    bad = (ctypes.c_int * 4096)()
    n = model.ikm_gather_check(png, len(png), z_off, tail, buf.ctypes.data, cap, bad, 4096)
    return n, bytes(buf[z_off:z_off + zlen]), bytes(buf[z_off + zlen:z_off + zlen + tail]), list(bad[:max(n, 0)])


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 255, 256, 257, 1023, 4096, 65535, 65536, 65537, 200001])
@pytest.mark.parametrize("run", [256, 65536])
def test_joined_crc_equals_zlib(model, n, run):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert model.ikm_crc32_joined(data, n, run) == zlib.crc32(data)


@pytest.mark.parametrize("chunk", [1, 7, 8192, 65535, 65536, 65537, 300000])
@pytest.mark.parametrize("z_off", [0, 1, 2, 3, 256])
def test_gather_assembles_stream_and_passes_crcs(model, chunk, z_off):
    px = ikutil.synth(300, 171, 4, seed=chunk % 97, pattern="N")
    png, z = _png_multi_idat(px, chunk)
    n, got, tail, bad = _run(model, png, z_off=z_off, tail=515)
    assert n == (len(z) + chunk - 1) // chunk
    assert got == z and tail == b"\0" * 515
    assert not any(bad)
    raw = zlib.decompress(got)
    assert len(raw) == (300 * 4 + 1) * 171


def test_pillow_stream_crcs(model):
    px = ikutil.synth(1024, 700, 3, seed=5, pattern="S")
    b = io.BytesIO()
    # Pillow writes one IDAT per MAXBLOCK bytes; other test modules enlarge it
    keep, ImageFile.MAXBLOCK = ImageFile.MAXBLOCK, 65536
    try:
        Image.fromarray(px).save(b, format="PNG")
    finally:
        ImageFile.MAXBLOCK = keep
    png = b.getvalue()
    n, got, _, bad = _run(model, png)
    assert n >= 2 and not any(bad)
    assert zlib.decompress(got)


@pytest.mark.parametrize("where", ["payload_first", "payload_mid", "payload_last_byte", "stored_crc"])
def test_corruption_fails_exactly_that_chunk(model, where):
    px = ikutil.synth(200, 150, 4, seed=3, pattern="N")
    png, z = _png_multi_idat(px, 20000)
    ch = [(t, o, n) for t, o, n in _chunks(png) if t == b"IDAT"]
    k = 1
    t, o, n = ch[k]
    pos = {"payload_first": o, "payload_mid": o + n // 2, "payload_last_byte": o + n - 1, "stored_crc": o + n + 2}[where]
    bad_png = bytearray(png)
    bad_png[pos] ^= 0x10
    cnt, _, _, bad = _run(model, bytes(bad_png))
    assert cnt == len(ch)
    assert bad == [1 if i == k else 0 for i in range(len(ch))]

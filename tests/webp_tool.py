"""libwebp through ctypes -- TEST INFRASTRUCTURE ONLY (the checker of the GPU WebP
decoder, never the product).

decode_rgb(): WebPDecodeRGB, the pixels the GPU decoder (ik_vp8d*.{h,cpp,hip}) must equal.
encode(): WebPEncode with an advanced WebPConfig, to make lossy files that exercise
what the default encoder never writes: several token partitions, the simple loop
filter, filter sharpness, one segment or four, no filter, method 0..6.

Struct offsets are those of WEBP_ENCODER_ABI_VERSION 0x020f (libwebp 1.2.x
encode.h; the system libwebp.so.7 is 1.2.2) -- the same layout oracle/libwebp_ref.c
relies on and checks."""
from __future__ import annotations

import ctypes
import struct

import numpy as np

_ABI = 0x020F
_lib = None

# WebPConfig fields (all 4 bytes), by index
CFG = dict(lossless=0, quality=1, method=2, image_hint=3, target_size=4, target_PSNR=5, segments=6,
           sns_strength=7, filter_strength=8, filter_sharpness=9, filter_type=10, autofilter=11,
           alpha_compression=12, alpha_filtering=13, alpha_quality=14, pass_=15, show_compressed=16,
           preprocessing=17, partitions=18, partition_limit=19)
_PIC_WIDTH, _PIC_HEIGHT, _PIC_WRITER, _PIC_CUSTOM = 8, 12, 96, 104


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL("libwebp.so.7")
        L.WebPConfigInitInternal.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int]
        L.WebPValidateConfig.argtypes = [ctypes.c_void_p]
        L.WebPPictureInitInternal.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.WebPPictureImportRGB.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.WebPPictureFree.argtypes = [ctypes.c_void_p]
        L.WebPMemoryWriterInit.argtypes = [ctypes.c_void_p]
        L.WebPMemoryWriterClear.argtypes = [ctypes.c_void_p]
        L.WebPEncode.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.WebPDecodeRGB.restype = ctypes.c_void_p
        L.WebPDecodeRGB.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
        L.WebPFree.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def decode_rgb(data: bytes) -> np.ndarray:
    L = lib()
    w, h = ctypes.c_int(), ctypes.c_int()
    p = L.WebPDecodeRGB(data, len(data), ctypes.byref(w), ctypes.byref(h))
    if not p:
        raise ValueError("WebPDecodeRGB failed")
    a = np.frombuffer(ctypes.string_at(p, w.value * h.value * 3), np.uint8).reshape(h.value, w.value, 3).copy()
    L.WebPFree(p)
    return a


def encode(rgb: np.ndarray, quality: float = 80.0, **opts) -> bytes:
    """WebPEncode of an RGB image with WebPConfigInit's defaults, quality and opts
    (keys of CFG; pass_ for `pass`)."""
    L = lib()
    rgb = np.ascontiguousarray(rgb)
    h, w, _ = rgb.shape
    cfg = (ctypes.c_int32 * 64)()
    assert L.WebPConfigInitInternal(cfg, 0, float(quality), _ABI)
    for k, v in opts.items():
        cfg[CFG[k]] = int(v)
    assert L.WebPValidateConfig(cfg), f"invalid config {opts}"
    pic = (ctypes.c_uint8 * 512)()
    assert L.WebPPictureInitInternal(pic, _ABI)
    struct.pack_into("<ii", pic, _PIC_WIDTH, w, h)
    assert L.WebPPictureImportRGB(pic, rgb.ctypes.data, 3 * w)
    writer = (ctypes.c_uint8 * 64)()  # WebPMemoryWriter: mem, size, max_size, pad
    L.WebPMemoryWriterInit(writer)
    write_fn = ctypes.cast(L.WebPMemoryWrite, ctypes.c_void_p).value
    struct.pack_into("<QQ", pic, _PIC_WRITER, write_fn, ctypes.addressof(writer))
    ok = L.WebPEncode(cfg, pic)
    mem, size = struct.unpack_from("<QQ", writer, 0)
    out = ctypes.string_at(mem, size) if ok else b""
    L.WebPMemoryWriterClear(writer)
    L.WebPPictureFree(pic)
    assert ok, f"WebPEncode failed {opts}"
    return out


def vp8_frame_info(data: bytes) -> dict:
    """What a simple lossy file's headers say (for the tests' coverage checks):
    token partitions, filter type, level, sharpness, segmentation."""
    assert data[:4] == b"RIFF" and data[8:12] == b"WEBP" and data[12:16] == b"VP8 "
    f = data[20:]
    part0 = (f[0] | f[1] << 8 | f[2] << 16) >> 5
    br = _Bits(f[10:10 + part0])
    br.bit(); br.bit()
    seg = br.bit()
    upd_map = 0
    if seg:
        upd_map = br.bit()
        if br.bit():
            br.bit()
            for _ in range(4):
                if br.bit():
                    br.val(7); br.bit()
            for _ in range(4):
                if br.bit():
                    br.val(6); br.bit()
        if upd_map:
            for _ in range(3):
                if br.bit():
                    br.val(8)
    simple, level, sharp = br.bit(), br.val(6), br.val(3)
    if br.bit() and br.bit():
        for _ in range(8):
            if br.bit():
                br.val(6); br.bit()
    parts = 1 << br.val(2)
    return dict(segments=bool(seg), update_map=bool(upd_map), simple=bool(simple), level=level, sharpness=sharp,
                partitions=parts)


class _Bits:  # RFC 6386 section 7 boolean decoder (probability 1/2 reads only)
    def __init__(self, b: bytes):
        self.b, self.i = b + bytes(8), 2
        self.value, self.range, self.count = (self.b[0] << 8) | self.b[1], 255, 0

    def bit(self, p: int = 128) -> int:
        split = 1 + (((self.range - 1) * p) >> 8)
        big = split << 8
        if self.value >= big:
            r, self.range, self.value = 1, self.range - split, self.value - big
        else:
            r, self.range = 0, split
        while self.range < 128:
            self.value <<= 1
            self.range <<= 1
            self.count += 1
            if self.count == 8:
                self.count = 0
                self.value |= self.b[self.i]
                self.i += 1
        return r

    def val(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

"""Host-side mirror of reference `imagekit::transform` (src/transform.rs).

The same three functions with the same argument meaning and error behaviour:

    decode_image(bytes) -> (DynamicImage, Optional[ImageFormat])       :27-43
    resize_image(img, w: Optional[int], h: Optional[int]) -> DynamicImage  :62-90
    encode_image(img, fmt: ImageFormat, quality: int) -> bytes          :113-150

Every call goes through libimagekit_hip.so (include/imagekit_hip.h): pixels live
in HBM as a device-resident `DynamicImage`; the resampler, the colour
conversions and the FDCT/quantiser are gfx950 kernels.  Failures raise
`TransformError`, as the reference maps every decode/encode failure to
`ImageKitError::TransformError`.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import enum
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from .config import ImageFormat
from .errors import InvalidArgument, TransformError


class FilterType(enum.IntEnum):
    """image::imageops::FilterType (image 0.25.8).  resize_image uses Lanczos3."""

    Nearest = 0
    Triangle = 1
    CatmullRom = 2
    Gaussian = 3
    Lanczos3 = 4


_COLOR = {1: "L8", 2: "La8", 3: "Rgb8", 4: "Rgba8"}


def _raise(status: int, what: str):
    msg = _lib.last_error()
    if status == 2:
        raise InvalidArgument(f"{what}: {msg}")
    raise TransformError(msg)


class DynamicImage:
    """An 8-bit image (L8 / La8 / Rgb8 / Rgba8) resident in device memory."""

    __slots__ = ("_h", "__weakref__")

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def from_array(cls, pixels: np.ndarray) -> "DynamicImage":
        """ImageBuffer::from_raw on an (H, W) or (H, W, C) array: uint8 (L8 / La8 /
        Rgb8 / Rgba8) or uint16 (L16 / La16 / Rgb16 / Rgba16)."""
        wide = np.asarray(pixels).dtype == np.uint16
        a = np.ascontiguousarray(pixels, dtype=np.uint16 if wide else np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        if a.ndim != 3 or not 1 <= a.shape[2] <= 4:
            raise InvalidArgument("expected (H, W, C) uint8 or uint16 with C in 1..4")
        h, w, c = a.shape
        lib = _lib.load()
        out = ctypes.c_void_p()
        st = (lib.ik_image_from_host16 if wide else lib.ik_image_from_host)(a.ctypes.data, w, h, c, ctypes.byref(out))
        if st:
            _raise(st, "from_array")
        return cls(out.value)

    @classmethod
    def new_rgb8(cls, w: int, h: int) -> "DynamicImage":
        """DynamicImage::new_rgb8 (all-zero pixels), as tests/transform.rs builds inputs."""
        return cls.from_array(np.zeros((h, w, 3), np.uint8))

    @classmethod
    def new_rgba8(cls, w: int, h: int) -> "DynamicImage":
        return cls.from_array(np.zeros((h, w, 4), np.uint8))

    def dimensions(self) -> Tuple[int, int]:
        w, h, c = self._info()
        return (w, h)

    def width(self) -> int:
        return self._info()[0]

    def height(self) -> int:
        return self._info()[1]

    @property
    def channels(self) -> int:
        return self._info()[2]

    def color(self) -> str:
        name = _COLOR[self._info()[2]]
        return name.replace("8", "16") if self.depth == 2 else name

    def _info(self):
        lib = _lib.load()
        w, h, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        st = lib.ik_image_info(self._h, ctypes.byref(w), ctypes.byref(h), ctypes.byref(c))
        if st:
            _raise(st, "image_info")
        return w.value, h.value, c.value

    @property
    def depth(self) -> int:
        """Bytes per sample: 1 (8-bit) or 2 (16-bit)."""
        return int(_lib.load().ik_image_depth(self._h))

    def to_array(self) -> np.ndarray:
        """Copy the pixels back to the host as an (H, W, C) array (uint8, or uint16
        for a 16-bit image)."""
        w, h, c = self._info()
        out = np.empty((h, w, c), np.uint16 if self.depth == 2 else np.uint8)
        st = _lib.load().ik_image_to_host(self._h, out.ctypes.data, out.nbytes)
        if st:
            _raise(st, "to_array")
        return out

    def resize(self, nw: int, nh: int, filter: FilterType = FilterType.Lanczos3) -> "DynamicImage":
        """imageops::resize to exactly nw x nh (the resampler under resize_image)."""
        out = ctypes.c_void_p()
        st = _lib.load().ik_resize_exact(self._h, nw, nh, int(filter), ctypes.byref(out))
        if st:
            _raise(st, "resize")
        return DynamicImage(out.value)

    def clone(self) -> "DynamicImage":
        return DynamicImage.from_array(self.to_array())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.ik_image_free(h)
            self._h = ctypes.c_void_p(0)

    def __repr__(self) -> str:
        w, h, c = self._info()
        return f"DynamicImage({_COLOR[c]}, {w}x{h}, device)"


def decode_image(data: bytes) -> Tuple[DynamicImage, Optional[ImageFormat]]:
    """src/transform.rs:27-43 -- guess_format + load_from_memory_with_format."""
    lib = _lib.load()
    b = bytes(data)
    out = ctypes.c_void_p()
    fmt = ctypes.c_int(-1)
    st = lib.ik_decode(b, len(b), ctypes.byref(out), ctypes.byref(fmt))
    if st:
        raise TransformError(_lib.last_error())
    f = None if fmt.value < 0 else ImageFormat(fmt.value)
    return DynamicImage(out.value), f


def decode_image_batch(datas) -> List[Tuple[DynamicImage, Optional[ImageFormat]]]:
    """decode_image over many inputs with one GPU entropy-decoding launch for the
    restart-interval JPEGs among them (ik_decode_batch).  Raises the first failure."""
    lib = _lib.load()
    bufs = [bytes(d) for d in datas]
    n = len(bufs)
    if n == 0:
        return []
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in bufs])
    lens = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
    outs = (ctypes.c_void_p * n)()
    fmts = (ctypes.c_int * n)()
    status = (ctypes.c_int * n)()
    st = lib.ik_decode_batch(ptrs, lens, n, outs, fmts, status)
    imgs = [DynamicImage(outs[i]) if outs[i] else None for i in range(n)]
    if st:
        raise TransformError(_lib.last_error())
    return [(imgs[i], None if fmts[i] < 0 else ImageFormat(fmts[i])) for i in range(n)]


class PinnedBytes:
    """Encoded input bytes in page-locked host memory (ik_host_alloc): the batch
    calls DMA them to the GPU in place, with no staging copy -- what a server does
    by reading request bodies into such buffers.  Accepted wherever the batch
    calls take `bytes`."""

    __slots__ = ("ptr", "len", "__weakref__")

    def __init__(self, data: bytes):
        lib = _lib.load()
        p = ctypes.c_void_p()
        if lib.ik_host_alloc(max(1, len(data)), ctypes.byref(p)) != 0:
            raise TransformError(_lib.last_error())
        ctypes.memmove(p, data, len(data))
        self.ptr, self.len = p.value, len(data)

    def __len__(self) -> int:
        return self.len

    def tobytes(self) -> bytes:
        return ctypes.string_at(self.ptr, self.len)

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                _lib.load().ik_host_free(ctypes.c_void_p(self.ptr))
            except Exception:
                pass
            self.ptr = None


class DeviceBytes:
    """Encoded input bytes in device memory (ik_dev_alloc on the current device):
    request bodies a caller already holds in HBM, for transform_batch_submit_device."""

    __slots__ = ("ptr", "len", "__weakref__")

    def __init__(self, data: bytes):
        lib = _lib.load()
        p = ctypes.c_void_p()
        if lib.ik_dev_alloc(max(1, len(data)), ctypes.byref(p)) != 0:
            raise TransformError(_lib.last_error())
        if len(data) and lib.ik_memcpy_h2d(p, bytes(data), len(data)) != 0:
            lib.ik_dev_free(p)
            raise TransformError(_lib.last_error())
        self.ptr, self.len = p.value, len(data)

    def __len__(self) -> int:
        return self.len

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                _lib.load().ik_dev_free(ctypes.c_void_p(self.ptr))
            except Exception:
                pass
            self.ptr = None


def _inputs(datas):
    """(keep-alive list, pointer array, length array) for a batch call."""
    keep = [d if isinstance(d, PinnedBytes) else bytes(d) for d in datas]
    n = len(keep)
    ptrs = (ctypes.c_void_p * n)(*[d.ptr if isinstance(d, PinnedBytes) else
                                   ctypes.cast(ctypes.c_char_p(d), ctypes.c_void_p).value for d in keep])
    lens = (ctypes.c_size_t * n)(*[len(d) for d in keep])
    return keep, ptrs, lens


def transform_batch(datas, sizes, fmts, qualities, filter: "FilterType" = None, threads: int = 0) -> List[bytes]:
    """ik_transform_batch: decode -> resize_image -> encode_image for many requests
    (sizes: (w, h) per request, None = unset; fmts: ImageFormat per request)."""
    lib = _lib.load()
    bufs, ptrs, lens = _inputs(datas)
    n = len(bufs)
    if n == 0:
        return []
    filt = int(FilterType.Lanczos3 if filter is None else filter)
    ws = (ctypes.c_int64 * n)(*[-1 if s[0] is None else int(s[0]) for s in sizes])
    hs = (ctypes.c_int64 * n)(*[-1 if s[1] is None else int(s[1]) for s in sizes])
    fs = (ctypes.c_int * n)(*[int(f.value if isinstance(f, ImageFormat) else f) for f in fmts])
    qs = (ctypes.c_int * n)(*[int(q) for q in qualities])
    outs = (ctypes.c_void_p * n)()
    olens = (ctypes.c_size_t * n)()
    status = (ctypes.c_int * n)()
    st = lib.ik_transform_batch(ptrs, lens, n, ws, hs, fs, qs, filt, threads, outs, olens, status)
    res = []
    for i in range(n):
        res.append(ctypes.string_at(outs[i], olens[i]) if outs[i] else None)
        if outs[i]:
            lib.ik_buf_free(outs[i])
    if st:
        raise TransformError(_lib.last_error())
    return res


class PendingBatch:
    """A submitted ik_transform_batch_submit: its device half has run; wait() blocks
    until its host coders are done and returns the encoded bytes per request (the
    ctypes arrays the library writes into live here until then)."""

    def __init__(self, keep, outs, olens, status, ticket, n):
        self._keep, self._outs, self._olens, self._status = keep, outs, olens, status
        self._ticket, self._n, self._done = ticket, n, False

    def wait(self) -> List[bytes]:
        if self._done:
            raise InvalidArgument("batch already waited for")
        lib = _lib.load()
        st = lib.ik_transform_batch_wait(self._ticket)
        self._done = True
        res = []
        for i in range(self._n):
            o = self._outs[i]
            res.append(ctypes.string_at(o, self._olens[i]) if o else None)
            if o:
                lib.ik_buf_free(o)
        if st:
            raise TransformError(_lib.last_error())
        return res


def transform_batch_submit(datas, sizes, fmts, qualities, filter: "FilterType" = None,
                           threads: int = 0) -> PendingBatch:
    """ik_transform_batch_submit: the device half of transform_batch now, the host
    coders in the background; PendingBatch.wait() gives what transform_batch gives."""
    lib = _lib.load()
    bufs, ptrs, lens = _inputs(datas)
    n = len(bufs)
    if n == 0:
        raise InvalidArgument("empty batch")
    filt = int(FilterType.Lanczos3 if filter is None else filter)
    ws = (ctypes.c_int64 * n)(*[-1 if s[0] is None else int(s[0]) for s in sizes])
    hs = (ctypes.c_int64 * n)(*[-1 if s[1] is None else int(s[1]) for s in sizes])
    fs = (ctypes.c_int * n)(*[int(f.value if isinstance(f, ImageFormat) else f) for f in fmts])
    qs = (ctypes.c_int * n)(*[int(q) for q in qualities])
    outs = (ctypes.c_void_p * n)()
    olens = (ctypes.c_size_t * n)()
    status = (ctypes.c_int * n)()
    ticket = ctypes.c_uint64()
    st = lib.ik_transform_batch_submit(ptrs, lens, n, ws, hs, fs, qs, filt, threads, outs, olens, status,
                                       ctypes.byref(ticket))
    if st:
        raise TransformError(_lib.last_error())
    return PendingBatch((bufs, ptrs, lens, ws, hs, fs, qs), outs, olens, status, ticket.value, n)


def transform_batch_submit_device(datas, sizes, fmts, qualities, filter: "FilterType" = None,
                                  threads: int = 0) -> PendingBatch:
    """ik_transform_batch_submit_device: as transform_batch_submit, over request
    bodies already in device memory (DeviceBytes)."""
    lib = _lib.load()
    keep = list(datas)
    n = len(keep)
    if n == 0:
        raise InvalidArgument("empty batch")
    if not all(isinstance(d, DeviceBytes) for d in keep):
        raise InvalidArgument("transform_batch_submit_device takes DeviceBytes")
    ptrs = (ctypes.c_void_p * n)(*[d.ptr for d in keep])
    lens = (ctypes.c_size_t * n)(*[len(d) for d in keep])
    filt = int(FilterType.Lanczos3 if filter is None else filter)
    ws = (ctypes.c_int64 * n)(*[-1 if s[0] is None else int(s[0]) for s in sizes])
    hs = (ctypes.c_int64 * n)(*[-1 if s[1] is None else int(s[1]) for s in sizes])
    fs = (ctypes.c_int * n)(*[int(f.value if isinstance(f, ImageFormat) else f) for f in fmts])
    qs = (ctypes.c_int * n)(*[int(q) for q in qualities])
    outs = (ctypes.c_void_p * n)()
    olens = (ctypes.c_size_t * n)()
    status = (ctypes.c_int * n)()
    ticket = ctypes.c_uint64()
    st = lib.ik_transform_batch_submit_device(ptrs, lens, n, ws, hs, fs, qs, filt, threads, outs, olens, status,
                                              ctypes.byref(ticket))
    if st:
        raise TransformError(_lib.last_error())
    return PendingBatch((keep, ptrs, lens, ws, hs, fs, qs), outs, olens, status, ticket.value, n)


def resize_image(img: DynamicImage, w: Optional[int], h: Optional[int],
                 filter: FilterType = FilterType.Lanczos3) -> DynamicImage:
    """src/transform.rs:62-90 (Lanczos3; `filter` is an extension)."""
    if w is None and h is None:
        return img
    for v in (w, h):
        if v is not None and not 0 <= v <= 0xFFFFFFFF:
            raise InvalidArgument("dimension must be a u32")
    out = ctypes.c_void_p()
    st = _lib.load().ik_resize(img._h, -1 if w is None else int(w), -1 if h is None else int(h),
                               int(filter), ctypes.byref(out))
    if st:
        _raise(st, "resize_image")
    return DynamicImage(out.value)


def encode_image(img: DynamicImage, fmt: ImageFormat, quality: int) -> bytes:
    """src/transform.rs:113-150.  quality is a u8, clamped to [1, 100]."""
    if not 0 <= int(quality) <= 255:
        raise InvalidArgument("quality must be a u8")
    lib = _lib.load()
    buf = _lib.u8p()
    n = ctypes.c_size_t()
    st = lib.ik_encode(img._h, ImageFormat(fmt).value, int(quality), ctypes.byref(buf), ctypes.byref(n))
    if st:
        raise TransformError(_lib.last_error())
    try:
        return ctypes.string_at(buf, n.value)
    finally:
        lib.ik_buf_free(buf)


def transform(data: bytes, w: Optional[int], h: Optional[int], fmt: ImageFormat, quality: int,
              filter: FilterType = FilterType.Lanczos3) -> bytes:
    """decode -> resize_image -> encode_image in one device-resident call."""
    lib = _lib.load()
    b = bytes(data)
    buf = _lib.u8p()
    n = ctypes.c_size_t()
    st = lib.ik_transform(b, len(b), -1 if w is None else int(w), -1 if h is None else int(h),
                          ImageFormat(fmt).value, int(quality), int(filter), ctypes.byref(buf),
                          ctypes.byref(n))
    if st:
        raise TransformError(_lib.last_error())
    try:
        return ctypes.string_at(buf, n.value)
    finally:
        lib.ik_buf_free(buf)

"""ctypes binding of libimagekit_hip.so (the C ABI in include/imagekit_hip.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every call raises.  `load()` builds nothing; run `make -C
rust-image-transform_amd` (or `__graft_entry__.build()`) first.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IK_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libimagekit_hip.so")

_lock = threading.Lock()
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
c_img_p = ctypes.c_void_p

# (name, restype, argtypes) for every entry point declared in include/imagekit_hip.h
SIGNATURES = [
    ("ik_init", ctypes.c_int, [ctypes.c_int]),
    ("ik_shutdown", ctypes.c_int, []),
    ("ik_close", ctypes.c_int, []),
    ("ik_memory_stats", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    ("ik_device_count", ctypes.c_int, []),
    ("ik_init_devices", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("ik_logical_device_count", ctypes.c_int, []),
    ("ik_logical_device_stats", ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("ik_request_cost", ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]),
    ("ik_schedule_plan", None, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
    ("ik_schedule_split", ctypes.c_uint32, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    ("ik_last_error", ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t]),
    ("ik_version", ctypes.c_char_p, []),
    ("ik_host_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("ik_host_free", ctypes.c_int, [ctypes.c_void_p]),
    ("ik_host_register", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    ("ik_host_unregister", ctypes.c_int, [ctypes.c_void_p]),
    ("ik_image_from_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(c_img_p)]),
    ("ik_image_wrap_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.POINTER(c_img_p)]),
    ("ik_image_info", ctypes.c_int, [c_img_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    ("ik_image_to_host", ctypes.c_int, [c_img_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("ik_image_depth", ctypes.c_int, [c_img_p]),
    ("ik_image_from_host16", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(c_img_p)]),
    ("ik_image_free", None, [c_img_p]),
    ("ik_buf_free", None, [ctypes.c_void_p]),
    ("ik_decode", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(c_img_p), ctypes.POINTER(ctypes.c_int)]),
    ("ik_resize", ctypes.c_int, [c_img_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(c_img_p)]),
    ("ik_resize_exact", ctypes.c_int, [c_img_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(c_img_p)]),
    ("ik_encode", ctypes.c_int, [c_img_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]),
    ("ik_transform", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]),
    ("ik_set_webp_encoder", ctypes.c_int, [ctypes.c_int]),
    ("ik_libwebp_version", ctypes.c_int, []),
    ("ik_codec_library", ctypes.c_size_t, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    ("ik_get_webp_encoder", ctypes.c_int, []),
    ("ik_pipeline_set_webp_encoder", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("ik_webp_encode_exact_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("ik_vp8_analyze_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]),
    ("ik_pipeline_create", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("ik_pipeline_run", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    ("ik_decode_batch", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("ik_transform_batch", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]),
    ("ik_transform_batch_submit", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)]),
    ("ik_transform_batch_submit_device", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_uint32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)]),
    ("ik_transform_batch_wait", ctypes.c_int, [ctypes.c_uint64]),
    ("ik_set_resize_mode", ctypes.c_int, [ctypes.c_int]),
    ("ik_set_png_gpu_min", ctypes.c_int, [ctypes.c_longlong]),
    ("ik_png_last_timing", ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ("ik_batch_last_timing", ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ("ik_png_counters", ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    ("ik_jpeg_counters", ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    ("ik_get_resize_mode", ctypes.c_int, []),
    ("ik_resize_kernel_name", ctypes.c_char_p, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]),
    ("ik_set_jpeg_reconstruction", ctypes.c_int, [ctypes.c_int]),
    ("ik_get_jpeg_reconstruction", ctypes.c_int, []),
    ("ik_pipeline_submit", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32]),
    ("ik_pipeline_collect", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32)]),
    ("ik_pipeline_run_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32]),
    ("ik_pipeline_kernel_ms", ctypes.c_double, [ctypes.c_void_p, ctypes.c_int]),
    ("ik_pipeline_fetch_resized", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    ("ik_pipeline_destroy", None, [ctypes.c_void_p]),
    ("ik_resize_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]),
    ("ik_webp_yuv420_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    ("ik_jpeg_coeffs_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("ik_dev_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("ik_dev_free", ctypes.c_int, [ctypes.c_void_p]),
    ("ik_memcpy_h2d", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("ik_memcpy_d2h", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("ik_dev_synchronize", ctypes.c_int, []),
]


class LibraryMissing(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} not found: build it with `make -C rust-image-transform_amd` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        # orderly teardown while the HIP runtime is alive (ik_close: callers still
        # inside the library return first, the worker and stage threads end,
        # streams and arenas are released, later calls fail instead of bringing
        # the library back up under daemon threads), not in destructors during
        # process exit
        atexit.register(lib.ik_close)
        return lib


def last_error() -> str:
    lib = load()
    buf = ctypes.create_string_buffer(1024)
    lib.ik_last_error(buf, len(buf))
    return buf.value.decode("utf-8", "replace")

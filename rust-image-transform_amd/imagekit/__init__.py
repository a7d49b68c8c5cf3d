"""imagekit (MI355X-native): drop-in for the reference crate's transform hot path.

Layout mirrors the crate: `imagekit.transform` (src/transform.rs),
`imagekit.config` (src/config.rs), `imagekit.ImageKitError` (src/lib.rs:34-52).
"""
from . import config, transform
from .config import DEFAULT_QUALITY, MAX_QUALITY, MIN_QUALITY, ImageFormat, ImageKitConfig
from .errors import ImageKitError, InvalidArgument, TransformError
from .transform import DeviceBytes, DynamicImage, FilterType, PinnedBytes, decode_image, decode_image_batch, encode_image, resize_image, transform_batch, transform_batch_submit, transform_batch_submit_device

__all__ = [
    "config", "transform", "ImageFormat", "ImageKitConfig", "DEFAULT_QUALITY", "MIN_QUALITY",
    "MAX_QUALITY", "ImageKitError", "TransformError", "InvalidArgument", "DynamicImage",
    "FilterType", "decode_image", "decode_image_batch", "encode_image", "resize_image", "transform_batch",
    "transform_batch_submit", "transform_batch_submit_device", "PinnedBytes", "DeviceBytes",
]

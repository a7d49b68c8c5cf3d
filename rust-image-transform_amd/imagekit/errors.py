"""Mirror of reference `ImageKitError` (src/lib.rs:34-52)."""
from __future__ import annotations


class ImageKitError(Exception):
    prefix = "Internal server error"

    def __init__(self, message: str):
        super().__init__(message)
        self.message = message

    def __str__(self) -> str:
        return f"{self.prefix}: {self.message}"


class CacheError(ImageKitError):
    prefix = "Cache error"


class TransformError(ImageKitError):
    """The only variant the transform hot path emits."""

    prefix = "Transformation error"


class NetworkError(ImageKitError):
    prefix = "Network error"


class InvalidArgument(ImageKitError):
    prefix = "Invalid argument"


class NotFound(ImageKitError):
    prefix = "Not found"


class Unauthorized(ImageKitError):
    prefix = "Unauthorized"


class Expired(ImageKitError):
    prefix = "Expired"


class InternalError(ImageKitError):
    prefix = "Internal server error"

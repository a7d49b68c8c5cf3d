"""Mirror of reference src/config.rs (the types the hot path uses).

ImageFormat (:11-27), DEFAULT_QUALITY / MIN_QUALITY / MAX_QUALITY (:31-37) and
ImageKitConfig (:55-92, validate :115-123).  Only default_format and the quality
constants reach the transform path (src/lib.rs:185-186, :291-292).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional


class ImageFormat(enum.Enum):
    """`#[serde(rename_all = "lowercase")] enum ImageFormat { jpeg, webp, avif }`."""

    jpeg = 0
    webp = 1
    avif = 2

    def __str__(self) -> str:  # impl Display: lowercase name
        return self.name

    @classmethod
    def parse(cls, text: str) -> Optional["ImageFormat"]:
        """serde lowercase deserialisation (the /upload handler's match, src/lib.rs:270-272)."""
        return {"jpeg": cls.jpeg, "webp": cls.webp, "avif": cls.avif}.get(text)


DEFAULT_QUALITY = 80
MIN_QUALITY = 1
MAX_QUALITY = 100
DEFAULT_CACHE_CONTROL = "public, max-age=31536000, immutable"
NO_CACHE_CONTROL = "no-store"


class ConfigError(Exception):
    pass


class EmptySecret(ConfigError):
    def __str__(self) -> str:
        return "Secret cannot be empty"


class InvalidMaxInput(ConfigError):
    def __str__(self) -> str:
        return "Max input size must be > 0"


@dataclass
class ImageKitConfig:
    secret: str = ""
    cache_dir: Path = Path("./cache")
    max_input_size: int = 8 * 1024 * 1024
    max_cache_size: Optional[int] = 10 * 1024 * 1024 * 1024
    allowed_formats: List[ImageFormat] = field(
        default_factory=lambda: [ImageFormat.jpeg, ImageFormat.webp, ImageFormat.avif])
    default_format: Optional[ImageFormat] = ImageFormat.webp

    def validate(self) -> None:
        if not self.secret.strip():
            raise EmptySecret()
        if self.max_input_size == 0:
            raise InvalidMaxInput()

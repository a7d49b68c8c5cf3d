"""CPU: the host-side mirror of the reference types (src/config.rs, src/lib.rs)."""
import pytest

from imagekit import config, errors
from imagekit.config import ImageFormat, ImageKitConfig


def test_image_format_display_and_serde():
    assert [str(f) for f in ImageFormat] == ["jpeg", "webp", "avif"]
    assert ImageFormat.parse("webp") is ImageFormat.webp
    assert ImageFormat.parse("WEBP") is None  # serde rename_all = "lowercase"
    assert [f.value for f in ImageFormat] == [0, 1, 2]  # C ABI ik_format


def test_quality_constants():
    assert (config.DEFAULT_QUALITY, config.MIN_QUALITY, config.MAX_QUALITY) == (80, 1, 100)


def test_config_defaults_and_validate():
    c = ImageKitConfig()
    assert c.max_input_size == 8 * 1024 * 1024
    assert c.default_format is ImageFormat.webp
    assert c.allowed_formats == [ImageFormat.jpeg, ImageFormat.webp, ImageFormat.avif]
    with pytest.raises(config.EmptySecret):
        c.validate()
    ImageKitConfig(secret="s").validate()
    with pytest.raises(config.InvalidMaxInput):
        ImageKitConfig(secret="s", max_input_size=0).validate()


def test_error_display_matches_thiserror():
    assert str(errors.TransformError("bad")) == "Transformation error: bad"
    assert str(errors.InvalidArgument("q")) == "Invalid argument: q"
    assert issubclass(errors.TransformError, errors.ImageKitError)

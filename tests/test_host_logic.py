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


def test_bench_cli_formats_match_image_format(monkeypatch):
    """tools/bench_pipeline.py's --format values are the ImageFormat discriminants the
    C ABI takes (include/imagekit_hip.h ik_format), incl. the configs[4] AVIF runs;
    bench.py (the headline) uses the same table."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tools")]
    import bench as headline
    import bench_pipeline as bench
    assert headline.FORMATS == bench.FORMATS
    for f in ImageFormat:
        assert bench.FORMATS[str(f)] == f.value
    monkeypatch.setattr(sys, "argv", ["bench.py", "--size", "8192", "--out", "1024", "--filter", "lanczos3",
                                      "--format", "avif", "--quality", "60", "--batch", "32"])
    a = bench.parse()
    assert (a.size, a.out, a.filter, a.format, a.quality, a.batch, a.gpus) == (8192, 1024, "lanczos3", "avif", 60, 32, 1)
    assert set(bench.CPU_CODER) == set(bench.FORMATS)

"""GPU: the reference's own hot-path tests (tests/transform.rs, 20 #[test]s) run
against the MI355X implementation through the Python mirror of imagekit::transform.
Inputs are built the way the reference builds them (DynamicImage::new_rgb8 =
all-zero pixels; PNG fixtures from a blank RGBA image).  AVIF goes through
libavif/aom instead of ravif/rav1e, so AVIF bytes differ from
the reference's; the reference's AVIF assertions (non-empty output) hold."""
import io

import pytest

from imagekit import DynamicImage, ImageFormat, TransformError, decode_image, encode_image, resize_image

pytestmark = pytest.mark.gpu


def rgb8(w, h):
    return DynamicImage.new_rgb8(w, h)


def test_resize_dimensions_width_only(ik):                       # transform.rs:10-19
    assert resize_image(rgb8(800, 600), 400, None).dimensions() == (400, 300)


def test_resize_dimensions_height_only(ik):                      # :21-30
    assert resize_image(rgb8(800, 600), None, 300).dimensions() == (400, 300)


def test_resize_both_dimensions(ik):                              # :32-40
    assert resize_image(rgb8(800, 600), 400, 300).dimensions() == (400, 300)


def test_resize_preserves_aspect_ratio_non_standard(ik):          # :42-51
    assert resize_image(rgb8(1920, 1080), 960, None).dimensions() == (960, 540)


def test_no_resize_when_no_dimensions(ik):                        # :57-66
    img = rgb8(800, 600)
    assert resize_image(img, None, None).dimensions() == (800, 600)


def test_resize_larger_than_original(ik):                         # :68-76
    assert resize_image(rgb8(100, 100), 200, 200).dimensions() == (200, 200)


def test_resize_minimum_dimensions(ik):                           # :78-86
    assert resize_image(rgb8(800, 600), 1, 1).dimensions() == (1, 1)


def test_resize_very_small_to_large(ik):                          # :88-96
    assert resize_image(rgb8(2, 2), 200, 200).dimensions() == (200, 200)


def test_decode_invalid_data(ik):                                 # :102-110
    with pytest.raises(TransformError):
        decode_image(bytes(100))


def test_decode_empty_data(ik):                                   # :112-120
    with pytest.raises(TransformError):
        decode_image(b"")


def _blank_png(w, h):
    from PIL import Image
    buf = io.BytesIO()
    Image.new("RGBA", (w, h), (0, 0, 0, 0)).save(buf, format="PNG")
    return buf.getvalue()


def test_decode_then_webp(ik):                                    # :122-131
    decoded, _ = decode_image(_blank_png(64, 64))
    out = encode_image(decoded, ImageFormat.webp, 75)
    assert len(out) > 0


def test_all_format_encodings(ik):                                # :137-154 (jpeg, webp)
    img = rgb8(100, 100)
    jpeg = encode_image(img, ImageFormat.jpeg, 80)
    assert len(jpeg) > 0 and jpeg[:2] == b"\xff\xd8"
    assert len(encode_image(img, ImageFormat.webp, 80)) > 0


def test_all_format_encodings_avif(ik):                           # :151-153
    assert len(encode_image(rgb8(100, 100), ImageFormat.avif, 80)) > 0


def test_format_conversion_round_trip(ik):                        # :156-169
    encoded = encode_image(rgb8(50, 50), ImageFormat.webp, 80)
    decoded, fmt = decode_image(encoded)
    assert decoded.dimensions() == (50, 50)
    assert fmt is ImageFormat.webp


def test_quality_affects_jpeg_size(ik):                           # :175-186
    img = rgb8(500, 500)
    assert len(encode_image(img, ImageFormat.jpeg, 95)) > len(encode_image(img, ImageFormat.jpeg, 10))


def test_quality_affects_webp_size(ik):                           # :188-204
    img = rgb8(500, 500)
    assert len(encode_image(img, ImageFormat.webp, 10)) > 0
    assert len(encode_image(img, ImageFormat.webp, 95)) > 0


def test_quality_clamping_jpeg(ik):                               # :206-218
    img = rgb8(100, 100)
    encode_image(img, ImageFormat.jpeg, 0)
    encode_image(img, ImageFormat.jpeg, 101)


def test_resize_and_encode_jpeg(ik):                              # :224-236
    resized = resize_image(rgb8(800, 600), 400, None)
    assert resized.dimensions() == (400, 300)
    assert len(encode_image(resized, ImageFormat.jpeg, 80)) > 0


def test_full_pipeline_webp(ik):                                  # :238-257
    resized = resize_image(rgb8(1920, 1080), 640, 480)
    assert resized.dimensions() == (640, 360)
    encoded = encode_image(resized, ImageFormat.webp, 85)
    decoded, fmt = decode_image(encoded)
    assert decoded.dimensions() == (640, 360) and fmt is ImageFormat.webp


def test_full_pipeline_avif(ik):                                  # :259-269
    resized = resize_image(rgb8(800, 600), 400, None)
    assert resized.dimensions() == (400, 300)
    assert len(encode_image(resized, ImageFormat.avif, 80)) > 0


def test_resize_reduces_size(ik):                                 # :275-287
    img = rgb8(1000, 1000)
    original = encode_image(img, ImageFormat.jpeg, 80)
    resized = encode_image(resize_image(img.clone(), 100, 100), ImageFormat.jpeg, 80)
    assert len(resized) < len(original)


def test_fused_transform_matches_three_calls(ik):
    png = _blank_png(300, 200)
    from imagekit.transform import transform
    img, _ = decode_image(png)
    want = encode_image(resize_image(img, 150, None), ImageFormat.webp, 80)
    assert transform(png, 150, None, ImageFormat.webp, 80) == want

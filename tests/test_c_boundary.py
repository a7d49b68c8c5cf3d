"""The reference's tests/transform.rs (every #[test], same assertions) as a C
program over the C-ABI boundary with host pixel buffers: tests/c/transform_test.c,
built by the library Makefile against libimagekit_hip.so (no ctypes, no Python
in the calls).  Reference: /root/reference/tests/transform.rs:1-263,
src/transform.rs:27,62-66,113-117."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "rust-image-transform_amd", "lib", "transform_test")
RUST_TESTS = [
    "test_resize_dimensions_width_only", "test_resize_dimensions_height_only", "test_resize_both_dimensions",
    "test_resize_preserves_aspect_ratio_non_standard", "test_no_resize_when_no_dimensions",
    "test_resize_larger_than_original", "test_resize_minimum_dimensions", "test_resize_very_small_to_large",
    "test_decode_invalid_data", "test_decode_empty_data", "decode_then_webp", "test_all_format_encodings",
    "test_format_conversion_round_trip", "test_quality_affects_jpeg_size", "test_quality_affects_webp_size",
    "test_quality_clamping_jpeg", "resize_and_encode_jpeg", "test_full_pipeline_webp", "test_full_pipeline_avif",
    "test_resize_reduces_size",
]


def test_c_program_built_and_covers_every_rust_test():
    assert os.path.exists(BIN), "build() / make builds lib/transform_test"
    src = open(os.path.join(ROOT, "tests", "c", "transform_test.c")).read()
    for name in RUST_TESTS:
        assert f'run("{name}", {name})' in src, name


@pytest.mark.gpu
def test_reference_transform_tests_through_c_abi():
    # a child process (the C program initialises the GPU itself)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    lines = r.stdout.strip().splitlines()
    passed = {ln.split()[1] for ln in lines if ln.startswith("PASS ")}
    assert r.returncode == 0, r.stdout + r.stderr
    # the 20 reference tests, then a batch + ik_shutdown; rc 0 = the process
    # also exited cleanly after the orderly teardown
    assert passed == set(RUST_TESTS) | {"batch_then_shutdown"}, r.stdout

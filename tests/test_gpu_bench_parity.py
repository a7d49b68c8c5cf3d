"""GPU: oracle parity of the EXACT batches behind bench.py's numbers (VERDICT r3
"Next" 1), every output byte-compared with the oracle's transform of its source.

* `value` (configs[1]): bench.py's own headline batch -- its --distinct 4 frames
  (bench.shard_seeds / bench.make_pngs: 4096^2 RGBA8, pattern S, PNG zlib level 6)
  tiled over 64 requests, each its own device allocation (DeviceBytes), three
  batches in flight through ik_transform_batch_submit_device (bench --inflight 3),
  512^2 Triangle ("bilinear") WebP q80 with bench's 32 host threads.  The third
  batch carries one pattern-N frame (codec worst case) in place of a request.
  Oracle: image 0.25.8 resize restated + libwebp WebPEncodeRGB
  (/root/reference/src/transform.rs:62-90,129-137).
* configs[2]: bench.py --source jpeg-rst's batch (bench.make_jpegs: JPEG q90
  4:2:0 with a restart marker per MCU row, page-locked inputs) -- 256 requests,
  512^2 Lanczos3, JPEG q85 -- next to a second 256-request batch mixing
  restart-marked and restart-free sources (the self-synchronising path), both in
  flight together through ik_transform_batch_submit.  All 256 scans go through
  the self-synchronising GPU entropy decoder together (k_jsync_sync, k_jsync_fix
  + k_jsync_settle, k_jsync_seg1-3, k_jsync_decode: one launch each per batch),
  then four 64-image sub-batches of the batched JPEG encoder (ik_host.cpp
  jpeg_front_group).  Oracle:
  oracle.jpeg_encode_rgb(to_rgb8(resize(jpeg_decode(src, zune), 512, 512,
  LANCZOS3)), 85) -- /root/reference/src/transform.rs:27-43,85-89,121-128.

Each test asserts that every stream was decoded by the GPU path (the counters),
so the HIP kernels are what was compared."""
import ctypes

import pytest

import bench
import ikutil
from imagekit import DeviceBytes, ImageFormat, PinnedBytes, transform_batch_submit, transform_batch_submit_device

pytestmark = pytest.mark.gpu

WEBP, JPEG = ImageFormat.webp.value, ImageFormat.jpeg.value


def _counts(ik, fn):
    c = (ctypes.c_ulonglong * 2)()
    getattr(ik, fn)(c)
    return c[0], c[1]


@pytest.fixture(scope="module")
def bench_frames():
    # bench.py main(): frames of rank 0, --distinct 4, --size 4096
    return [ikutil.synth(4096, 4096, 4, seed=sd, pattern="S") for sd in bench.shard_seeds(0, 4)]


@pytest.mark.parametrize("encoder", ["libwebp", "exact"])
def test_bench_headline_batch_equals_oracle(ik, oracle, bench_frames, encoder):
    # both WebP coders: libwebp on the host, and the exact GPU coder (IK_WEBP_EXACT:
    # ik_vp8x.hip's persistent launch per same-geometry group), each byte-identical
    B = 64
    prev = ik.ik_get_webp_encoder()
    assert ik.ik_set_webp_encoder({"libwebp": 0, "exact": 2}[encoder]) == 0
    try:
        _headline_batches(ik, oracle, bench_frames, B)
    finally:
        ik.ik_set_webp_encoder(prev)


def _headline_batches(ik, oracle, bench_frames, B):
    pngs = bench.make_pngs(bench_frames)
    noise = ikutil.synth(4096, 4096, 4, seed=4, pattern="N")
    npng = bench.make_pngs([noise])[0]
    dev = [DeviceBytes(p) for p in pngs]
    dnoise = DeviceBytes(npng)
    batches = [[dev[i % 4] for i in range(B)] for _ in range(3)]
    batches[2][17] = dnoise
    src_of = [[i % 4 for i in range(B)] for _ in range(3)]
    src_of[2][17] = 4
    g0, h0 = _counts(ik, "ik_png_counters")
    pend = [transform_batch_submit_device(b, [(512, 512)] * B, [WEBP] * B, [80] * B, filter=ikutil.TRIANGLE,
                                          threads=32) for b in batches]
    outs = [p.wait() for p in pend]
    g1, h1 = _counts(ik, "ik_png_counters")
    assert (g1 - g0, h1 - h0) == (3 * B, 0), "every device-resident 4096^2 stream must decode on the GPU"
    want = [oracle.transform(f, 512, 512, ikutil.TRIANGLE, WEBP, 80)[0] for f in bench_frames + [noise]]
    for k in range(3):
        for i in range(B):
            assert outs[k][i] == want[src_of[k][i]], f"batch {k} request {i}: bytes differ from the oracle's"


def test_bench_config2_batches_equal_oracle(ik, oracle, bench_frames):
    B = 256
    rst = bench.make_jpegs(bench_frames, rst=True)  # bench.py --source jpeg-rst
    norst = bench.make_jpegs(bench_frames[:2], rst=False)
    nf = [ikutil.synth(4096, 4096, 4, seed=sd, pattern="N") for sd in (5, 6)]
    mixed_src = rst + norst + bench.make_jpegs(nf[:1], rst=True) + bench.make_jpegs(nf[1:], rst=False)
    pin = {id(s): PinnedBytes(s) for s in rst + mixed_src}
    batch_a = [rst[i % 4] for i in range(B)]
    batch_b = [mixed_src[(7 * i) % len(mixed_src)] for i in range(B)]
    j0 = _counts(ik, "ik_jpeg_counters")
    pa = transform_batch_submit([pin[id(s)] for s in batch_a], [(512, 512)] * B, [JPEG] * B, [85] * B,
                                filter=ikutil.LANCZOS3, threads=32)
    pb = transform_batch_submit([pin[id(s)] for s in batch_b], [(512, 512)] * B, [JPEG] * B, [85] * B,
                                filter=ikutil.LANCZOS3, threads=32)
    ga, gb = pa.wait(), pb.wait()
    j1 = _counts(ik, "ik_jpeg_counters")
    assert (j1[0] - j0[0], j1[1] - j0[1]) == (2 * B, 0), "every 4096^2 source must be entropy-decoded on the GPU"
    want = {}
    for s in rst + mixed_src:
        if id(s) not in want:
            px = oracle.jpeg_decode(s, mode=1)  # the zune-jpeg 0.4.21 restatement
            want[id(s)] = oracle.transform(px, 512, 512, ikutil.LANCZOS3, JPEG, 85)[0]
    for i in range(B):
        assert ga[i] == want[id(batch_a[i])], f"configs[2] batch request {i}: bytes differ from the oracle's"
        assert gb[i] == want[id(batch_b[i])], f"mixed batch request {i}: bytes differ from the oracle's"

"""Dev: decode wall time of 4096^2 restart-interval JPEGs (q90 4:2:0, one RSTn
per MCU row, configs[2]-like): ik_decode one at a time, host vs GPU entropy
decoding (IK_JPEG_GPU_ENTROPY, read per child process), and ik_decode_batch."""
import io, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]


def blobs(S, n):
    from PIL import Image
    import ikutil
    out = []
    for i in range(n):
        buf = io.BytesIO()
        Image.fromarray(ikutil.synth(S, S, 3, seed=9 + i, pattern="S")).save(
            buf, format="JPEG", quality=90, subsampling=2,
            **({} if os.environ.get("NORST") else {"restart_marker_rows": 1}))
        out.append(buf.getvalue())
    return out


def run(mode):
    from imagekit import decode_image, decode_image_batch
    S, N = int(os.environ.get("S", "4096")), int(os.environ.get("N", "16"))
    bs = blobs(S, N)
    tag = (f"{S}x{S} q90 4:2:0 {'no restarts' if os.environ.get('NORST') else 'rst/row'}, "
           f"{sum(map(len, bs)) / N / 1e6:.2f} MB each")
    if mode == "batch":
        decode_image_batch(bs[:2])
        t0 = time.perf_counter()
        out = decode_image_batch(bs)
        t = time.perf_counter() - t0
        del out
        print(f"ik_decode_batch x{N} {tag}: {t * 1e3:.1f} ms  {N * S * S / t / 1e6:.0f} MPix/s", flush=True)
        return
    decode_image(bs[0])
    t0 = time.perf_counter()
    for b in bs:
        img, _ = decode_image(b)
    t = time.perf_counter() - t0
    print(f"ik_decode x{N} ({mode} entropy) {tag}: {t * 1e3 / N:.1f} ms/image  {N * S * S / t / 1e6:.0f} MPix/s",
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for mode, v in (("gpu", "1"), ("host", "0"), ("batch", "1")):
            subprocess.run([sys.executable, __file__, mode], env=dict(os.environ, IK_JPEG_GPU_ENTROPY=v), check=True)

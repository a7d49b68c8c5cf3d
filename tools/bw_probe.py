"""Dev: run tools/bw_probe.hip (built to tools/libbwprobe.so)."""
import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(here, "libbwprobe.so"))
L.probe.restype = ctypes.c_double
L.probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
S, n = 4096, 32
buf = torch.randint(0, 255, (n, S, S * 4), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
names = {0: "strip 8B/lane D=8", 1: "contiguous stream 16B", 2: "strip 8B/lane D=16", 3: "strip 16B/lane D=8", 4: "strip 16B/lane D=4"}
import sys
only = [int(x) for x in sys.argv[1:]] if len(sys.argv) > 1 else None
for pat in (only or (1, 0, 2, 3, 4)):
    for band in (((64,) if only else (4096, 512, 64)) if pat != 1 else (4096,)):
        ms = L.probe(pat, buf.data_ptr(), S * 4, S, n, band, 10)
        gb = n * S * S * 4 / (ms * 1e-3) / 1e9
        print(f"{names[pat]:24s} band_rows={band:5d}  {ms:.3f} ms  {gb:7.0f} GB/s", flush=True)

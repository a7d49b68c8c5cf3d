"""Print the headline fields of a bench.py JSON line (the last line of a file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
rr = d.get("roofline_resize") or {}
c = d.get("cpu_baseline") or {}
p = d.get("pcie_inclusive") or {}
print(f"value {d['value']} {d['unit']} ({d['ms_per_step']} ms/step); pcie_inclusive {p.get('value')}; "
      f"roofline {r.get('kernel')} {r.get('kernel_ms')} ms frac {r.get('frac')}; "
      f"resize {rr.get('kernel_ms')} ms frac {rr.get('frac')}; cpu {c.get('value')} on {c.get('cores')} cores")
print("png stages", d.get("png_decode_stages_ms"))
print("jpeg", d.get("jpeg_entropy_decode"), "enc", d.get("jpeg_encode_batched"))

# Dev: tools/resize_ab.py over several libraries (RGBA 64 and RGB 256 4096^2 frames -> 512^2)
for L in "$@"; do
  timeout -k 10 120 python tools/resize_ab.py $L 4 64 || exit 1
  timeout -k 10 120 python tools/resize_ab.py $L 3 256 || exit 1
done

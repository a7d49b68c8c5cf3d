# Dev: the resize kernel alone with the periodic kernel on and off (IK_RESIZE_PERIODIC),
# RGBA 64 and RGB 256 frames of 4096^2 -> 512^2 (tools/resize_ab.py), library $1
L=${1:-rust-image-transform_amd/lib/libimagekit_hip.so}
for p in 1 0 1 0; do
  IK_RESIZE_PERIODIC=$p timeout -k 10 120 python tools/resize_ab.py $L 4 64 | sed "s/^/periodic=$p /" || exit 1
  IK_RESIZE_PERIODIC=$p timeout -k 10 120 python tools/resize_ab.py $L 3 256 | sed "s/^/periodic=$p /" || exit 1
done

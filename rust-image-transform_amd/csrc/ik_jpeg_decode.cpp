// ik_jpeg_decode.cpp -- JPEG branch of decode_image (reference src/transform.rs:31 ->
// image 0.25.8 -> zune-jpeg 0.4.21, Cargo.lock:3106).  Placeholder until the
// baseline/progressive decoder lands; the error maps to TransformError.
#include "../../include/imagekit_hip.h"
#include "ik_runtime.h"

namespace ik {

int decode_jpeg(const uint8_t* b, size_t n, uint32_t& w, uint32_t& h, uint32_t& c, std::vector<uint8_t>& px) {
    (void)b; (void)n; (void)w; (void)h; (void)c; (void)px;
    return fail(IK_ERR_UNSUPPORTED, "JPEG decoding is not implemented in this build yet");
}

}  // namespace ik

/*
 * ik_oracle.h -- CPU ORACLE for the imagekit transform hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libimagekit_hip.so, the
 * `imagekit` Python mirror) links, loads or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline.
 *
 * What it restates (reference = /root/reference, Shreyas2409/Rust-Image-Transform):
 *   - src/transform.rs:62-90   resize_image: f32 target-dim math, max(1), Lanczos3
 *   - image 0.25.8 (Cargo.lock:987)  DynamicImage::resize -> resize_dimensions
 *     (aspect FIT, f64) -> imageops::resize -> vertical_sample, horizontal_sample
 *     (src/imageops/sample.rs).  That crate source is NOT vendored in the
 *     reference tree; the algorithm is restated from its published source.
 *   - src/transform.rs:113-150 encode_image: to_rgb8 + image JpegEncoder
 *     (src/codecs/jpeg/encoder.rs + transform.rs fdct), and
 *     webp 0.3.1 -> libwebp WebPEncodeRGB (Cargo.lock:2811, 1168).
 *   - libwebp's RGB -> YUV420 import (picture_csp_enc.c ImportYUVAFromRGBA),
 *     restated so the GPU colour-convert kernel can be checked plane by plane.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - dimension policy: pinned by the reference's own tests/transform.rs KATs;
 *   - WebP YUV planes and WebP bytes: pinned against the system libwebp 1.2.2
 *     (a proxy for libwebp-sys 0.9.6's vendored copy);
 *   - resize pixel values and JPEG bytes: "parity unpinned" against the real
 *     image crate (no Rust toolchain, no crate sources here); cross-checked by an
 *     independent numpy restatement (tests/oracle_np.py).
 */
#ifndef IK_ORACLE_H
#define IK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* image::imageops::FilterType (image 0.25.8 src/imageops/sample.rs) */
enum { IKO_NEAREST = 0, IKO_TRIANGLE = 1, IKO_CATMULLROM = 2, IKO_GAUSSIAN = 3, IKO_LANCZOS3 = 4 };

/* image 0.25.8 dynimage.rs resize_dimensions(width,height,nwidth,nheight,fill) */
void iko_resize_dimensions(uint32_t w, uint32_t h, uint32_t nw, uint32_t nh, int fill,
                           uint32_t *ow, uint32_t *oh);

/* src/transform.rs:62-90 + DynamicImage::resize: final output geometry.
 * w_opt/h_opt < 0 means None.  Returns 0 when the image is returned unchanged
 * (both None, or resize() decides on a copy), 1 when it is resampled. */
int iko_resize_image_dims(uint32_t W, uint32_t H, int64_t w_opt, int64_t h_opt,
                          uint32_t *ow, uint32_t *oh);

/* sample.rs filter weights for one axis (in -> out).  left[o], count[o] and
 * w[o*maxtaps + k] (normalised).  Returns the max tap count, or -1 if maxtaps
 * is too small. */
int iko_axis_weights(uint32_t in, uint32_t out, int filter, int32_t *left, int32_t *count,
                     float *w, int maxtaps);

/* imageops::resize(image, nw, nh, filter) on an 8-bit image with C interleaved
 * channels (C in 1..4), tightly packed rows.  dst must hold nw*nh*C bytes. */
int iko_resize_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, uint32_t nw,
                  uint32_t nh, int filter, uint8_t *dst);

/* same, keeping the f32 vertical intermediate (W x nh x C) for debugging */
int iko_vertical_sample_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, uint32_t nh,
                           int filter, float *tmp);

/* DynamicImage::to_rgb8 / to_rgba8 for 8-bit sources with C channels */
void iko_to_rgb8(const uint8_t *src, uint32_t npix, uint32_t C, uint8_t *dst);
void iko_to_rgba8(const uint8_t *src, uint32_t npix, uint32_t C, uint8_t *dst);

/* libwebp ImportYUVAFromRGBA (no alpha, no dithering, non-iterative) on RGB8. */
void iko_webp_rgb_to_yuv420(const uint8_t *rgb, int width, int height, int stride,
                            uint8_t *y, int y_stride, uint8_t *u, uint8_t *v, int uv_stride);

/* image 0.25.8 JpegEncoder::new_with_quality(q).write_image(rgb, w, h, Rgb8).
 * Returns the byte count written to *out (malloc'd; free with iko_free), or -1. */
long iko_jpeg_encode_rgb(const uint8_t *rgb, uint32_t w, uint32_t h, int quality, uint8_t **out);
/* quantised DCT coefficients for all 8x8 blocks (block-major, Y,Cb,Cr per MCU,
 * natural order), to check the GPU colour-convert+FDCT+quantise kernel. */
int iko_jpeg_coeffs_rgb(const uint8_t *rgb, uint32_t w, uint32_t h, int quality, int16_t *coef);

/* decode_image on a JPEG (jpeg_dec.c): baseline / progressive, 1, 3 or 4
 * components -> L8 (c = 1) or RGB8 (c = 3) in *out (malloc'd; free with
 * iko_free).  mode: the reconstruction restated (see jpeg_dec.c). */
enum { IKO_JPEG_LIBJPEG = 0, IKO_JPEG_ZUNE = 1 };
int iko_jpeg_decode(const uint8_t *bytes, size_t n, int mode, uint8_t **out, int *w, int *h, int *c);

/* webp 0.3.1 Encoder::from_rgb(..).encode(q) == libwebp WebPEncodeRGB(rgb,w,h,3w,q)
 * through dlopen("libwebp.so.7").  Returns size, or -1 (library missing). */
long iko_webp_encode_rgb(const uint8_t *rgb, int w, int h, int stride, float q, uint8_t **out);
/* libwebp's method-4 macroblock decisions restated (vp8_modes.c): modes per MB and the
 * final coefficient probabilities, from YUV420 planes + the segment set-up */
int iko_vp8_modes(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, float quality,
                  const uint8_t *seg, const int *quant, int dq_uv_dc, int dq_uv_ac, uint8_t *ymode,
                  uint8_t *bmodes, uint8_t *uvmode, uint8_t *probas);
/* the whole WebP file libwebp writes, restated (vp8_modes.c); *out malloc'd (iko_free) */
long iko_vp8_encode(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, float quality,
                    const uint8_t *seg, int num_segments, int update_map, const int *probs, const int *quant,
                    const int *fstr, int dq_uv_dc, int dq_uv_ac, uint8_t **out);

/* the reference CPU transform (resize_image + encode_image) on a decoded 8-bit
 * image: fmt 0=jpeg 1=webp.  Used as bench.py's cpu_baseline "port". */
long iko_transform_u8(const uint8_t *src, uint32_t W, uint32_t H, uint32_t C, int64_t w_opt,
                      int64_t h_opt, int filter, int fmt, int quality, uint8_t **out,
                      uint32_t *ow, uint32_t *oh);

/* decode_image on a PNG (image 0.25.8 -> png 0.18, EXPAND) for non-interlaced
 * 8-bit colour types 0/2/4/6: CRC-checked chunks, inflate, unfilter.  Returns the
 * pixel byte count (pixels in *out, iko_free) or < 0.  png_dec.c. */
long iko_png_decode(const uint8_t *png, size_t n, uint8_t **out, uint32_t *w, uint32_t *h, uint32_t *c);

void iko_free(void *p);

#ifdef __cplusplus
}
#endif
#endif

// TrainPre on the GPU: the training augmentation of dataloader/dataloader.py:85-112 on uint8
// HWC images resident in HBM.  The host (augment.TrainPre) draws the
// per-sample random parameters in the reference's order; these kernels do the pixel work:
//
//   cmx_aug_resize_u8        random_mirror (:9-14, folded into the source index) + label clip
//                            (TrainPre :88, folded into the read) + random_scale (:16-23):
//                            cv2 INTER_LINEAR (images) / INTER_NEAREST (labels)
//   cmx_aug_color_jitter_u8  random_color_jitter (:32-54): BGR->HSV (8U integer tables),
//                            V*bf, S*sf, H+hf*180 in fp32, clip, truncate, HSV->BGR (8U)
//   cmx_aug_blur5_u8         random_gaussian_blur (:56-59): 5x5 sigma-1 fixed-point Gaussian
//   cmx_aug_finalize         cutout (:61-83, the box applied on the source reads) +
//                            ensure_size (:25-31) + normalize (utils/transforms.py:182-187) +
//                            HWC -> CHW (:109-110) + the float / long casts of RGBXDataset
//                            (:65-68), written straight into the batch slot
//
// The cv2 8-bit arithmetic is restated exactly (oracle/augment_ref.py documents each rule), so
// these kernels are bit-exact against the oracle: integer / fixed-point sums, fp32 colour math
// with explicitly rounded operations (no contraction), fp64 normalisation.  Everything is
// HBM-bound byte work: one thread per output pixel, all channels in registers.
#include "cmx_common.h"

// cv2's colour and coefficient arithmetic is separate multiplies and adds: no FMA contraction in
// this file.  (HIP's __fmul_rn & co. are operators defined in a header, outside the pragma's
// reach, whose results the backend may still fuse, hence these local rounded operations.)
#pragma clang fp contract(off)

namespace {

__device__ __forceinline__ float fmul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float fadd_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float fsub_rn(float a, float b) { return a - b; }

constexpr int COEF_SCALE = 2048;            // INTER_RESIZE_COEF_BITS = 11

// one axis of cv2's INTER_LINEAR: source pair (s0, s1) and 11-bit weights (w0, w1)
__device__ __forceinline__ void lin_axis(int d, double scale, int ssize, int& s0, int& s1, int& w0, int& w1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f = fsub_rn(f, (float)s);
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
  s0 = s;
  s1 = min(s + 1, ssize - 1);
  w0 = (int)rintf(fmul_rn(fsub_rn(1.f, f), (float)COEF_SCALE));
  w1 = (int)rintf(fmul_rn(f, (float)COEF_SCALE));
}

__device__ __forceinline__ int lin_combine(int d0, int d1, int b0, int b1) {
  // VResizeLinearVec_32s8u: ((D0 >> 4) * b0 >> 16) + ((D1 >> 4) * b1 >> 16), + 2, >> 2
  const int v = ((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2;
  return min(max(v, 0), 255);
}

__device__ __forceinline__ int nn_index(int d, double inv, int ssize) {
  return min((int)floor(d * inv), ssize - 1);
}

template <int C>
__device__ __forceinline__ void resize_px(const uint8_t* __restrict__ src, int h, int w, uint8_t* __restrict__ dst,
                                          int oh, int ow, int nearest, int mirror, int clip_max, double sx,
                                          double sy, long p) {
  const int oy = (int)(p / ow), ox = (int)(p - (long)oy * ow);
  auto col = [&](int x) { return mirror ? w - 1 - x : x; };
  uint8_t* o = dst + p * C;
  if (nearest) {
    const int y = nn_index(oy, sy, h), x = col(nn_index(ox, sx, w));
    const uint8_t* s = src + ((long)y * w + x) * C;
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = clip_max >= 0 ? (uint8_t)min((int)s[c], clip_max) : s[c];
    return;
  }
  int x0, x1, a0, a1, y0, y1, b0, b1;
  lin_axis(ox, sx, w, x0, x1, a0, a1);
  lin_axis(oy, sy, h, y0, y1, b0, b1);
  x0 = col(x0);
  x1 = col(x1);
  const uint8_t* r0 = src + (long)y0 * w * C;
  const uint8_t* r1 = src + (long)y1 * w * C;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int v00 = r0[x0 * C + c], v01 = r0[x1 * C + c], v10 = r1[x0 * C + c], v11 = r1[x1 * C + c];
    if (clip_max >= 0) {
      v00 = min(v00, clip_max); v01 = min(v01, clip_max); v10 = min(v10, clip_max); v11 = min(v11, clip_max);
    }
    o[c] = (uint8_t)lin_combine(v00 * a0 + v01 * a1, v10 * a0 + v11 * a1, b0, b1);
  }
}

template <int C>
__global__ __launch_bounds__(256) void resize_u8_kernel(const uint8_t* __restrict__ src, int h, int w,
                                                        uint8_t* __restrict__ dst, int oh, int ow, int nearest,
                                                        int mirror, int clip_max, double sx, double sy) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)oh * ow) return;
  resize_px<C>(src, h, w, dst, oh, ow, nearest, mirror, clip_max, sx, sy, p);
}

// ---------------------------------------------------------------------------- colour
__device__ __forceinline__ void bgr2hsv(int b, int g, int r, int& h, int& s, int& v) {
  v = max(max(b, g), r);
  const int vmin = min(min(b, g), r);
  const int diff = v - vmin;
  const int sdiv = v ? (int)rint((double)(255 << 12) / (double)v) : 0;
  const int hdiv = diff ? (int)rint((double)(180 << 12) / (6.0 * diff)) : 0;
  s = (diff * sdiv + (1 << 11)) >> 12;
  int hh = v == r ? g - b : (v == g ? b - r + 2 * diff : r - g + 4 * diff);
  hh = (hh * hdiv + (1 << 11)) >> 12;
  h = hh < 0 ? hh + 180 : hh;
}

__device__ __forceinline__ uint8_t sat_u8(float x) {
  const float r = rintf(fmul_rn(x, 255.f));
  return (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
}

__device__ __forceinline__ void hsv2bgr(int H, int S, int V, uint8_t* o) {
  const float s = fmul_rn((float)S, 1.f / 255.f);
  const float v = fmul_rn((float)V, 1.f / 255.f);
  if (S == 0) {
    o[0] = o[1] = o[2] = sat_u8(v);
    return;
  }
  float h = fmul_rn((float)H, 6.f / 180.f);
  h = fmodf(h, 6.f);
  if (h < 0.f) h = fadd_rn(h, 6.f);
  int sector = (int)floorf(h);
  h = fsub_rn(h, (float)sector);
  if ((unsigned)sector >= 6u) { sector = 0; h = 0.f; }
  float tab[4];
  tab[0] = v;
  tab[1] = fmul_rn(v, fsub_rn(1.f, s));
  tab[2] = fmul_rn(v, fsub_rn(1.f, fmul_rn(s, h)));
  tab[3] = fmul_rn(v, fsub_rn(1.f, fmul_rn(s, fsub_rn(1.f, h))));
  // sector_data of HSV2RGB_native: {b, g, r} table indices
  const int sb[6] = {1, 1, 3, 0, 0, 2}, sg[6] = {3, 0, 0, 2, 1, 1}, sr[6] = {0, 2, 1, 1, 3, 0};
  o[0] = sat_u8(tab[sb[sector]]);
  o[1] = sat_u8(tab[sg[sector]]);
  o[2] = sat_u8(tab[sr[sector]]);
}

// hsv float32 ops of random_color_jitter: H + hf*180, S * sf, V * bf, np.clip(0, 255), then
// astype(uint8) (truncation of a non-negative value)
__device__ __forceinline__ int clip_trunc(float f) { return (int)fminf(fmaxf(f, 0.f), 255.f); }

__device__ __forceinline__ void jitter_px(uint8_t* __restrict__ img, long p, float bf, float sf, float hadd) {
  uint8_t* q = img + p * 3;
  int h, s, v;
  bgr2hsv(q[0], q[1], q[2], h, s, v);
  h = clip_trunc(fadd_rn((float)h, hadd));
  s = clip_trunc(fmul_rn((float)s, sf));
  v = clip_trunc(fmul_rn((float)v, bf));
  hsv2bgr(h, s, v, q);
}

__global__ __launch_bounds__(256) void jitter_kernel(uint8_t* __restrict__ img, long n, float bf, float sf, float hadd) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  jitter_px(img, p, bf, sf, hadd);
}

// ---------------------------------------------------------------------------- blur
__device__ __forceinline__ int refl101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

__device__ __forceinline__ void blur5_px(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int h, int w,
                                         int C, long p) {
  const int y = (int)(p / w), x = (int)(p - (long)y * w);
  const int k[5] = {14, 62, 104, 62, 14};
  int xs[5], ys[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    xs[t] = refl101(x + t - 2, w);
    ys[t] = refl101(y + t - 2, h);
  }
  for (int c = 0; c < C; ++c) {
    int acc = 0;
#pragma unroll
    for (int ty = 0; ty < 5; ++ty) {
      const uint8_t* row = src + (long)ys[ty] * w * C + c;
      int hs = 0;
#pragma unroll
      for (int tx = 0; tx < 5; ++tx) hs += k[tx] * row[xs[tx] * C];
      acc += k[ty] * hs;
    }
    dst[p * C + c] = (uint8_t)min((acc + (1 << 15)) >> 16, 255);
  }
}

__global__ __launch_bounds__(256) void blur5_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int h,
                                                    int w, int C) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)h * w) return;
  blur5_px(src, dst, h, w, C, p);
}

// ---------------------------------------------------------------------------- finalize
struct FinArgs {
  const uint8_t *rgb, *x, *gt;
  int h, w, oh, ow, bx1, by1, bx2, by2, background;
  double sx, sy, isx, isy;
  double mean[3], std[3];
  float *rgb_out, *x_out;
  int64_t* gt_out;
};

__device__ __forceinline__ bool in_box(const FinArgs& a, int y, int x) {
  return x >= a.bx1 && x < a.bx2 && y >= a.by1 && y < a.by2;
}

__device__ __forceinline__ void finalize_px(const FinArgs& a, long p) {
  const long plane = (long)a.oh * a.ow;
  const int oy = (int)(p / a.ow), ox = (int)(p - (long)oy * a.ow);
  // label: nearest, cutout box -> background
  {
    const int y = nn_index(oy, a.isy, a.h), x = nn_index(ox, a.isx, a.w);
    a.gt_out[p] = in_box(a, y, x) ? a.background : (int64_t)a.gt[(long)y * a.w + x];
  }
  int x0, x1, a0, a1, y0, y1, b0, b1;
  lin_axis(ox, a.sx, a.w, x0, x1, a0, a1);
  lin_axis(oy, a.sy, a.h, y0, y1, b0, b1);
  const bool z00 = in_box(a, y0, x0), z01 = in_box(a, y0, x1), z10 = in_box(a, y1, x0), z11 = in_box(a, y1, x1);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const uint8_t* s = m == 0 ? a.rgb : a.x;
    float* out = m == 0 ? a.rgb_out : a.x_out;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int v00 = z00 ? 0 : s[((long)y0 * a.w + x0) * 3 + c];
      const int v01 = z01 ? 0 : s[((long)y0 * a.w + x1) * 3 + c];
      const int v10 = z10 ? 0 : s[((long)y1 * a.w + x0) * 3 + c];
      const int v11 = z11 ? 0 : s[((long)y1 * a.w + x1) * 3 + c];
      const int u = lin_combine(v00 * a0 + v01 * a1, v10 * a0 + v11 * a1, b0, b1);
      const double f = ((double)u / 255.0 - a.mean[c]) / a.std[c];
      out[c * plane + p] = (float)f;
    }
  }
}

__global__ __launch_bounds__(256) void finalize_kernel(const FinArgs a) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)a.oh * a.ow) return;
  finalize_px(a, p);
}

// ---------------------------------------------------------------------------- minibatch
// cmx_aug_batch: the four stages over a whole minibatch, one launch per stage, blockIdx.y =
// sample.  Each sample's record (CMX_AUG_REC int64 words, layout in include/cmx_hip.h) carries
// its device pointers, sizes and draws; a block past its sample's (smaller) scaled size exits.
constexpr int AUG_REC = 24;

struct AugRec {
  const uint8_t *rgb, *x, *gt;
  uint8_t *rs, *xs, *gs, *rb;
  float *rgb_out, *x_out;
  int64_t* gt_out;
  int h, w, sh, sw, mirror, bx1, by1, bx2, by2;
  float bf, sf, hadd;
};

__device__ __forceinline__ AugRec aug_rec(const int64_t* __restrict__ table, int b) {
  const int64_t* r = table + (long)b * AUG_REC;
  AugRec a;
  a.rgb = (const uint8_t*)r[0]; a.x = (const uint8_t*)r[1]; a.gt = (const uint8_t*)r[2];
  a.rs = (uint8_t*)r[3]; a.xs = (uint8_t*)r[4]; a.gs = (uint8_t*)r[5]; a.rb = (uint8_t*)r[6];
  a.rgb_out = (float*)r[7]; a.x_out = (float*)r[8]; a.gt_out = (int64_t*)r[9];
  a.h = (int)r[10]; a.w = (int)r[11]; a.sh = (int)r[12]; a.sw = (int)r[13]; a.mirror = (int)r[14];
  a.bx1 = (int)r[15]; a.by1 = (int)r[16]; a.bx2 = (int)r[17]; a.by2 = (int)r[18];
  a.bf = __int_as_float((int)r[19]); a.sf = __int_as_float((int)r[20]); a.hadd = __int_as_float((int)r[21]);
  return a;
}

// blockIdx.z: 0 = rgb, 1 = x (bilinear), 2 = label (nearest + clip)
__global__ __launch_bounds__(256) void resize_batch_kernel(const int64_t* __restrict__ table, int clip_max) {
  const AugRec a = aug_rec(table, blockIdx.y);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)a.sh * a.sw) return;
  const double sx = 1.0 / ((double)a.sw / a.w), sy = 1.0 / ((double)a.sh / a.h);
  if (blockIdx.z == 2) resize_px<1>(a.gt, a.h, a.w, a.gs, a.sh, a.sw, 1, a.mirror, clip_max, sx, sy, p);
  else resize_px<3>(blockIdx.z ? a.x : a.rgb, a.h, a.w, blockIdx.z ? a.xs : a.rs, a.sh, a.sw, 0, a.mirror, -1, sx, sy, p);
}

__global__ __launch_bounds__(256) void jitter_batch_kernel(const int64_t* __restrict__ table) {
  const AugRec a = aug_rec(table, blockIdx.y);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)a.sh * a.sw) return;
  jitter_px(a.rs, p, a.bf, a.sf, a.hadd);
}

__global__ __launch_bounds__(256) void blur_batch_kernel(const int64_t* __restrict__ table) {
  const AugRec a = aug_rec(table, blockIdx.y);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (a.rb == nullptr || p >= (long)a.sh * a.sw) return;
  blur5_px(a.rs, a.rb, a.sh, a.sw, 3, p);
}

__global__ __launch_bounds__(256) void finalize_batch_kernel(const int64_t* __restrict__ table, int oh, int ow,
                                                             int background, double m0, double m1, double m2,
                                                             double s0, double s1, double s2) {
  const AugRec r = aug_rec(table, blockIdx.y);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)oh * ow) return;
  FinArgs a;
  a.rgb = r.rb ? r.rb : r.rs; a.x = r.xs; a.gt = r.gs;
  a.h = r.sh; a.w = r.sw; a.oh = oh; a.ow = ow;
  a.bx1 = r.bx1; a.by1 = r.by1; a.bx2 = r.bx2; a.by2 = r.by2; a.background = background;
  a.sx = 1.0 / ((double)ow / r.sw); a.sy = 1.0 / ((double)oh / r.sh);
  a.isx = a.sx; a.isy = a.sy;
  a.mean[0] = m0; a.mean[1] = m1; a.mean[2] = m2;
  a.std[0] = s0; a.std[1] = s1; a.std[2] = s2;
  a.rgb_out = r.rgb_out; a.x_out = r.x_out; a.gt_out = r.gt_out;
  finalize_px(a, p);
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" {

int cmx_aug_resize_u8(const uint8_t* src, int h, int w, int C, uint8_t* dst, int oh, int ow, int nearest, int mirror,
                      int clip_max, hipStream_t s) {
  CMX_REQUIRE(src && dst && h > 0 && w > 0 && oh > 0 && ow > 0, CMX_ERR_SHAPE, "aug_resize: %dx%d -> %dx%d", h, w,
              oh, ow);
  CMX_REQUIRE(C == 1 || C == 3, CMX_ERR_SHAPE, "aug_resize: C=%d (1 or 3)", C);
  CMX_REQUIRE(clip_max < 256, CMX_ERR_ARG, "aug_resize: clip_max %d", clip_max);
  // cv2: inv_scale = dsize / ssize, scale = 1 / inv_scale (double)
  const double sx = 1.0 / ((double)ow / w), sy = 1.0 / ((double)oh / h);
  const long n = (long)oh * ow;
  if (C == 1)
    hipLaunchKernelGGL((resize_u8_kernel<1>), dim3(nblk(n)), dim3(256), 0, s, src, h, w, dst, oh, ow, nearest, mirror,
                       clip_max, sx, sy);
  else
    hipLaunchKernelGGL((resize_u8_kernel<3>), dim3(nblk(n)), dim3(256), 0, s, src, h, w, dst, oh, ow, nearest, mirror,
                       clip_max, sx, sy);
  return cmx_check_launch("aug_resize");
}

int cmx_aug_color_jitter_u8(uint8_t* img, int h, int w, float bf, float sf, float hadd, hipStream_t s) {
  CMX_REQUIRE(img && h > 0 && w > 0, CMX_ERR_SHAPE, "aug_color_jitter: %dx%d", h, w);
  const long n = (long)h * w;
  hipLaunchKernelGGL(jitter_kernel, dim3(nblk(n)), dim3(256), 0, s, img, n, bf, sf, hadd);
  return cmx_check_launch("aug_color_jitter");
}

int cmx_aug_blur5_u8(const uint8_t* src, uint8_t* dst, int h, int w, int C, hipStream_t s) {
  CMX_REQUIRE(src && dst && src != dst && h >= 3 && w >= 3 && C > 0 && C <= 4, CMX_ERR_SHAPE,
              "aug_blur5: %dx%dx%d (needs >= 3x3, out of place)", h, w, C);
  hipLaunchKernelGGL(blur5_kernel, dim3(nblk((long)h * w)), dim3(256), 0, s, src, dst, h, w, C);
  return cmx_check_launch("aug_blur5");
}

int cmx_aug_finalize(const uint8_t* rgb, const uint8_t* x, const uint8_t* gt, int h, int w, int oh, int ow, int bx1,
                     int by1, int bx2, int by2, int background, double m0, double m1, double m2, double s0, double s1,
                     double s2, float* rgb_out, float* x_out, int64_t* gt_out, hipStream_t s) {
  CMX_REQUIRE(rgb && x && gt && rgb_out && x_out && gt_out && h > 0 && w > 0 && oh > 0 && ow > 0, CMX_ERR_SHAPE,
              "aug_finalize: %dx%d -> %dx%d", h, w, oh, ow);
  FinArgs a;
  a.rgb = rgb; a.x = x; a.gt = gt;
  a.h = h; a.w = w; a.oh = oh; a.ow = ow;
  a.bx1 = bx1; a.by1 = by1; a.bx2 = bx2; a.by2 = by2; a.background = background;
  a.sx = 1.0 / ((double)ow / w); a.sy = 1.0 / ((double)oh / h);
  a.isx = a.sx; a.isy = a.sy;
  a.mean[0] = m0; a.mean[1] = m1; a.mean[2] = m2;
  a.std[0] = s0; a.std[1] = s1; a.std[2] = s2;
  a.rgb_out = rgb_out; a.x_out = x_out; a.gt_out = gt_out;
  hipLaunchKernelGGL(finalize_kernel, dim3(nblk((long)oh * ow)), dim3(256), 0, s, a);
  return cmx_check_launch("aug_finalize");
}

int cmx_aug_batch(const int64_t* table, int B, int max_sh, int max_sw, int oh, int ow, int clip_max, int background,
                  double m0, double m1, double m2, double s0, double s1, double s2, hipStream_t s) {
  CMX_REQUIRE(table && B > 0 && B <= 65535 && max_sh > 0 && max_sw > 0 && oh > 0 && ow > 0, CMX_ERR_SHAPE,
              "aug_batch: B=%d max %dx%d -> %dx%d", B, max_sh, max_sw, oh, ow);
  CMX_REQUIRE(clip_max < 256, CMX_ERR_ARG, "aug_batch: clip_max %d", clip_max);
  const unsigned gs = nblk((long)max_sh * max_sw);
  hipLaunchKernelGGL(resize_batch_kernel, dim3(gs, B, 3), dim3(256), 0, s, table, clip_max);
  hipLaunchKernelGGL(jitter_batch_kernel, dim3(gs, B), dim3(256), 0, s, table);
  hipLaunchKernelGGL(blur_batch_kernel, dim3(gs, B), dim3(256), 0, s, table);
  hipLaunchKernelGGL(finalize_batch_kernel, dim3(nblk((long)oh * ow), B), dim3(256), 0, s, table, oh, ow, background,
                     m0, m1, m2, s0, s1, s2);
  return cmx_check_launch("aug_batch");
}

}  // extern "C"

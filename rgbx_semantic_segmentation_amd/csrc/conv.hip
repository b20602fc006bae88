// Convolution support for the OverlapPatchEmbed convs and the SRA spatial-reduction conv.
//
// Replaces  OverlapPatchEmbed.proj  (Conv2d k7/s4/p3 and k3/s2/p1, dual_segformer.py:196-197)
// and  Attention.sr  (Conv2d kR/sR, :95-96, a non-overlapping patchify) as
//   cols = im2col(x)  ->  GEMM with the weight (stored tap-major: (Cout, kh, kw, Cin))
// on token-major NHWC activations.  Backward dX = col2im(dCols) is a gather over the
// (kh, kw) taps that read each input pixel, so it needs no atomics.
//
// cols row = one output pixel (n, oy, ox); column = (kh*KW + kw)*C + c, row stride ldc
// (>= KH*KW*C, padding columns written as zero).  Output spatial size follows
// torch.nn.Conv2d floor semantics: Ho = (H + 2p - KH)/s + 1.
#include "cmx_common.h"

template <typename T>
__global__ void im2col_nhwc_kernel(const T* __restrict__ x, T* __restrict__ cols, int NI, int H, int W,
                                   int C, int KH, int KW, int stride, int pad, int Ho, int Wo, long ldc) {
  constexpr int V = VecT<T>::N;
  const int CPT = C / V;                       // chunks per tap
  const int taps = KH * KW;
  const long total = (long)NI * Ho * Wo * taps * CPT;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int ch = i % CPT;
    const int tap = (i / CPT) % taps;
    const int row = i / (CPT * taps);
    const int ox = row % Wo;
    const int oy = (row / Wo) % Ho;
    const int n = row / (Wo * Ho);
    const int iy = oy * stride - pad + tap / KW;
    const int ix = ox * stride - pad + tap % KW;
    float v[V];
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      load_vec<T>(x + (((long)n * H + iy) * W + ix) * C + ch * V, v);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = 0.f;
    }
    store_vec<T>(cols + row * ldc + (long)tap * C + ch * V, v);
  }
}

// zero the padding columns [K, ldc) of every row
template <typename T>
__global__ void zero_pad_cols_kernel(T* __restrict__ cols, long rows, int K, long ldc) {
  const int padw = (int)(ldc - K);
  const long total = rows * padw;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x)
    cols[(i / padw) * ldc + K + i % padw] = from_f32<T>(0.f);
}

// NCHW fp32 image -> cols in (c, kh, kw) order (= reference weight flatten order).  One thread
// per 8 consecutive columns of one row (ldc % 8 == 0, host-checked): the row and the first
// column are decoded once, the next 7 columns step (kw, kh, c) incrementally, and the 8 values
// leave as one 16-B (bf16) / two 16-B (fp32) stores.  The gathers hit the 7.4 MB image in L2.
template <typename T>
__global__ __launch_bounds__(256) void im2col_nchw_kernel(const float* __restrict__ x, T* __restrict__ cols, int NI,
                                                          int C, int H, int W, int KH, int KW, int stride, int pad,
                                                          int Ho, int Wo, long ldc, const float* __restrict__ x2,
                                                          int nsplit) {
  const int K = C * KH * KW;
  const int cpr = (int)(ldc / 8);
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)NI * Ho * Wo * cpr) return;
  const long row = i / cpr;
  const int k0 = (int)(i - row * cpr) * 8;
  const int ox = (int)(row % Wo);
  const int oy = (int)((row / Wo) % Ho);
  const int n = (int)(row / ((long)Wo * Ho));
  int c = k0 / (KH * KW), kh = (k0 / KW) % KH, kw = k0 % KW;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = 0.f;
    if (k0 + j < K) {
      const int iy = oy * stride - pad + kh, ix = ox * stride - pad + kw;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W)
        t = n < nsplit ? x[(((long)n * C + c) * H + iy) * W + ix] : x2[(((long)(n - nsplit) * C + c) * H + iy) * W + ix];
    }
    v[j] = t;
    if (++kw == KW) {
      kw = 0;
      if (++kh == KH) { kh = 0; ++c; }
    }
  }
  T* o = cols + row * ldc + k0;
  store_vec<T>(o, v);
  if constexpr (sizeof(T) == 4) store_vec<T>(o + 4, v + 4);
}

template <typename T>
__global__ void col2im_nhwc_kernel(const T* __restrict__ cols, T* __restrict__ dx, int NI, int H, int W,
                                   int C, int KH, int KW, int stride, int pad, int Ho, int Wo, long ldc) {
  constexpr int V = VecT<T>::N;
  const int CPR = C / V;
  const long total = (long)NI * H * W * CPR;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int ch = i % CPR;
    const int pix = i / CPR;
    const int x = pix % W;
    const int y = (pix / W) % H;
    const int n = pix / (W * H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int ty = y + pad - kh;
      if (ty < 0 || ty % stride) continue;
      const int oy = ty / stride;
      if (oy >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tx = x + pad - kw;
        if (tx < 0 || tx % stride) continue;
        const int ox = tx / stride;
        if (ox >= Wo) continue;
        float v[V];
        load_vec<T>(cols + (((long)n * Ho + oy) * Wo + ox) * ldc + (long)(kh * KW + kw) * C + ch * V, v);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += v[j];
      }
    }
    store_vec<T>(dx + pix * C + ch * V, acc);
  }
}

static unsigned grid_for(long total) {
  const unsigned g = cdiv(total, 256);
  return g < 16384 ? (g > 0 ? g : 1) : 16384;
}

extern "C" {

int cmx_im2col_nhwc(const void* x, void* cols, int NI, int H, int W, int C, int KH, int KW, int stride, int pad,
                    int Ho, int Wo, int64_t ldc, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && ldc >= (long)KH * KW * C && ldc % V == 0, CMX_ERR_SHAPE,
              "im2col_nhwc: C=%d ldc=%ld", C, (long)ldc);
  CMX_REQUIRE(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1, CMX_ERR_SHAPE,
              "im2col_nhwc: output size mismatch");
  const long rows = (long)NI * Ho * Wo;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(im2col_nhwc_kernel<T>, dim3(grid_for(rows * KH * KW * (C / V))), dim3(256), 0, s,
                       (const T*)x, (T*)cols, NI, H, W, C, KH, KW, stride, pad, Ho, Wo, (long)ldc);
    if (ldc > (long)KH * KW * C)
      hipLaunchKernelGGL(zero_pad_cols_kernel<T>, dim3(grid_for(rows * (ldc - KH * KW * C))), dim3(256), 0, s,
                         (T*)cols, rows, KH * KW * C, (long)ldc);
  });
  return cmx_check_launch("im2col_nhwc");
}

int cmx_im2col_nchw2_f32(const float* x, const float* x2, int nsplit, void* cols, int NI, int C, int H, int W, int KH,
                         int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t s);

int cmx_im2col_nchw_f32(const float* x, void* cols, int NI, int C, int H, int W, int KH, int KW, int stride,
                        int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t s) {
  return cmx_im2col_nchw2_f32(x, x, NI, cols, NI, C, H, W, KH, KW, stride, pad, Ho, Wo, ldc, dtype, s);
}

// images n < nsplit from x, the rest from x2 (the RGB and X batches of EncoderDecoder.forward,
// builder.py:240-253, without concatenating them first)
int cmx_im2col_nchw2_f32(const float* x, const float* x2, int nsplit, void* cols, int NI, int C, int H, int W, int KH,
                         int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t s) {
  CMX_REQUIRE(x && x2 && nsplit >= 0 && nsplit <= NI, CMX_ERR_ARG, "im2col_nchw2: nsplit %d of %d", nsplit, NI);
  CMX_REQUIRE(ldc >= (long)KH * KW * C && ldc % 8 == 0, CMX_ERR_SHAPE, "im2col_nchw: ldc %ld (>= K, multiple of 8)",
              (long)ldc);
  CMX_REQUIRE(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1, CMX_ERR_SHAPE,
              "im2col_nchw: output size mismatch");
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(im2col_nchw_kernel<T>, dim3((unsigned)(((long)NI * Ho * Wo * (ldc / 8) + 255) / 256)), dim3(256),
                       0, s, x,
                       (T*)cols, NI, C, H, W, KH, KW, stride, pad, Ho, Wo, (long)ldc, x2, nsplit);
  });
  return cmx_check_launch("im2col_nchw");
}

int cmx_col2im_nhwc(const void* cols, void* dx, int NI, int H, int W, int C, int KH, int KW, int stride, int pad,
                    int Ho, int Wo, int64_t ldc, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && ldc % V == 0, CMX_ERR_SHAPE, "col2im_nhwc: C=%d", C);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(col2im_nhwc_kernel<T>, dim3(grid_for((long)NI * H * W * (C / V))), dim3(256), 0, s,
                       (const T*)cols, (T*)dx, NI, H, W, C, KH, KW, stride, pad, Ho, Wo, (long)ldc);
  });
  return cmx_check_launch("col2im_nhwc");
}

}  // extern "C"

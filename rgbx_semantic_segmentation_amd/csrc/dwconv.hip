// Depthwise 3x3 (pad 1, stride 1) convolution + bias + activation on token-major NHWC.
//
// Replaces  DWConv.forward + act  of Mix-FFN (dual_segformer.py:27-33, 67-71:
//   x.permute(0,2,1).reshape(B,C,H,W) -> Conv2d(C,C,3,1,1,groups=C) -> flatten/transpose -> GELU)
// and the DW3x3 + ReLU of ChannelEmbed (net_utils.py:315-318).  No NCHW round trip: the
// channel dim is contiguous, each lane owns one 16-byte channel vector of one pixel.
//
// Images: NI = G*B images of H x W x C; image n belongs to group n / imgs_per_group (the
// RGB and X streams carry separate weights).  w: (G, C, 9) fp32, b: (G, C) fp32.
// Algorithmic bytes (fwd): read h once + write a once (the 3x3 halo re-reads hit L1/L2).
#include "cmx_common.h"

template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ out,
                                                     int NI, int ipg, int H, int W, int C, int act,
                                                     int flip) {
  constexpr int V = VecT<T>::N;
  const int CPR = C / V;
  const long total = (long)NI * H * W * CPR;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int ch = idx % CPR;
    const long pix = idx / CPR;
    const int x = pix % W;
    const int y = (pix / W) % H;
    const int n = pix / ((long)W * H);
    const int g = n / ipg;
    const int c0 = ch * V;
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = b ? b[(long)g * C + c0 + j] : 0.f;
    const T* img = h + (long)n * H * W * C + c0;
    const float* wg = w + ((long)g * C + c0) * 9;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int yy = y + i - 1;
      if (yy < 0 || yy >= H) continue;
#pragma unroll
      for (int jx = 0; jx < 3; ++jx) {
        const int xx = x + jx - 1;
        if (xx < 0 || xx >= W) continue;
        float v[V];
        load_vec<T>(img + ((long)yy * W + xx) * C, v);
        const int tap = flip ? (8 - (i * 3 + jx)) : (i * 3 + jx);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += wg[j * 9 + tap] * v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = act_fwd(acc[j], act);
    store_vec<T>(out + pix * C + c0, acc);
  }
}

// dz = da * act'(z) with z recomputed; partial sums of dW (9 taps) and db per block.
// Block = 32 channel-chunk lanes (x) x 8 pixel slots (y); blockIdx.y = chunk tile,
// blockIdx.x = pixel range of group blockIdx.z.
template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_dz_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ b, T* __restrict__ dz,
                                                        float* __restrict__ ws, int ipg, int H, int W, int C,
                                                        int act, int pix_per_blk) {
  constexpr int V = VecT<T>::N;
  __shared__ float red[4][32 * V * 10];
  const int CPR = C / V;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int ch = blockIdx.y * 32 + tx;
  const bool live = ch < CPR;
  const int g = blockIdx.z;
  const long gpix = (long)ipg * H * W;
  const long p0 = (long)blockIdx.x * pix_per_blk;
  const long p1 = min(gpix, p0 + pix_per_blk);
  const int c0 = ch * V;
  float aw[V][9], ab[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    ab[j] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) aw[j][t] = 0.f;
  }
  if (live) {
    const float* wg = w + ((long)g * C + c0) * 9;
    for (long p = p0 + ty; p < p1; p += 8) {
      const int x = p % W;
      const int y = (p / W) % H;
      const long nimg = (long)g * ipg + p / ((long)W * H);
      const T* img = h + nimg * H * W * C + c0;
      float hv[9][V];
      float z[V];
#pragma unroll
      for (int j = 0; j < V; ++j) z[j] = b ? b[(long)g * C + c0 + j] : 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          load_vec<T>(img + ((long)yy * W + xx) * C, hv[t]);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) hv[t][j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) z[j] += wg[j * 9 + t] * hv[t][j];
      }
      const long pofs = (nimg * H * W + (long)y * W + x) * C + c0;
      float d[V];
      load_vec<T>(da + pofs, d);
#pragma unroll
      for (int j = 0; j < V; ++j) d[j] *= act_grad(z[j], act);
      store_vec<T>(dz + pofs, d);
      // accumulate with the value as stored (bf16-rounded) so dW matches dz exactly
      float dq[V];
      load_vec<T>(dz + pofs, dq);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        ab[j] += dq[j];
#pragma unroll
        for (int t = 0; t < 9; ++t) aw[j][t] += dq[j] * hv[t][j];
      }
    }
  }
  // combine the two pixel slots of each wave, then the 4 waves through LDS
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    ab[j] += __shfl_xor(ab[j], 32, 64);
#pragma unroll
    for (int t = 0; t < 9; ++t) aw[j][t] += __shfl_xor(aw[j][t], 32, 64);
  }
  if ((threadIdx.x & 63) < 32) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
#pragma unroll
      for (int t = 0; t < 9; ++t) red[wv][(tx * V + j) * 10 + t] = aw[j][t];
      red[wv][(tx * V + j) * 10 + 9] = ab[j];
    }
  }
  __syncthreads();
  float* out = ws + ((long)g * gridDim.x + blockIdx.x) * (long)C * 10;
  for (int e = threadIdx.x; e < 32 * V * 10; e += 256) {
    const int c = blockIdx.y * 32 * V + e / 10;
    if (c < C) out[(long)c * 10 + e % 10] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
  }
}

// dw[g][c][t] = sum_b ws[g][b][c][t], db[g][c] = sum_b ws[g][b][c][9]
__global__ void dw_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, float* __restrict__ db,
                                 int G, int nblk, int C, int accumulate) {
  const long total = (long)G * C * 10;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int e = i % (C * 10);
    const int g = i / (C * 10);
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += ws[((long)g * nblk + k) * C * 10 + e];
    const int c = e / 10, t = e % 10;
    float* o = t < 9 ? &dw[((long)g * C + c) * 9 + t] : (db ? &db[(long)g * C + c] : nullptr);
    if (o) *o = accumulate ? *o + s : s;
  }
}

static int dw_pix_per_blk(long gpix) {
  long ppb = 256;
  while (gpix / ppb > 192 && ppb < 4096) ppb *= 2;
  return (int)ppb;
}

extern "C" {

int cmx_dwconv3x3_fwd(const void* h, const float* w, const float* b, void* out, int NI, int imgs_per_group,
                      int H, int W, int C, int act, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_fwd: C=%d", C);
  const long total = (long)NI * H * W * (C / V);
  const unsigned grid = cdiv(total, 256) < 16384 ? cdiv(total, 256) : 16384;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(grid), dim3(256), 0, s, (const T*)h, w, b, (T*)out, NI,
                       imgs_per_group, H, W, C, act, 0);
  });
  return cmx_check_launch("dwconv_fwd");
}

size_t cmx_dwconv3x3_bwd_workspace(int NI, int imgs_per_group, int H, int W, int C) {
  const int G = NI / imgs_per_group;
  const long gpix = (long)imgs_per_group * H * W;
  const int ppb = dw_pix_per_blk(gpix);
  return (size_t)G * ((gpix + ppb - 1) / ppb) * C * 10 * sizeof(float);
}

// da: upstream grad of the activation output; dz (workspace-sized like h, dtype) receives
// da * act'(z); dh = conv^T(dz); dw (G,C,9), db (G,C) fp32 (db may be NULL).
int cmx_dwconv3x3_bwd(const void* da, const void* h, const float* w, const float* b, void* dz, void* dh,
                      float* dw, float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C,
                      int act, int accumulate, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_bwd: C=%d", C);
  const int G = NI / imgs_per_group;
  const long gpix = (long)imgs_per_group * H * W;
  const int ppb = dw_pix_per_blk(gpix);
  const int nblk = (int)((gpix + ppb - 1) / ppb);
  const int CPR = C / V;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(dw_bwd_dz_kernel<T>, dim3(nblk, cdiv(CPR, 32), G), dim3(256), 0, s, (const T*)da,
                       (const T*)h, w, b, (T*)dz, workspace, imgs_per_group, H, W, C, act, ppb);
    if (dh) {
      const long total = (long)NI * H * W * CPR;
      const unsigned grid = cdiv(total, 256) < 16384 ? cdiv(total, 256) : 16384;
      hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(grid), dim3(256), 0, s, (const T*)dz, w, (const float*)nullptr,
                         (T*)dh, NI, imgs_per_group, H, W, C, (int)ACT_NONE, 1);
    }
  });
  const long tot = (long)G * C * 10;
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(cdiv(tot, 256) < 4096 ? cdiv(tot, 256) : 4096), dim3(256), 0, s,
                     workspace, dw, db, G, nblk, C, accumulate);
  return cmx_check_launch("dwconv_bwd");
}

}  // extern "C"

// Bilinear resampling, align_corners=False, with PyTorch's source-index rule
//   src = max(0, (dst + 0.5) * in/out - 0.5); i0 = floor(src); i1 = min(i0 + 1, in - 1)
// Replaces F.interpolate in DecoderHead (MLPDecoder.py:67-73: c2..c4 up to the 1/4 grid,
// written straight into the channel slices of the 4*E concat buffer, no torch.cat) and the
// final logits upsample of EncoderDecoder.encode_decode (builder.py:233).
// The backward (adjoint) is separable: two 1-D gather passes (no atomics), the first along
// x into an fp32 temp, the second along y, each output gathering the contiguous range of
// destination indices whose stencil touches it.
#include "cmx_common.h"

namespace {

__device__ __forceinline__ void src_index(int dst, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  cmx_bilin_src(dst, scale, in, i0, i1, l0, l1);
}

// in (NB, Hi, Wi, C) dense; out pixel p at out + ((n*Ho + y)*Wo + x)*ops + c
template <typename T>
__global__ void bilinear_fwd_nhwc_kernel(const T* __restrict__ in, T* __restrict__ out, int NB, int Hi, int Wi, int Ho,
                                         int Wo, int C, long ops, float sh, float sw) {
  constexpr int V = VecT<T>::N;
  const int CPR = C / V;
  const long total = (long)NB * Ho * Wo * CPR;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int ch = i % CPR;
    const int pix = i / CPR;
    const int x = pix % Wo;
    const int y = (pix / Wo) % Ho;
    const int n = pix / (Wo * Ho);
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    src_index(y, sh, Hi, y0, y1, ly0, ly1);
    src_index(x, sw, Wi, x0, x1, lx0, lx1);
    const T* base = in + (long)n * Hi * Wi * C + ch * V;
    float a[V], b[V], c[V], d[V], o[V];
    load_vec<T>(base + ((long)y0 * Wi + x0) * C, a);
    load_vec<T>(base + ((long)y0 * Wi + x1) * C, b);
    load_vec<T>(base + ((long)y1 * Wi + x0) * C, c);
    load_vec<T>(base + ((long)y1 * Wi + x1) * C, d);
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = ly0 * (lx0 * a[j] + lx1 * b[j]) + ly1 * (lx0 * c[j] + lx1 * d[j]);
    store_vec<T>(out + pix * ops + ch * V, o);
  }
}

// NHWC (dtype) -> NCHW fp32 (inference logits); thread per output element, x fastest
template <typename T>
__global__ void bilinear_fwd_nchw_kernel(const T* __restrict__ in, float* __restrict__ out, int NB, int Hi, int Wi,
                                         int Ho, int Wo, int C, float sh, float sw) {
  const long total = (long)NB * C * Ho * Wo;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int x = i % Wo;
    const int y = (i / Wo) % Ho;
    const int c = (i / (Wo * Ho)) % C;
    const int n = i / (Wo * Ho * C);
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    src_index(y, sh, Hi, y0, y1, ly0, ly1);
    src_index(x, sw, Wi, x0, x1, lx0, lx1);
    const T* base = in + (long)n * Hi * Wi * C + c;
    const float a = to_f32(base[((long)y0 * Wi + x0) * C]), b = to_f32(base[((long)y0 * Wi + x1) * C]);
    const float cc = to_f32(base[((long)y1 * Wi + x0) * C]), d = to_f32(base[((long)y1 * Wi + x1) * C]);
    out[i] = ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * cc + lx1 * d);
  }
}

// 1-D adjoint along one axis: in (P, Lo, Q) with strides (sp, so, 1) -> out (P, Li, Q) dense;
// out[p][i][q] = alpha * sum_{o : i0(o)==i or i1(o)==i} w(o, i) * in[p][o][q]
template <typename TI, typename TO>
__global__ void bilinear_adj_kernel(const TI* __restrict__ in, TO* __restrict__ out, long P, int Lo, int Li, int Q,
                                    long sp, long so, float scale, const float* __restrict__ a1,
                                    const float* __restrict__ a2, float alpha0) {
  const float alpha = alpha0 * (a1 ? *a1 : 1.f) * (a2 ? *a2 : 1.f);
  const long total = P * Li * Q;
  const float inv = 1.f / scale;  // out/in
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < (int)total; e += gridDim.x * blockDim.x) {
    const int q = e % Q;
    const int i = (e / Q) % Li;
    const int p = e / (Q * Li);
    int olo = (int)floorf((i - 1.5f) * inv) - 1;
    int ohi = (int)ceilf((i + 1.5f) * inv) + 1;
    if (olo < 0) olo = 0;
    if (ohi > Lo - 1) ohi = Lo - 1;
    float acc = 0.f;
    for (int o = olo; o <= ohi; ++o) {
      int i0, i1;
      float l0, l1;
      src_index(o, scale, Li, i0, i1, l0, l1);
      float w = 0.f;
      if (i0 == i) w += l0;
      if (i1 == i) w += l1;
      if (w != 0.f) acc += w * to_f32(in[p * sp + (long)o * so + q]);
    }
    out[e] = from_f32<TO>(alpha * acc);
  }
}

// same, 8 consecutive q per thread (16-B bf16 / 32-B fp32 loads): Q % 8 == 0, aligned rows
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void bilinear_adj8_kernel(const TI* __restrict__ in, TO* __restrict__ out, long P,
                                                            int Lo, int Li, int Q, long sp, long so, float scale,
                                                            const float* __restrict__ a1, const float* __restrict__ a2,
                                                            float alpha0) {
  const float alpha = alpha0 * (a1 ? *a1 : 1.f) * (a2 ? *a2 : 1.f);
  const int Q8 = Q >> 3;
  const long total = P * Li * Q8;
  const float inv = 1.f / scale;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e % Q8) * 8;
    const int i = (int)((e / Q8) % Li);
    const long p = e / ((long)Q8 * Li);
    int olo = (int)floorf((i - 1.5f) * inv) - 1;
    int ohi = (int)ceilf((i + 1.5f) * inv) + 1;
    if (olo < 0) olo = 0;
    if (ohi > Lo - 1) ohi = Lo - 1;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int o = olo; o <= ohi; ++o) {
      int i0, i1;
      float l0, l1;
      src_index(o, scale, Li, i0, i1, l0, l1);
      float w = 0.f;
      if (i0 == i) w += l0;
      if (i1 == i) w += l1;
      if (w != 0.f) {
        float v[8];
        const TI* src = in + p * sp + (long)o * so + q;
        load_vec<TI>(src, v);
        if constexpr (sizeof(TI) == 4) load_vec<TI>(src + 4, v + 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += w * v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= alpha;
    TO* dst = out + ((p * Li + i) * (long)Q + q);
    store_vec<TO>(dst, acc);
    if constexpr (sizeof(TO) == 4) store_vec<TO>(dst + 4, acc + 4);
  }
}

unsigned gridcap(long total) {
  const unsigned g = cdiv(total, 256);
  return g < 16384 ? (g ? g : 1) : 16384;
}
// ---------------------------------------------------------------- decoder upsample-sum
// U (B, H, W, C) = bias + sum_s up_s(z_s), z_s (B, h_s, w_s, C): the three upsampled branches of
// DecoderHead (MLPDecoder.py:67-73, here already multiplied by their linear_fuse slices) summed in
// one pass, so the c1 GEMM adds U as a plain residual.  A workgroup owns one output row and a
// 64-channel slice: it stages each source's two contributing rows, already y-interpolated (fp32,
// (w_0 + w_1 + w_2) x 64 floats), in LDS -- one coalesced read of each source row -- and every
// output 8-vector then takes 2 taps per source from LDS.
constexpr int U3_CS = 64;
constexpr int U3_NI = 5;                           // staged items per thread: sum of widths x 8 <= 1280
template <typename T>
__global__ __launch_bounds__(256) void up3_add_kernel(const T* __restrict__ z0, const T* __restrict__ z1,
                                                      const T* __restrict__ z2, int h0, int w0, int h1, int w1, int h2,
                                                      int w2, const float* __restrict__ bias, T* __restrict__ out,
                                                      int H, int W, int C, int nsrc) {
  extern __shared__ float srow[];                  // [source][x][64 channels], fp32
  const int cslices = C / U3_CS;
  const int cs = blockIdx.x % cslices, Y = (blockIdx.x / cslices) % H, b = blockIdx.x / (cslices * H);
  const int c0 = cs * U3_CS;
  const T* zs[3] = {z0, z1, z2};
  const int hs[3] = {h0, h1, h2}, ws[3] = {w0, w1, w2};
  int off[4];
  off[0] = 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) off[q + 1] = off[q] + (q < nsrc ? ws[q] * U3_CS : 0);
  // stage: y-interpolated source rows, 8 channels per item.  The items of all sources form one
  // index space; every load of the thread is issued before the first LDS store (U3_NI per thread)
  constexpr int VPX = U3_CS / 8;
  int rowa[3], rowb[3];
  float wla[3], wlb[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (q < nsrc) {
      src_index(Y, (float)hs[q] / H, hs[q], rowa[q], rowb[q], wla[q], wlb[q]);
    } else {
      rowa[q] = rowb[q] = 0;
      wla[q] = wlb[q] = 0.f;
    }
  }
  const int nitems = off[3] / 8;                   // sum_q w_q * VPX
  uint4 ga[U3_NI][VecT<T>::N == 8 ? 1 : 2], gb[U3_NI][VecT<T>::N == 8 ? 1 : 2];
#pragma unroll
  for (int i = 0; i < U3_NI; ++i) {
    const int e = threadIdx.x + i * 256;
    if (e < nitems) {
      const int q = e * 8 < off[1] ? 0 : (e * 8 < off[2] ? 1 : 2);
      const int el = e - off[q] / 8;
      const int x = el / VPX, v8 = (el % VPX) * 8;
      const T* ra = zs[q] + (((long)b * hs[q] + rowa[q]) * ws[q] + x) * C + c0 + v8;
      const T* rb = zs[q] + (((long)b * hs[q] + rowb[q]) * ws[q] + x) * C + c0 + v8;
#pragma unroll
      for (int h = 0; h < (VecT<T>::N == 8 ? 1 : 2); ++h) {
        ga[i][h] = reinterpret_cast<const uint4*>(ra)[h];
        gb[i][h] = reinterpret_cast<const uint4*>(rb)[h];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < U3_NI; ++i) {
    const int e = threadIdx.x + i * 256;
    if (e < nitems) {
      const int q = e * 8 < off[1] ? 0 : (e * 8 < off[2] ? 1 : 2);
      float a[8], bb[8];
      if constexpr (VecT<T>::N == 8) {
        load_vec<T>(reinterpret_cast<const T*>(&ga[i][0]), a);
        load_vec<T>(reinterpret_cast<const T*>(&gb[i][0]), bb);
      } else {
        load_vec<T>(reinterpret_cast<const T*>(&ga[i][0]), a);
        load_vec<T>(reinterpret_cast<const T*>(&ga[i][1]), a + 4);
        load_vec<T>(reinterpret_cast<const T*>(&gb[i][0]), bb);
        load_vec<T>(reinterpret_cast<const T*>(&gb[i][1]), bb + 4);
      }
      const float la = wla[q], lb = wlb[q];
      float4* d = reinterpret_cast<float4*>(srow + e * 8);                    // 16-B LDS stores
      d[0] = make_float4(la * a[0] + lb * bb[0], la * a[1] + lb * bb[1], la * a[2] + lb * bb[2], la * a[3] + lb * bb[3]);
      d[1] = make_float4(la * a[4] + lb * bb[4], la * a[5] + lb * bb[5], la * a[6] + lb * bb[6], la * a[7] + lb * bb[7]);
    }
  }
  __syncthreads();
  // outputs: 8 channels per item, x-interpolation from LDS
  T* orow = out + (((long)b * H + Y) * W) * C + c0;
  for (int e = threadIdx.x; e < W * (U3_CS / 8); e += blockDim.x) {
    const int x = e / (U3_CS / 8), v8 = (e % (U3_CS / 8)) * 8;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = bias ? bias[c0 + v8 + k] : 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (q >= nsrc) continue;
      int x0, x1;
      float l0, l1;
      src_index(x, (float)ws[q] / W, ws[q], x0, x1, l0, l1);
      const float4* p0 = reinterpret_cast<const float4*>(srow + off[q] + x0 * U3_CS + v8);
      const float4* p1 = reinterpret_cast<const float4*>(srow + off[q] + x1 * U3_CS + v8);
      const float4 a0 = p0[0], a1 = p0[1], b0 = p1[0], b1 = p1[1];
      acc[0] += l0 * a0.x + l1 * b0.x; acc[1] += l0 * a0.y + l1 * b0.y;
      acc[2] += l0 * a0.z + l1 * b0.z; acc[3] += l0 * a0.w + l1 * b0.w;
      acc[4] += l0 * a1.x + l1 * b1.x; acc[5] += l0 * a1.y + l1 * b1.y;
      acc[6] += l0 * a1.z + l1 * b1.z; acc[7] += l0 * a1.w + l1 * b1.w;
    }
    store_vec<T>(orow + (long)x * C + v8, acc);
    if constexpr (sizeof(T) == 4) store_vec<T>(orow + (long)x * C + v8 + 4, acc + 4);
  }
}

// ---------------------------------------------------------------- decoder adjoint (3 grids)
// The backward of the three upsampled branches: dY_s = up_s^T dZ for s = 0..2 from ONE read of
// dZ (B, H, W, C).  Pass x (adj3_x_kernel): a workgroup owns one full-res row and a 128-channel
// slice, stages the row in LDS, builds each grid's tap table for the row (output column i <- the
// full-res columns whose bilinear pair touches i, with their weights; A3_TAPS_s slots, zero
// padded), and writes the three x-adjoints (B*H, w_s, C) in fp32.  Pass y (adj3_y_kernel): the
// row adjoint of each, all three grids in one grid-stride launch.  (Replaces three pairs of
// cmx_bilinear_adjoint_1d launches that read dZ once per grid.)  Channel slice A3_CS = 128 for
// 16-bit rows, 64 for fp32 (the staged row stays within 64 KB).
__device__ __forceinline__ int a3_taps(int Lo, int Li) { return (2 * Lo + Li - 1) / Li + 3; }

template <typename T, int A3_CS>
__global__ __launch_bounds__(256) void adj3_x_kernel(const T* __restrict__ dz, float* __restrict__ t0,
                                                     float* __restrict__ t1, float* __restrict__ t2, int w0, int w1,
                                                     int w2, int W, int C, int nsrc) {
  extern __shared__ float a3_lds[];
  const int cslices = C / A3_CS;
  const long p = blockIdx.x / cslices;
  const int c0 = (blockIdx.x % cslices) * A3_CS;
  const int wsz[3] = {w0, w1, w2};
  float* outs[3] = {t0, t1, t2};
  int nt[3], toff[3], tot = 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    nt[q] = q < nsrc ? a3_taps(W, wsz[q]) : 0;
    toff[q] = tot;
    tot += q < nsrc ? wsz[q] * nt[q] : 0;
  }
  int* tap_o = reinterpret_cast<int*>(a3_lds);           // [tot]
  float* tap_w = a3_lds + tot;                            // [tot]
  T* row = reinterpret_cast<T*>(a3_lds + (2 * tot + 3) / 4 * 4);   // [W][A3_CS], 16-B aligned
  // tap tables: entry (i, j) = full-res column olo(i) + j and its weight on i (0 outside)
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (q >= nsrc) continue;
    const float scale = (float)wsz[q] / W, inv = (float)W / wsz[q];
    for (int e = threadIdx.x; e < wsz[q] * nt[q]; e += blockDim.x) {
      // o reaches column i iff src(o) in (i - 1, i + 1): o in ((i - 0.5) inv - 0.5, (i + 1.5) inv - 0.5),
      // 2 inv wide; the slots start one column early (rounding) and run a3_taps = ceil(2 inv) + 3
      const int i = e / nt[q], j = e % nt[q];
      int olo = (int)floorf((i - 0.5f) * inv - 0.5f) - 1;
      if (olo < 0) olo = 0;
      const int o = olo + j;
      float wgt = 0.f;
      if (o < W) {
        int i0, i1;
        float l0, l1;
        src_index(o, scale, wsz[q], i0, i1, l0, l1);
        if (i0 == i) wgt += l0;
        if (i1 == i) wgt += l1;
      }
      tap_o[toff[q] + e] = o < W ? o : 0;
      tap_w[toff[q] + e] = wgt;
    }
  }
  const T* src = dz + p * W * C + c0;
  for (int e = threadIdx.x; e < W * (A3_CS / 8); e += blockDim.x) {
    const int x = e / (A3_CS / 8), v8 = (e % (A3_CS / 8)) * 8;
    *reinterpret_cast<uint4*>(row + x * A3_CS + v8) = *reinterpret_cast<const uint4*>(src + (long)x * C + v8);
    if constexpr (sizeof(T) == 4)
      *reinterpret_cast<uint4*>(row + x * A3_CS + v8 + 4) = *reinterpret_cast<const uint4*>(src + (long)x * C + v8 + 4);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (q >= nsrc) continue;
    float* dst = outs[q] + p * wsz[q] * C + c0;
    for (int e = threadIdx.x; e < wsz[q] * (A3_CS / 8); e += blockDim.x) {
      const int i = e / (A3_CS / 8), v8 = (e % (A3_CS / 8)) * 8;
      const int* to = tap_o + toff[q] + i * nt[q];
      const float* tw = tap_w + toff[q] + i * nt[q];
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < nt[q]; ++j) {
        const float wgt = tw[j];
        float v[8];
        load_vec<T>(row + to[j] * A3_CS + v8, v);
        if constexpr (sizeof(T) == 4) load_vec<T>(row + to[j] * A3_CS + v8 + 4, v + 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += wgt * v[k];
      }
      float* d = dst + (long)i * C + v8;
      *reinterpret_cast<float4*>(d) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  }
}

// dY_s (B, h_s, w_s, C) = row adjoint of t_s (B, H, w_s, C) fp32, the three grids in one launch
template <typename T>
__global__ __launch_bounds__(256) void adj3_y_kernel(const float* __restrict__ t0, const float* __restrict__ t1,
                                                     const float* __restrict__ t2, T* __restrict__ y0,
                                                     T* __restrict__ y1, T* __restrict__ y2, int h0, int w0, int h1,
                                                     int w1, int h2, int w2, int B, int H, int C, int nsrc) {
  const int C8 = C / 8;
  const long n0 = (long)B * h0 * w0 * C8, n1 = nsrc > 1 ? (long)B * h1 * w1 * C8 : 0,
             n2 = nsrc > 2 ? (long)B * h2 * w2 * C8 : 0;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n0 + n1 + n2; e += (long)gridDim.x * blockDim.x) {
    const bool s0 = e < n0, s1 = !s0 && e < n0 + n1;
    const long f = s0 ? e : (s1 ? e - n0 : e - n0 - n1);
    const int hs = s0 ? h0 : (s1 ? h1 : h2), ws = s0 ? w0 : (s1 ? w1 : w2);
    const float* t = s0 ? t0 : (s1 ? t1 : t2);
    T* out = s0 ? y0 : (s1 ? y1 : y2);
    const int v8 = (int)(f % C8) * 8;
    const int i = (int)((f / C8) % ws);
    const int y = (int)((f / ((long)C8 * ws)) % hs);
    const int b = (int)(f / ((long)C8 * ws * hs));
    const float scale = (float)hs / H, inv = (float)H / hs;
    int olo = (int)floorf((y - 1.5f) * inv) - 1;
    int ohi = (int)ceilf((y + 1.5f) * inv) + 1;
    if (olo < 0) olo = 0;
    if (ohi > H - 1) ohi = H - 1;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int o = olo; o <= ohi; ++o) {
      int i0, i1;
      float l0, l1;
      src_index(o, scale, hs, i0, i1, l0, l1);
      const float wgt = (i0 == y ? l0 : 0.f) + (i1 == y ? l1 : 0.f);
      if (wgt != 0.f) {
        const float* r = t + (((long)b * H + o) * ws + i) * C + v8;
        const float4 a = *reinterpret_cast<const float4*>(r), c = *reinterpret_cast<const float4*>(r + 4);
        acc[0] += wgt * a.x; acc[1] += wgt * a.y; acc[2] += wgt * a.z; acc[3] += wgt * a.w;
        acc[4] += wgt * c.x; acc[5] += wgt * c.y; acc[6] += wgt * c.z; acc[7] += wgt * c.w;
      }
    }
    store_vec<T>(out + (((long)b * hs + y) * ws + i) * C + v8, acc);
    if constexpr (sizeof(T) == 4) store_vec<T>(out + (((long)b * hs + y) * ws + i) * C + v8 + 4, acc + 4);
  }
}

}  // namespace

extern "C" {

int cmx_bilinear_fwd_nhwc(const void* in, void* out, int NB, int Hi, int Wi, int Ho, int Wo, int C, int64_t out_pix_stride,
                          int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(C % V == 0 && out_pix_stride % V == 0, CMX_ERR_SHAPE, "bilinear_fwd_nhwc: C=%d", C);
  const float sh = (float)Hi / Ho, sw = (float)Wi / Wo;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bilinear_fwd_nhwc_kernel<T>, dim3(gridcap((long)NB * Ho * Wo * (C / V))), dim3(256), 0, s,
                       (const T*)in, (T*)out, NB, Hi, Wi, Ho, Wo, C, (long)out_pix_stride, sh, sw);
  });
  return cmx_check_launch("bilinear_fwd_nhwc");
}

int cmx_bilinear_fwd_nchw_f32(const void* in, float* out, int NB, int Hi, int Wi, int Ho, int Wo, int C, int dtype,
                              hipStream_t s) {
  const float sh = (float)Hi / Ho, sw = (float)Wi / Wo;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(bilinear_fwd_nchw_kernel<T>, dim3(gridcap((long)NB * C * Ho * Wo)), dim3(256), 0, s,
                       (const T*)in, out, NB, Hi, Wi, Ho, Wo, C, sh, sw);
  });
  return cmx_check_launch("bilinear_fwd_nchw");
}

// in/out dtypes independent (0 fp32, 1 bf16, 2 fp16); alpha = alpha0 * (*a1) * (*a2) (NULL -> 1)
int cmx_bilinear_adjoint_1d(const void* in, void* out, int64_t P, int Lo, int Li, int Q, int64_t sp, int64_t so,
                            const float* a1, const float* a2, float alpha0, int in_dtype, int out_dtype,
                            hipStream_t s) {
  const float scale = (float)Li / Lo;
  const int ei = in_dtype == 0 ? 4 : 2;
  const bool v8 = Q % 8 == 0 && sp % 8 == 0 && so % 8 == 0 && ((uintptr_t)in % (8 * ei)) == 0 &&
                  ((uintptr_t)out % 16) == 0;
  const unsigned grid = gridcap(v8 ? P * Li * (Q / 8) : P * Li * Q);
#define ADJ(TI, TO)                                                                                   \
  if (v8)                                                                                             \
    hipLaunchKernelGGL((bilinear_adj8_kernel<TI, TO>), dim3(grid), dim3(256), 0, s, (const TI*)in, (TO*)out, \
                       (long)P, Lo, Li, Q, (long)sp, (long)so, scale, a1, a2, alpha0);                 \
  else                                                                                                \
    hipLaunchKernelGGL((bilinear_adj_kernel<TI, TO>), dim3(grid), dim3(256), 0, s, (const TI*)in, (TO*)out, \
                       (long)P, Lo, Li, Q, (long)sp, (long)so, scale, a1, a2, alpha0)
  if (in_dtype == 0 && out_dtype == 0) ADJ(float, float);
  else if (in_dtype == 0 && out_dtype == 1) ADJ(float, bf16);
  else if (in_dtype == 1 && out_dtype == 0) ADJ(bf16, float);
  else if (in_dtype == 1 && out_dtype == 1) ADJ(bf16, bf16);
  else if (in_dtype == 0 && out_dtype == 2) ADJ(float, f16);
  else if (in_dtype == 2 && out_dtype == 0) ADJ(f16, float);
  else if (in_dtype == 2 && out_dtype == 2) ADJ(f16, f16);
  else { cmx_set_error("bilinear_adjoint: dtype"); return CMX_ERR_DTYPE; }
#undef ADJ
  return cmx_check_launch("bilinear_adjoint_1d");
}

// dY_s = up_s^T dZ for up to three grids (y_s NULL: absent): t_s (B*H, w_s, C) fp32 workspaces
int cmx_bilinear_adjoint3(const void* dz, float* t0, float* t1, float* t2, void* y0, void* y1, void* y2, int B, int H,
                          int W, int h0, int w0, int h1, int w1, int h2, int w2, int C, int dtype, hipStream_t s) {
  const int A3_CS = dtype == 0 ? 64 : 128;
  CMX_REQUIRE(dz && y0 && t0 && B > 0 && H > 0 && W > 0 && C % A3_CS == 0, CMX_ERR_SHAPE,
              "bilinear_adjoint3: C=%d (a multiple of %d)", C, A3_CS);
  const int n = y2 ? 3 : (y1 ? 2 : 1);
  CMX_REQUIRE((n < 2 || t1) && (n < 3 || t2), CMX_ERR_ARG, "bilinear_adjoint3: workspaces");
  const int ws[3] = {w0, w1, w2};
  long tot = 0;
  for (int q = 0; q < n; ++q) {
    CMX_REQUIRE(ws[q] > 0 && ws[q] <= W, CMX_ERR_SHAPE, "bilinear_adjoint3: grid %d width %d", q, ws[q]);
    tot += (long)ws[q] * ((2 * W + ws[q] - 1) / ws[q] + 3);
  }
  const size_t lds = (size_t)(2 * tot + 3) / 4 * 16 + (size_t)W * A3_CS * (dtype == 0 ? 4 : 2);
  CMX_REQUIRE(lds <= 64 * 1024, CMX_ERR_SHAPE, "bilinear_adjoint3: %zu B of LDS for W=%d", lds, W);
  const long ny = (long)B * (h0 * w0 + (n > 1 ? h1 * w1 : 0) + (n > 2 ? h2 * w2 : 0)) * (C / 8);
  CMX_DISPATCH(dtype, T, {
    if constexpr (sizeof(T) == 4)
      hipLaunchKernelGGL((adj3_x_kernel<T, 64>), dim3(B * H * (C / 64)), dim3(256), lds, s, (const T*)dz, t0, t1, t2, w0,
                         w1, w2, W, C, n);
    else
      hipLaunchKernelGGL((adj3_x_kernel<T, 128>), dim3(B * H * (C / 128)), dim3(256), lds, s, (const T*)dz, t0, t1, t2,
                         w0, w1, w2, W, C, n);
    hipLaunchKernelGGL(adj3_y_kernel<T>, dim3(gridcap(ny)), dim3(256), 0, s, (const float*)t0, (const float*)t1,
                       (const float*)t2, (T*)y0, (T*)y1, (T*)y2, h0, w0, h1, w1, h2, w2, B, H, C, n);
  });
  return cmx_check_launch("bilinear_adjoint3");
}

// U (B, H, W, C) = bias + sum of the bilinear upsamples of z0, z1, z2 (NULL: absent; bias NULL: 0)
int cmx_bilinear_up3_add(const void* z0, const void* z1, const void* z2, int B, int h0, int w0, int h1, int w1,
                         int h2, int w2, const float* bias, void* out, int H, int W, int C, int dtype, hipStream_t s) {
  const void* zz[3] = {z0, z1, z2};
  const int hh[3] = {h0, h1, h2}, ww[3] = {w0, w1, w2};
  const void* src[3] = {nullptr, nullptr, nullptr};
  int sh_[3] = {1, 1, 1}, sw_[3] = {1, 1, 1}, n = 0;
  for (int q = 0; q < 3; ++q) {
    if (!zz[q]) continue;
    CMX_REQUIRE(hh[q] > 0 && ww[q] > 0 && ((uintptr_t)zz[q] & 15) == 0, CMX_ERR_ARG, "bilinear_up3_add: source %d", q);
    src[n] = zz[q]; sh_[n] = hh[q]; sw_[n] = ww[q]; ++n;
  }
  CMX_REQUIRE(B > 0 && H > 0 && W > 0 && C % U3_CS == 0 && ((uintptr_t)out & 15) == 0, CMX_ERR_SHAPE,
              "bilinear_up3_add: C=%d (a multiple of %d), 16-B aligned maps", C, U3_CS);
  const size_t lds = (size_t)(sw_[0] * (n > 0) + sw_[1] * (n > 1) + sw_[2] * (n > 2)) * U3_CS * sizeof(float);
  CMX_REQUIRE(lds <= (size_t)U3_NI * 256 * 8 * sizeof(float), CMX_ERR_SHAPE,
              "bilinear_up3_add: source rows of %zu B exceed the %d staged items per thread", lds, U3_NI);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(up3_add_kernel<T>, dim3(B * H * (C / U3_CS)), dim3(256), lds, s, (const T*)src[0],
                       (const T*)src[1], (const T*)src[2], sh_[0], sw_[0], sh_[1], sw_[1], sh_[2], sw_[2], bias, (T*)out,
                       H, W, C, n);
  });
  return cmx_check_launch("bilinear_up3_add");
}

}  // extern "C"

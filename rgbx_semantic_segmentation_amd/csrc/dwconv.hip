// Depthwise 3x3 (pad 1, stride 1) convolution + bias + activation on token-major NHWC.
//
// Replaces  DWConv.forward + act  of Mix-FFN (dual_segformer.py:27-33, 67-71:
//   x.permute(0,2,1).reshape(B,C,H,W) -> Conv2d(C,C,3,1,1,groups=C) -> flatten/transpose -> GELU)
// and the DW3x3 + ReLU of ChannelEmbed (net_utils.py:315-318).  No NCHW round trip: the
// channel dim is contiguous.
//
// Images: NI = G*B images of H x W x C; image n belongs to group n / imgs_per_group (the
// RGB and X streams carry separate weights).  w: (G, C, 9) fp32, b: (G, C) fp32.
//
// Thread mapping (HBM/VALU-balanced stencil): a thread owns ONE quad of 4 channels (two
// packed fp32 pairs, so the taps and the GELU run as v_pk_fma_f32) and a strip of RX x RY
// output pixels.  It keeps a sliding window of 3 input rows (RX + 2 pixels each) in
// registers, so each input row is fetched once per strip ((RY+2)(RX+2) loads for RX*RY
// outputs), and its 36 weights + 4 biases stay in registers.  All loads are straight-line
// (out-of-image taps are predicated to zero, stores predicated), so a strip's loads can be
// in flight together.  Lanes of a wave are consecutive quads: every load / store is a
// coalesced 8-byte (bf16) / 16-byte (fp32) segment of a channel-contiguous NHWC row.
// The activation is a template argument: the GELU kernels carry no dead ReLU/sigmoid code.
// (That strip path now serves only channel counts that are not multiples of 32; see the
// LDS-tiled path below for every layer of B0 / B2.)
#include "cmx_common.h"

namespace {
constexpr int RXF = 4;           // output pixels per strip along x (forward / transposed pass)
constexpr int RXB = 2;           // ... in the dW-accumulating backward pass (register budget)
constexpr int RY = 8;            // output rows per strip
constexpr int DW_BWD_THREADS = 65536;   // target threads per group for the dW-accumulating pass

typedef cmx_f2 Px[2];            // 4 channels as two packed pairs

template <typename T>
__device__ __forceinline__ void ld4(const T* p, Px& v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = (cmx_f2){a.x, a.y};
    v[1] = (cmx_f2){a.z, a.w};
  } else {
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    v[0] = unpack2<T>(a.x);
    v[1] = unpack2<T>(a.y);
  }
}

template <typename T>
__device__ __forceinline__ void st4(T* p, const Px& v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
  } else {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2<T>(v[0].x, v[0].y), pack2<T>(v[1].x, v[1].y));
  }
}

// the pair as it is stored in T (16-bit types: round-to-nearest-even)
template <typename T>
__device__ __forceinline__ cmx_f2 stored(cmx_f2 v) {
  if constexpr (sizeof(T) == 4) {
    return v;
  } else {
    return unpack2<T>(pack2<T>(v.x, v.y));
  }
}

// the 4 channels' 9 taps are 36 contiguous floats (c0 % 4 == 0 -> 16-byte aligned);
// w2[pair][tap] = {w[2 pair][tap], w[2 pair + 1][tap]}
__device__ __forceinline__ void load_w36(const float* wg, cmx_f2 (&w2)[2][9]) {
  const float4* p = reinterpret_cast<const float4*>(wg);
  float w[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 a = p[i];
    w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    w2[0][k] = (cmx_f2){w[k], w[9 + k]};
    w2[1][k] = (cmx_f2){w[18 + k], w[27 + k]};
  }
}

__device__ __forceinline__ void load_bias(const float* b, Px& bias) {
  if (b) {
    const float4 bb = *reinterpret_cast<const float4*>(b);
    bias[0] = (cmx_f2){bb.x, bb.y};
    bias[1] = (cmx_f2){bb.z, bb.w};
  } else {
    bias[0] = bias[1] = pk_splat(0.f);
  }
}

// input row y, pixels x0-1 .. x0+R of one image (ib already offset to channel c0)
template <typename T, int R>
__device__ __forceinline__ void load_row(const T* ib, int y, int x0, int H, int W, int C, Px (&r)[R + 2]) {
  const bool yok = y >= 0 && y < H;
#pragma unroll
  for (int j = 0; j < R + 2; ++j) {
    const int x = x0 - 1 + j;
    if (yok && x >= 0 && x < W) {
      ld4<T>(ib + (y * W + x) * C, r[j]);
    } else {
      r[j][0] = pk_splat(0.f);
      r[j][1] = pk_splat(0.f);
    }
  }
}

struct Strip {
  int img, x0, y0;
};

template <int R>
__device__ __forceinline__ Strip strip_of(int s, int NXS, int NYS) {
  Strip st;
  st.x0 = (s % NXS) * R;
  const int r = s / NXS;
  st.y0 = (r % NYS) * RY;
  st.img = r / NYS;
  return st;
}

// forward (FLIP = false: cross-correlation + bias + act) or the transposed conv of the
// backward (FLIP = true: taps mirrored, no bias, ACT = 0).  One strip per thread.
template <typename T, bool FLIP, int ACT>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ out, int ipg, int H,
                                                     int W, int C, int NXS, int NYS) {
  const int CQ = C >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * NXS * NYS * ipg) return;
  const int g = blockIdx.y;
  const int c0 = (t % CQ) * 4;
  const Strip st = strip_of<RXF>(t / CQ, NXS, NYS);
  cmx_f2 wr[2][9];
  load_w36(w + ((long)g * C + c0) * 9, wr);
  Px bias;
  load_bias(b ? b + g * C + c0 : nullptr, bias);
  const long off = ((long)g * ipg + st.img) * H * W * C + c0;
  const T* ib = h + off;
  T* ob = out + off;
  Px rin[3][RXF + 2];
  load_row<T, RXF>(ib, st.y0 - 1, st.x0, H, W, C, rin[0]);
  load_row<T, RXF>(ib, st.y0, st.x0, H, W, C, rin[1]);
#pragma unroll
  for (int rr = 0; rr < RY; ++rr) {
    const int y = st.y0 + rr;
    load_row<T, RXF>(ib, y + 1, st.x0, H, W, C, rin[(rr + 2) % 3]);
#pragma unroll
    for (int xi = 0; xi < RXF; ++xi) {
      Px acc = {bias[0], bias[1]};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int tap = FLIP ? 8 - (i * 3 + j) : i * 3 + j;
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[u] = pk_fma(wr[u][tap], rin[(rr + i) % 3][xi + j][u], acc[u]);
        }
      acc[0] = act2_fwd<ACT>(acc[0]);
      acc[1] = act2_fwd<ACT>(acc[1]);
      if (y < H && st.x0 + xi < W) st4<T>(ob + (y * W + st.x0 + xi) * C, acc);
    }
  }
}

// dz = da * act'(z) with z recomputed from h; per-thread partial dW (9 taps) / db of the
// thread's quad over its strips go to ws[(g, slot)][c][10] (reduced afterwards over the P
// slots).  Thread (q, slot) processes strips slot, slot + P, ...
template <typename T, int ACT>
__global__ __launch_bounds__(256) void dw_bwd_dz_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        T* __restrict__ dz, float* __restrict__ ws, int ipg, int H,
                                                        int W, int C, int NXS, int NYS, int P) {
  const int CQ = C >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CQ * P) return;
  const int g = blockIdx.y;
  const int q = t % CQ, slot = t / CQ;
  const int c0 = q * 4;
  cmx_f2 wr[2][9], aw[2][9];
  Px bias, ab;
  load_w36(w + ((long)g * C + c0) * 9, wr);
  load_bias(b ? b + g * C + c0 : nullptr, bias);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    ab[u] = pk_splat(0.f);
#pragma unroll
    for (int k = 0; k < 9; ++k) aw[u][k] = pk_splat(0.f);
  }
  const int nstrips = NXS * NYS * ipg;
  for (int s = slot; s < nstrips; s += P) {
    const Strip st = strip_of<RXB>(s, NXS, NYS);
    const long off = ((long)g * ipg + st.img) * H * W * C + c0;
    const T* ib = h + off;
    const T* dab = da + off;
    T* dzb = dz + off;
    Px rin[3][RXB + 2];
    load_row<T, RXB>(ib, st.y0 - 1, st.x0, H, W, C, rin[0]);
    load_row<T, RXB>(ib, st.y0, st.x0, H, W, C, rin[1]);
#pragma unroll
    for (int rr = 0; rr < RY; ++rr) {
      const int y = st.y0 + rr;
      load_row<T, RXB>(ib, y + 1, st.x0, H, W, C, rin[(rr + 2) % 3]);
#pragma unroll
      for (int xi = 0; xi < RXB; ++xi) {
        const bool in = y < H && st.x0 + xi < W;
        Px d = {pk_splat(0.f), pk_splat(0.f)};
        if (in) {
          Px z = {bias[0], bias[1]};
#pragma unroll
          for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int u = 0; u < 2; ++u) z[u] = pk_fma(wr[u][k], rin[(rr + k / 3) % 3][xi + k % 3][u], z[u]);
          const int pofs = (y * W + st.x0 + xi) * C;
          ld4<T>(dab + pofs, d);
#pragma unroll
          for (int u = 0; u < 2; ++u) d[u] = d[u] * act2_grad<ACT>(z[u]);
          st4<T>(dzb + pofs, d);
          // accumulate with the value as stored so dW matches the dz used for dh
#pragma unroll
          for (int u = 0; u < 2; ++u) d[u] = stored<T>(d[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ab[u] += d[u];
#pragma unroll
          for (int k = 0; k < 9; ++k) aw[u][k] = pk_fma(d[u], rin[(rr + k / 3) % 3][xi + k % 3][u], aw[u][k]);
        }
      }
    }
  }
  float* o = ws + ((long)g * P + slot) * C * 10 + (long)c0 * 10;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      o[(2 * u) * 10 + k] = aw[u][k].x;
      o[(2 * u + 1) * 10 + k] = aw[u][k].y;
    }
    o[(2 * u) * 10 + 9] = ab[u].x;
    o[(2 * u + 1) * 10 + 9] = ab[u].y;
  }
}

// tmp (G, C, 10) -> dw (G, C, 9), db (G, C)
__global__ void dw_scatter_kernel(const float* __restrict__ tmp, float* __restrict__ dw, float* __restrict__ db, int G,
                                  int C, int accumulate) {
  const long total = (long)G * C * 10;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)total; i += gridDim.x * blockDim.x) {
    const int k = i % 10;
    const int gc = i / 10;
    const float s = tmp[i];
    float* o = k < 9 ? &dw[gc * 9 + k] : (db ? &db[gc] : nullptr);
    if (o) *o = accumulate ? *o + s : s;
  }
}

// ============================================================================ LDS-tiled path
// Block = one tile of TY x TX output pixels x CB channels (CB = 32 or 64) of one image.
// Input tiles (with halo) are staged in LDS by fully coalesced 16-B-per-lane loads (8
// consecutive lanes = one pixel's CB channels); each thread then owns ONE group of 8
// channels -- its 72 taps and 8 biases stay in registers -- and walks tile pixels, reading
// the 3x3 neighbourhood from LDS (lanes on consecutive pixels: conflict-free).
//
// The backward is one kernel: dz = da * act'(z) is recomputed (z from the h tile) on the
// tile plus a 1-pixel halo into LDS, then dh = conv^T(dz) and the dW / db partial sums of
// the inner pixels come from that LDS image.  dz never goes to HBM (the old path wrote it,
// read it back for dh, and re-read h for dW).  Per-block dW / db partials are summed across
// the threads of a channel group by a butterfly reduce-scatter (80 -> 5 values per lane)
// and written to a (group, tile) slab that reduce_partials folds.
constexpr int TY2 = 8, TX2 = 16;                 // inner tile
constexpr int EY = TY2 + 2, EX = TX2 + 2;         // + 1-pixel halo
constexpr int HY = TY2 + 4, HX = TX2 + 4;         // + 2-pixel halo (backward h tile)
// saved-act backward tile: 16 x 16 (halo 1.27x instead of 1.41x; measured stage 1 70.6 -> 52.3 us,
// while the forward is faster at 8 x 16: 34.2 vs 37.0 us, scripts/bench_dw.py)
constexpr int TYB = 16, TXB = 16, EYB = TYB + 2, EXB = TXB + 2;

template <typename T> struct V8;                  // 8 channels as stored
template <> struct V8<bf16> { uint4 a; };
template <> struct V8<f16> { uint4 a; };
template <> struct V8<float> { float4 a, b; };

template <typename T>
__device__ __forceinline__ V8<T> v8_load(const T* p) {
  V8<T> v;
  if constexpr (sizeof(T) == 2) v.a = *reinterpret_cast<const uint4*>(p);
  else { v.a = reinterpret_cast<const float4*>(p)[0]; v.b = reinterpret_cast<const float4*>(p)[1]; }
  return v;
}
template <typename T>
__device__ __forceinline__ void v8_store(T* p, const V8<T>& v) {
  if constexpr (sizeof(T) == 2) *reinterpret_cast<uint4*>(p) = v.a;
  else { reinterpret_cast<float4*>(p)[0] = v.a; reinterpret_cast<float4*>(p)[1] = v.b; }
}
template <typename T>
__device__ __forceinline__ V8<T> v8_zero() {
  V8<T> v;
  if constexpr (sizeof(T) == 2) v.a = make_uint4(0, 0, 0, 0);
  else { v.a = make_float4(0.f, 0.f, 0.f, 0.f); v.b = v.a; }
  return v;
}
// unpack to 4 packed pairs
template <typename T>
__device__ __forceinline__ void v8_unpack(const V8<T>& v, cmx_f2 (&o)[4]) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t w[4] = {v.a.x, v.a.y, v.a.z, v.a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = unpack2<T>(w[i]);
  } else {
    o[0] = (cmx_f2){v.a.x, v.a.y}; o[1] = (cmx_f2){v.a.z, v.a.w};
    o[2] = (cmx_f2){v.b.x, v.b.y}; o[3] = (cmx_f2){v.b.z, v.b.w};
  }
}
template <typename T>
__device__ __forceinline__ V8<T> v8_pack(const cmx_f2 (&o)[4]) {
  V8<T> v;
  if constexpr (sizeof(T) == 2) {
    v.a = make_uint4(pack2<T>(o[0].x, o[0].y), pack2<T>(o[1].x, o[1].y), pack2<T>(o[2].x, o[2].y),
                     pack2<T>(o[3].x, o[3].y));
  } else {
    v.a = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
    v.b = make_float4(o[2].x, o[2].y, o[3].x, o[3].y);
  }
  return v;
}

// 8 channels' 9 taps (72 contiguous floats) as pairs: w2[pair][tap] = {w[2p][tap], w[2p+1][tap]}
__device__ __forceinline__ void load_w72(const float* wg, cmx_f2 (&w2)[4][9]) {
  cmx_f2 (&a)[2][9] = *reinterpret_cast<cmx_f2 (*)[2][9]>(&w2[0]);
  cmx_f2 (&b)[2][9] = *reinterpret_cast<cmx_f2 (*)[2][9]>(&w2[2]);
  load_w36(wg, a);
  load_w36(wg + 36, b);
}

struct Tile2 {
  int g, img, ty0, tx0, cb0, sp;
};
template <int TY_ = TY2, int TX_ = TX2>
__device__ __forceinline__ Tile2 tile2_of(int CB, int ipg, int tiles_x, int tiles_y, int ncb) {
  Tile2 t;
  int b = blockIdx.x;
  const int cb = b % ncb; b /= ncb;
  t.sp = b;                                        // spatial tile index within the group
  const int tx = b % tiles_x; b /= tiles_x;
  const int ty = b % tiles_y; b /= tiles_y;
  t.img = b;
  t.g = blockIdx.y;
  t.ty0 = ty * TY_; t.tx0 = tx * TX_; t.cb0 = cb * CB;
  return t;
}

// stage a (RY x RX)-pixel region with origin (y0, x0) of image `base` (channels cb0..cb0+CB)
// into img[cg][px][8]; zeros outside the image
// Two phases, unrolled: every global load of the thread is issued before the first LDS store,
// so the region costs one memory latency instead of one per 256-item round (the stores would
// otherwise order each round's load after the previous round's LDS write).
template <typename T, int CB, int RY_, int RX_>
__device__ __forceinline__ void stage_region(const T* __restrict__ base, T* img, int y0, int x0, int H, int W, int C) {
  constexpr int NCG = CB / 8, NPX = RY_ * RX_;
  constexpr int ITER = (NCG * NPX + 255) / 256;
  V8<T> v[ITER];
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int it = threadIdx.x + k * 256;
    const int cg = it % NCG, px = it / NCG;
    const int y = y0 + px / RX_, x = x0 + px % RX_;
    v[k] = v8_zero<T>();
    if (it < NCG * NPX && y >= 0 && y < H && x >= 0 && x < W) v[k] = v8_load<T>(base + ((long)y * W + x) * C + cg * 8);
  }
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int it = threadIdx.x + k * 256;
    if (it < NCG * NPX) v8_store<T>(img + ((it % NCG) * NPX + it / NCG) * 8, v[k]);
  }
}

// Channel-fast thread mapping (forward and saved-act backward): thread t owns the 4 channels
// cq = t % (CB / 4) of pixels p = t / (CB / 4), + 256 / (CB / 4), ... of the tile.  LDS images are
// pixel-major [px][CB] (a straight copy of the NHWC rows), so the 16 (CB = 64) lanes of one
// pixel read 128 contiguous bytes (conflict-free) and every global store is a coalesced
// 128-B (bf16, CB = 64) row segment -- not one 8-B / 16-B piece per lane at a C-element stride.
template <typename T> struct V4;                  // 4 channels as stored
template <> struct V4<bf16> { uint2 a; };
template <> struct V4<f16> { uint2 a; };
template <> struct V4<float> { float4 a; };
template <typename T>
__device__ __forceinline__ V4<T> v4_load(const T* p) {
  V4<T> v;
  if constexpr (sizeof(T) == 2) v.a = *reinterpret_cast<const uint2*>(p);
  else v.a = *reinterpret_cast<const float4*>(p);
  return v;
}
template <typename T>
__device__ __forceinline__ void v4_unpack(const V4<T>& v, cmx_f2 (&o)[2]) {
  if constexpr (sizeof(T) == 2) {
    o[0] = unpack2<T>(v.a.x);
    o[1] = unpack2<T>(v.a.y);
  } else {
    o[0] = (cmx_f2){v.a.x, v.a.y}; o[1] = (cmx_f2){v.a.z, v.a.w};
  }
}
template <typename T>
__device__ __forceinline__ void v4_store(T* p, const cmx_f2 (&o)[2]) {
  if constexpr (sizeof(T) == 2) *reinterpret_cast<uint2*>(p) = make_uint2(pack2<T>(o[0].x, o[0].y), pack2<T>(o[1].x, o[1].y));
  else *reinterpret_cast<float4*>(p) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
}
// stage a (RY x RX)-pixel region into a pixel-major image img[px][CB]; zeros outside the image
template <typename T, int CB, int RY_, int RX_>
__device__ __forceinline__ void stage_region_pm(const T* __restrict__ base, T* img, int y0, int x0, int H, int W, int C) {
  constexpr int NCG = CB / 8, NPX = RY_ * RX_;
  constexpr int ITER = (NCG * NPX + 255) / 256;
  V8<T> v[ITER];
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int it = threadIdx.x + k * 256;
    const int cg = it % NCG, px = it / NCG;
    const int y = y0 + px / RX_, x = x0 + px % RX_;
    v[k] = v8_zero<T>();
    if (it < NCG * NPX && y >= 0 && y < H && x >= 0 && x < W) v[k] = v8_load<T>(base + ((long)y * W + x) * C + cg * 8);
  }
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int it = threadIdx.x + k * 256;
    if (it < NCG * NPX) v8_store<T>(img + it * 8, v[k]);
  }
}

template <typename T, int CB, int ACT, bool FLIP>
__global__ __launch_bounds__(256) void dw2_fwd_kernel(const T* __restrict__ h, const float* __restrict__ w,
                                                      const float* __restrict__ b, T* __restrict__ out, int ipg, int H,
                                                      int W, int C, int tiles_x, int tiles_y, int ncb,
                                                      T* __restrict__ gprime) {
  constexpr int NCQ = CB / 4, PPI = 256 / NCQ;     // channel quads; pixels per block-wide step
  __shared__ __attribute__((aligned(16))) T hs[EY * EX * CB];
  const Tile2 t = tile2_of(CB, ipg, tiles_x, tiles_y, ncb);
  const long ibase = ((long)t.g * ipg + t.img) * H * W * C + t.cb0;
  stage_region_pm<T, CB, EY, EX>(h + ibase, hs, t.ty0 - 1, t.tx0 - 1, H, W, C);
  const int cq = threadIdx.x % NCQ, pl = threadIdx.x / NCQ;
  const int c0 = t.cb0 + cq * 4;
  __syncthreads();
  cmx_f2 wr[2][9], bias[2];
  load_w36(w + ((long)t.g * C + c0) * 9, wr);
  if (b) {
    const float4 b0 = *reinterpret_cast<const float4*>(b + (long)t.g * C + c0);
    bias[0] = (cmx_f2){b0.x, b0.y}; bias[1] = (cmx_f2){b0.z, b0.w};
  } else {
    bias[0] = bias[1] = pk_splat(0.f);
  }
  const T* hc = hs + cq * 4;
  for (int it = pl; it < TY2 * TX2; it += PPI) {
    const int r = it / TX2, c = it % TX2;
    const int y = t.ty0 + r, x = t.tx0 + c;
    if (y >= H || x >= W) continue;
    cmx_f2 acc[2] = {bias[0], bias[1]};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        cmx_f2 v[2];
        v4_unpack<T>(v4_load<T>(hc + ((r + i) * EX + c + j) * CB), v);
        const int tap = FLIP ? 8 - (i * 3 + j) : i * 3 + j;
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u] = pk_fma(wr[u][tap], v[u], acc[u]);
      }
    const long o = ibase + ((long)y * W + x) * C + cq * 4;
    if (gprime) {              // act'(z), saved so the backward needs no conv recompute
      cmx_f2 gd[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) gd[u] = act2_grad<ACT>(acc[u]);
      v4_store<T>(gprime + o, gd);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = act2_fwd<ACT>(acc[u]);
    v4_store<T>(out + o, acc);
  }
}

// butterfly reduce-scatter of N values over the lanes (xor offsets o): lanes with bit o set
// keep the upper half
template <int N>
__device__ __forceinline__ void rs_step(const float (&v)[N], float (&o)[N / 2], int off, bool up) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const float send = up ? v[k] : v[k + N / 2];
    const float keep = up ? v[k + N / 2] : v[k];
    o[k] = keep + xor_lane(send, off);
  }
}

// Backward from a saved act'(z) (cmx_dwconv3x3_fwd_save).  Staging: da and act'(z) of the tile
// + 1-pixel halo are loaded together (16-B loads, all issued before the first LDS store) and
// multiplied in registers, so ONE LDS image holds dz = da * act'(z) (zero outside the image);
// h is staged for the inner tile only.  Then ONE pass over the inner pixels reads each
// pixel's 3 x 3 dz neighbourhood once and uses it twice:
//   dh[y][x]  = sum_ij w[i][j] dz[y-i+1][x-j+1]     (transposed conv)
//   dW[i][j] += h[y][x] dz[y-i+1][x-j+1]            (each in-image h pixel owned by one tile)
// and db += dz[y][x] (the centre tap).  Channel-fast mapping (see dw2_fwd_kernel): 4 channels
// per thread, pixel-major LDS images, coalesced dh rows.  The 40 dW / db partials of a thread
// are reduce-scattered over the lanes of its quad inside the wave, then summed over the 4
// waves through LDS (reusing the dz image) into the block's (group, tile) slab.
template <typename T, int CB>
__device__ __forceinline__ void stage_dz(const T* __restrict__ da, const T* __restrict__ gp, T* dzs, int ty0, int tx0,
                                         int H, int W, int C) {
  constexpr int NCG = CB / 8, NE = EYB * EXB;
  constexpr int ITE = (NCG * NE + 255) / 256;
  V8<T> a[ITE], g[ITE];
#pragma unroll
  for (int k = 0; k < ITE; ++k) {
    const int it = threadIdx.x + k * 256;
    const int cg = it % NCG, px = it / NCG;
    const int y = ty0 - 1 + px / EXB, x = tx0 - 1 + px % EXB;
    a[k] = v8_zero<T>();
    g[k] = v8_zero<T>();
    if (it < NCG * NE && y >= 0 && y < H && x >= 0 && x < W) {
      const long o = ((long)y * W + x) * C + cg * 8;
      a[k] = v8_load<T>(da + o);
      g[k] = v8_load<T>(gp + o);
    }
  }
#pragma unroll
  for (int k = 0; k < ITE; ++k) {
    const int it = threadIdx.x + k * 256;
    if (it < NCG * NE) {
      cmx_f2 d[4], gd[4];
      v8_unpack<T>(a[k], d);
      v8_unpack<T>(g[k], gd);
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = d[u] * gd[u];
      v8_store<T>(dzs + it * 8, v8_pack<T>(d));
    }
  }
}

template <typename T, int CB>
__global__ __launch_bounds__(256, 3) void dw2_bwdg_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                       const T* __restrict__ gprime, const float* __restrict__ w,
                                                       T* __restrict__ dh, float* __restrict__ part, int ipg, int H,
                                                       int W, int C, int tiles_x, int tiles_y, int ncb, int nsp) {
  constexpr int NCQ = CB / 4, PPI = 256 / NCQ;
  constexpr int NE = EYB * EXB, NIN = TYB * TXB;
  constexpr int LPQ = 64 / NCQ;                     // lanes of one quad in a wave (4 or 8)
  constexpr int NV = LPQ == 4 ? 10 : 5;             // partials per lane after the in-wave reduce-scatter
  // only the dz image lives in LDS (41 KB at CB = 64: three blocks per CU); each thread's h
  // pixels (4 channels, 16 lanes of a pixel = one 128-B row segment) go straight to registers
  constexpr int NIT = NIN / PPI;
  __shared__ __attribute__((aligned(16))) T dzs[NE * CB];
  static_assert(sizeof(dzs) >= 4 * 64 * NV * sizeof(float), "cross-wave reduce buffer");
  static_assert(NIN % PPI == 0, "pixel rounds");
  const Tile2 t = tile2_of<TYB, TXB>(CB, ipg, tiles_x, tiles_y, ncb);
  const long ibase = ((long)t.g * ipg + t.img) * H * W * C + t.cb0;
  stage_dz<T, CB>(da + ibase, gprime + ibase, dzs, t.ty0, t.tx0, H, W, C);
  const int cq = threadIdx.x % NCQ, pl = threadIdx.x / NCQ;
  const int c0 = t.cb0 + cq * 4;
  V4<T> hreg[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int it = pl + k * PPI;
    const int y = t.ty0 + it / TXB, x = t.tx0 + it % TXB;
    hreg[k].a = {};
    if (y < H && x < W) hreg[k] = v4_load<T>(h + ibase + ((long)y * W + x) * C + cq * 4);
  }
  __syncthreads();
  cmx_f2 wr[2][9];
  load_w36(w + ((long)t.g * C + c0) * 9, wr);
  const T* dzc = dzs + cq * 4;
  cmx_f2 acc[2][10];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[u][k] = pk_splat(0.f);
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int it = pl + k * PPI;
    const int r = it / TXB, c = it % TXB;
    const int y = t.ty0 + r, x = t.tx0 + c;
    if (y >= H || x >= W) continue;
    cmx_f2 hv[2];
    v4_unpack<T>(hreg[k], hv);
    cmx_f2 g[2] = {pk_splat(0.f), pk_splat(0.f)};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        cmx_f2 dv[2];
        v4_unpack<T>(v4_load<T>(dzc + ((r + 2 - i) * EXB + c + 2 - j) * CB), dv);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          g[u] = pk_fma(wr[u][i * 3 + j], dv[u], g[u]);
          acc[u][i * 3 + j] = pk_fma(hv[u], dv[u], acc[u][i * 3 + j]);
        }
        if (i == 1 && j == 1) {
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[u][9] += dv[u];
        }
      }
    if (dh) v4_store<T>(dh + ibase + ((long)y * W + x) * C + cq * 4, g);
  }
  // in-wave reduce-scatter over the LPQ lanes of the quad (xor NCQ, 2 NCQ, ...): 40 -> NV
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float flat[40], r20[20], r10[10];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      flat[(2 * u) * 10 + k] = acc[u][k].x;
      flat[(2 * u + 1) * 10 + k] = acc[u][k].y;
    }
  int seg = 0;
  rs_step<40>(flat, r20, NCQ, (lane & NCQ) != 0); seg = seg * 2 + ((lane & NCQ) != 0);
  rs_step<20>(r20, r10, 2 * NCQ, (lane & (2 * NCQ)) != 0); seg = seg * 2 + ((lane & (2 * NCQ)) != 0);
  float rv[NV];
  if constexpr (NV == 5) {
    rs_step<10>(r10, rv, 4 * NCQ, (lane & (4 * NCQ)) != 0); seg = seg * 2 + ((lane & (4 * NCQ)) != 0);
  } else {
#pragma unroll
    for (int k = 0; k < 10; ++k) rv[k] = r10[k];
  }
  // lane holds values [seg * NV, seg * NV + NV) of its quad's 40 (4 channels x 10)
  __syncthreads();                                  // every wave is done reading dzs
  float* red = reinterpret_cast<float*>(dzs);
#pragma unroll
  for (int k = 0; k < NV; ++k) red[(wv * 64 + lane) * NV + k] = rv[k];
  __syncthreads();
  float* o = part + ((long)t.g * nsp + t.sp) * C * 10 + (long)t.cb0 * 10;
  for (int e = threadIdx.x; e < 64 * NV; e += 256) {
    const float v = red[e] + red[64 * NV + e] + red[128 * NV + e] + red[192 * NV + e];
    const int l = e / NV, k = e % NV;
    const int q = l % NCQ, sg = (l / NCQ);          // lane l's quad and its segment bits (xor order)
    // seg was accumulated high bit first from (lane & NCQ), (lane & 2NCQ)[, (lane & 4NCQ)]
    int sgi = 0;
#pragma unroll
    for (int bit = 0; bit < (NV == 5 ? 3 : 2); ++bit) sgi = sgi * 2 + ((sg >> bit) & 1);
    o[q * 40 + sgi * NV + k] = v;
  }
}


template <typename T, int CB, int ACT>
__global__ __launch_bounds__(256, 2) void dw2_bwd_kernel(const T* __restrict__ da, const T* __restrict__ h,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      T* __restrict__ dh, float* __restrict__ part, int ipg, int H,
                                                      int W, int C, int tiles_x, int tiles_y, int ncb, int nsp) {
  constexpr int NCG = CB / 8, TPC = 256 / NCG;
  __shared__ __attribute__((aligned(16))) T hs[NCG * HY * HX * 8];
  __shared__ __attribute__((aligned(16))) T das[NCG * EY * EX * 8];
  __shared__ __attribute__((aligned(16))) T dzs[NCG * EY * EX * 8];
  const Tile2 t = tile2_of(CB, ipg, tiles_x, tiles_y, ncb);
  const long ibase = ((long)t.g * ipg + t.img) * H * W * C + t.cb0;
  stage_region<T, CB, HY, HX>(h + ibase, hs, t.ty0 - 2, t.tx0 - 2, H, W, C);
  stage_region<T, CB, EY, EX>(da + ibase, das, t.ty0 - 1, t.tx0 - 1, H, W, C);
  const int cg = threadIdx.x / TPC, pl = threadIdx.x % TPC;
  const int c0 = t.cb0 + cg * 8;
  cmx_f2 wr[4][9], bias[4];
  load_w72(w + ((long)t.g * C + c0) * 9, wr);
  if (b) {
    const float4 b0 = *reinterpret_cast<const float4*>(b + (long)t.g * C + c0);
    const float4 b1 = *reinterpret_cast<const float4*>(b + (long)t.g * C + c0 + 4);
    bias[0] = (cmx_f2){b0.x, b0.y}; bias[1] = (cmx_f2){b0.z, b0.w};
    bias[2] = (cmx_f2){b1.x, b1.y}; bias[3] = (cmx_f2){b1.z, b1.w};
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) bias[u] = pk_splat(0.f);
  }
  __syncthreads();
  const T* hc = hs + cg * HY * HX * 8;
  const T* dac = das + cg * EY * EX * 8;
  T* dzc = dzs + cg * EY * EX * 8;
  // dz on the tile + 1-pixel halo (zero outside the image: no such output pixel)
  for (int it = pl; it < EY * EX; it += TPC) {
    const int r = it / EX, c = it % EX;
    const int y = t.ty0 - 1 + r, x = t.tx0 - 1 + c;
    V8<T> dzv = v8_zero<T>();
    if (y >= 0 && y < H && x >= 0 && x < W) {
      cmx_f2 z[4] = {bias[0], bias[1], bias[2], bias[3]};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          cmx_f2 v[4];
          v8_unpack<T>(v8_load<T>(hc + ((r + i) * HX + c + j) * 8), v);
#pragma unroll
          for (int u = 0; u < 4; ++u) z[u] = pk_fma(wr[u][i * 3 + j], v[u], z[u]);
        }
      cmx_f2 d[4];
      v8_unpack<T>(v8_load<T>(dac + it * 8), d);
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = d[u] * act2_grad<ACT>(z[u]);
      dzv = v8_pack<T>(d);
    }
    v8_store<T>(dzc + it * 8, dzv);
  }
  __syncthreads();
  // dh = conv^T(dz) on the inner tile (needs the taps; they die after this loop)
  if (dh) {
    for (int it = pl; it < TY2 * TX2; it += TPC) {
      const int r = it / TX2, c = it % TX2;
      const int y = t.ty0 + r, x = t.tx0 + c;
      if (y >= H || x >= W) continue;
      cmx_f2 g[4] = {pk_splat(0.f), pk_splat(0.f), pk_splat(0.f), pk_splat(0.f)};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          cmx_f2 dv[4];           // dh[y][x] += w[i][j] dz[y-i+1][x-j+1]
          v8_unpack<T>(v8_load<T>(dzc + ((r + 2 - i) * EX + c + 2 - j) * 8), dv);
#pragma unroll
          for (int u = 0; u < 4; ++u) g[u] = pk_fma(wr[u][i * 3 + j], dv[u], g[u]);
        }
      v8_store<T>(dh + ibase + ((long)y * W + x) * C + cg * 8, v8_pack<T>(g));
    }
  }
  // dW[i][j] += dz[y][x] h[y+i-1][x+j-1], db += dz over the inner tile
  cmx_f2 acc[4][10];                                // [channel pair][9 taps + bias]
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[u][k] = pk_splat(0.f);
  for (int it = pl; it < TY2 * TX2; it += TPC) {
    const int r = it / TX2, c = it % TX2;
    if (t.ty0 + r >= H || t.tx0 + c >= W) continue;
    cmx_f2 dz0[4];
    v8_unpack<T>(v8_load<T>(dzc + ((r + 1) * EX + c + 1) * 8), dz0);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        cmx_f2 hv[4];
        v8_unpack<T>(v8_load<T>(hc + ((r + 1 + i) * HX + c + 1 + j) * 8), hv);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u][i * 3 + j] = pk_fma(dz0[u], hv[u], acc[u][i * 3 + j]);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u][9] += dz0[u];
  }
  // reduce the 80 partials over the TPC lanes of this channel group (TPC = 32 or 64)
  const int lane = threadIdx.x & 63;
  float flat[80], r40[40], r20[20], r10[10], r5[5];   // flat[ch * 10 + k]
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      flat[(2 * u) * 10 + k] = acc[u][k].x;
      flat[(2 * u + 1) * 10 + k] = acc[u][k].y;
    }
  int seg = 0, s_off = TPC >> 1;
  rs_step<80>(flat, r40, s_off, (lane & s_off) != 0); seg = seg * 2 + ((lane & s_off) != 0); s_off >>= 1;
  rs_step<40>(r40, r20, s_off, (lane & s_off) != 0); seg = seg * 2 + ((lane & s_off) != 0); s_off >>= 1;
  rs_step<20>(r20, r10, s_off, (lane & s_off) != 0); seg = seg * 2 + ((lane & s_off) != 0); s_off >>= 1;
  rs_step<10>(r10, r5, s_off, (lane & s_off) != 0); seg = seg * 2 + ((lane & s_off) != 0); s_off >>= 1;
  for (; s_off > 0; s_off >>= 1) {
#pragma unroll
    for (int k = 0; k < 5; ++k) r5[k] += xor_lane(r5[k], s_off);
  }
  if ((lane & (TPC / 16 - 1)) == 0) {              // one lane per 5-value segment
    float* o = part + ((long)t.g * nsp + t.sp) * C * 10 + (long)c0 * 10 + seg * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = r5[k];
  }
}

int bwd_slots(int CQ, int nstrips) {
  int pmax = DW_BWD_THREADS / CQ;
  if (pmax < 1) pmax = 1;
  if (pmax >= nstrips) return nstrips;
  const int per = (nstrips + pmax - 1) / pmax;    // strips per thread, balanced
  return (nstrips + per - 1) / per;
}
}  // namespace

// LDS-tiled path when the channel count splits into 32-channel blocks (every B0/B2 layer)
// (fp32 parity mode: 32-channel blocks, so the backward's three tiles fit twice per CU)
static int tile_cb(int C, int dtype) { return (C % 64 == 0 && (dtype == 1 || dtype == 2)) ? 64 : C % 32 == 0 ? 32 : 0; }

extern "C" {

int cmx_dwconv3x3_fwd(const void* h, const float* w, const float* b, void* out, int NI, int imgs_per_group, int H,
                      int W, int C, int act, int dtype, hipStream_t s) {
  return cmx_dwconv3x3_fwd_save(h, w, b, out, nullptr, NI, imgs_per_group, H, W, C, act, dtype, s);
}

int cmx_dwconv3x3_fwd_save(const void* h, const float* w, const float* b, void* out, void* gprime, int NI,
                           int imgs_per_group, int H, int W, int C, int act, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_fwd: C=%d", C);
  CMX_REQUIRE(!gprime || tile_cb(C, dtype), CMX_ERR_SHAPE, "dwconv_fwd_save: C=%d has no LDS-tiled path", C);
  CMX_REQUIRE((long)NI * H * W * C < (1L << 31), CMX_ERR_SHAPE, "dwconv_fwd: tensor too large for 32-bit indexing");
  const int G = NI / imgs_per_group;
  const int CB = tile_cb(C, dtype);
  if (CB) {
    const int tx = cdiv(W, TX2), ty = cdiv(H, TY2), ncb = C / CB;
    const dim3 grid((unsigned)imgs_per_group * ty * tx * ncb, G);
    CMX_DISPATCH(dtype, T, {
      CMX_ACT_DISPATCH(act, A, {
        if (CB == 32) {
          hipLaunchKernelGGL((dw2_fwd_kernel<T, 32, A, false>), grid, dim3(256), 0, s, (const T*)h, w, b, (T*)out,
                             imgs_per_group, H, W, C, tx, ty, ncb, (T*)gprime);
        } else if constexpr (sizeof(T) == 2) {
          hipLaunchKernelGGL((dw2_fwd_kernel<T, 64, A, false>), grid, dim3(256), 0, s, (const T*)h, w, b, (T*)out,
                             imgs_per_group, H, W, C, tx, ty, ncb, (T*)gprime);
        }
      });
    });
    return cmx_check_launch("dwconv_fwd");
  }
  const int NXS = cdiv(W, RXF), NYS = cdiv(H, RY);
  const long threads = (long)(C / 4) * NXS * NYS * imgs_per_group;
  CMX_DISPATCH(dtype, T, {
    CMX_ACT_DISPATCH(act, A, {
      hipLaunchKernelGGL((dw_fwd_kernel<T, false, A>), dim3(cdiv(threads, 256), G), dim3(256), 0, s, (const T*)h, w,
                         b, (T*)out, imgs_per_group, H, W, C, NXS, NYS);
    });
  });
  return cmx_check_launch("dwconv_fwd");
}

int cmx_dwconv3x3_bwd_saved(const void* da, const void* h, const void* gprime, const float* w, void* dh, float* dw,
                            float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int accumulate,
                            int dtype, hipStream_t s) {
  const int CB = tile_cb(C, dtype);
  CMX_REQUIRE(CB && NI % imgs_per_group == 0 && gprime, CMX_ERR_SHAPE, "dwconv_bwd_saved: C=%d", C);
  CMX_REQUIRE((long)NI * H * W * C < (1L << 31), CMX_ERR_SHAPE, "dwconv_bwd_saved: tensor too large");
  const int G = NI / imgs_per_group;
  const int tx = cdiv(W, TXB), ty = cdiv(H, TYB), ncb = C / CB;
  const int P = imgs_per_group * ty * tx;
  const dim3 grid((unsigned)P * ncb, G);
  CMX_DISPATCH(dtype, T, {
    if (CB == 32) {
      hipLaunchKernelGGL((dw2_bwdg_kernel<T, 32>), grid, dim3(256), 0, s, (const T*)da, (const T*)h,
                         (const T*)gprime, w, (T*)dh, workspace, imgs_per_group, H, W, C, tx, ty, ncb, P);
    } else if constexpr (sizeof(T) == 2) {
      hipLaunchKernelGGL((dw2_bwdg_kernel<T, 64>), grid, dim3(256), 0, s, (const T*)da, (const T*)h,
                         (const T*)gprime, w, (T*)dh, workspace, imgs_per_group, H, W, C, tx, ty, ncb, P);
    }
  });
  if (!dw && !db) return cmx_check_launch("dwconv_bwd_saved");
  float* tmp = workspace + (size_t)G * P * C * 10;
  int st = cmx_reduce_partials(workspace, tmp, G, P, C * 10, 0, 1.f, s);
  if (st) return st;
  const long tot = (long)G * C * 10;
  hipLaunchKernelGGL(dw_scatter_kernel, dim3(cdiv(tot, 256) < 4096 ? cdiv(tot, 256) : 4096), dim3(256), 0, s, tmp, dw,
                     db, G, C, accumulate);
  return cmx_check_launch("dwconv_bwd_saved");
}

// partial-slab count (tiles per group) of cmx_dwconv3x3_bwd_saved: its dW / db partials occupy
// the first G * P * C * 10 floats of the (larger) cmx_dwconv3x3_bwd_workspace
int cmx_dwconv3x3_bwd_saved_tiles(int imgs_per_group, int H, int W) {
  return imgs_per_group * cdiv(H, TYB) * cdiv(W, TXB);
}

size_t cmx_dwconv3x3_bwd_workspace(int NI, int imgs_per_group, int H, int W, int C) {
  const int G = NI / imgs_per_group;
  // one workspace serves both LDS-tiled backwards: the recompute path's TY2 x TX2 tiles and
  // the saved-act path's TYB x TXB tiles (cmx_dwconv3x3_bwd_saved_tiles); partial slabs are
  // sized for whichever has more tiles, and the reduce's tmp sits after them
  int P;
  if (tile_cb(C, 0)) {
    const int p8 = imgs_per_group * cdiv(H, TY2) * cdiv(W, TX2);
    const int p16 = cmx_dwconv3x3_bwd_saved_tiles(imgs_per_group, H, W);
    P = p8 > p16 ? p8 : p16;
  } else {
    P = bwd_slots(C / 4, cdiv(W, RXB) * cdiv(H, RY) * imgs_per_group);
  }
  return ((size_t)G * P * C * 10 + (size_t)G * C * 10) * sizeof(float);
}

// da: upstream grad of the activation output; dh = conv^T(dz) (may be NULL) with
// dz = da * act'(z); dw (G,C,9), db (G,C) fp32 (db may be NULL).  dz (sized like h, dtype)
// receives dz on the strip path only; the LDS-tiled path keeps dz on chip (dz may be NULL).
int cmx_dwconv3x3_bwd(const void* da, const void* h, const float* w, const float* b, void* dz, void* dh, float* dw,
                      float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int act,
                      int accumulate, int dtype, hipStream_t s) {
  CMX_REQUIRE(C % 4 == 0 && NI % imgs_per_group == 0, CMX_ERR_SHAPE, "dwconv_bwd: C=%d", C);
  CMX_REQUIRE((long)NI * H * W * C < (1L << 31), CMX_ERR_SHAPE, "dwconv_bwd: tensor too large for 32-bit indexing");
  const int G = NI / imgs_per_group;
  const int CB = tile_cb(C, dtype);
  int P;
  if (CB) {
    const int tx = cdiv(W, TX2), ty = cdiv(H, TY2), ncb = C / CB;
    P = imgs_per_group * ty * tx;
    const dim3 grid((unsigned)P * ncb, G);
    CMX_DISPATCH(dtype, T, {
      CMX_ACT_DISPATCH(act, A, {
        if (CB == 32) {
          hipLaunchKernelGGL((dw2_bwd_kernel<T, 32, A>), grid, dim3(256), 0, s, (const T*)da, (const T*)h, w, b,
                             (T*)dh, workspace, imgs_per_group, H, W, C, tx, ty, ncb, P);
        } else if constexpr (sizeof(T) == 2) {
          hipLaunchKernelGGL((dw2_bwd_kernel<T, 64, A>), grid, dim3(256), 0, s, (const T*)da, (const T*)h, w, b,
                             (T*)dh, workspace, imgs_per_group, H, W, C, tx, ty, ncb, P);
        }
      });
    });
  } else {
    CMX_REQUIRE(dz, CMX_ERR_ARG, "dwconv_bwd: C=%d takes the strip path, which needs a dz buffer", C);
    const int CQ = C / 4;
    const int NXB = cdiv(W, RXB), NXS = cdiv(W, RXF), NYS = cdiv(H, RY);
    P = bwd_slots(CQ, NXB * NYS * imgs_per_group);
    CMX_DISPATCH(dtype, T, {
      CMX_ACT_DISPATCH(act, A, {
        hipLaunchKernelGGL((dw_bwd_dz_kernel<T, A>), dim3(cdiv((long)CQ * P, 256), G), dim3(256), 0, s, (const T*)da,
                           (const T*)h, w, b, (T*)dz, workspace, imgs_per_group, H, W, C, NXB, NYS, P);
      });
      if (dh) {
        const long threads = (long)CQ * NXS * NYS * imgs_per_group;
        hipLaunchKernelGGL((dw_fwd_kernel<T, true, 0>), dim3(cdiv(threads, 256), G), dim3(256), 0, s, (const T*)dz, w,
                           (const float*)nullptr, (T*)dh, imgs_per_group, H, W, C, NXS, NYS);
      }
    });
  }
  if (!dw && !db) return cmx_check_launch("dwconv_bwd");   // partials (G, P, C*10) left for a deferred reduce
  float* tmp = workspace + (size_t)G * P * C * 10;
  int st = cmx_reduce_partials(workspace, tmp, G, P, C * 10, 0, 1.f, s);
  if (st) return st;
  const long tot = (long)G * C * 10;
  hipLaunchKernelGGL(dw_scatter_kernel, dim3(cdiv(tot, 256) < 4096 ? cdiv(tot, 256) : 4096), dim3(256), 0, s, tmp, dw,
                     db, G, C, accumulate);
  return cmx_check_launch("dwconv_bwd");
}

}  // extern "C"

// gemm_kernels.h -- device code and launchers of the MFMA GEMM family (see gemm.hip for the
// design notes).  Split out so the template instantiations compile in parallel translation
// units: gemm_fast_bf16.hip / gemm_fast_f16.hip (the 16-bit LDS-DMA tile kernels),
// gemm_generic_*.hip (the register-staged path per element type), gemm.hip (entry points,
// grouped launches).  Launchers instantiated elsewhere are declared `extern template` in the
// TUs that call them (GEMM_EXTERN_LAUNCHERS below).
#pragma once
#include "cmx_mfma.h"
#include "cmx_dma.h"
#include <string.h>
#include <stdlib.h>

namespace gemmk {

struct GemmArgs {
  const void* A; const void* A2; const void* B; void* C; const float* bias; const void* R; const float* rscale;
  float* dbias; float* ws;
  int G, M, N, K, K1, kt_per_split, rows_per_sample, act, out_mode, tiles_m, tiles_n, ones_col, nsplit, vec, cvec;
  long lda, lda2, ldb, ldc, sA, sA2, sB, sC, sbias, sdb;
  // implicit convolution (NHWC input x of H x W x C per image, KH x KW taps, stride, pad -> Ho x Wo):
  //   conv = 1: A(i = output pixel, k = (kh, kw, c)) gathered from x (forward, no im2col);
  //   conv = 2: B(j = c, k = output pixel) = x at tap `ctap` of pixel k (weight gradient of one tap)
  int conv, cH, cW, cC, cKW, cst, cpad, cHo, cWo, ctap;
  // upsample-add epilogue (cmx_decoder_fuse_fwd): v += sum_s bilinear_s(up[s]) at output row i =
  // pixel (n, y, x) of an uoH x uoW grid; up[s] is (NB, uh[s], uw[s], N) in C's dtype
  const void* up[3];
  int uh[3], uw[3], nup, uoH, uoW;
  // scatter epilogue (cmx_conv_patch_dgrad): row i = patch (n, oy, ox) of an scHo x scWo grid,
  // column j = (kh, kw, c) of an scR x scR patch of scC channels -> C pixel (n, oy*scR + kh,
  // ox*scR + kw) of an scH x scW NHWC image (col2im of a non-overlapping patchify conv)
  int scatter, scH, scW, scC, scR, scHo, scWo;
  // two-level batch (cmx_gemm_h2): batch g = (g / gh, g % gh), operand offset
  // (g / gh) * sX + (g % gh) * sXh -- e.g. (image, head) pairs of per-head products; gh = 1:
  // the plain stride g * sX
  int gh;
  long sAh, sBh, sCh;
  // ReLU-backward mask (NULL: none): after the residual, C(i, j) = 0 where mask(i, j) <= 0; the
  // mask has C's layout and dtype (the saved ReLU output of the layer whose gradient this is)
  const void* mask;
  // LayerNorm in the epilogue (the consumer norm of a residual Linear's output: Block.norm2 after
  // proj, the next norm1 / stage norm after fc2, dual_segformer.py:168-169,382):
  // tail = 2 (N <= 128, N % 8 == 0: 64 x 64 / 64 x 128 tiles span the row): the same LayerNorm
  // in the epilogue by the lanes that store the row (row_layernorm), no tickets, no re-read
  // tail = 3: the LayerNorm BACKWARD in a dgrad's epilogue (row_layernorm_bwd): the GEMM result is
  // dy of a norm (rounded as it would be stored), C receives that norm's dx = LN'(dy [+ lnb_dy2])
  // + R (the residual branch's gradient), lnb_dxs = rscale[row / rows_per_sample] * dx, and
  // lnb_part[(g * tiles_m + tm) * 2N + (0 | N) + j] the tile's dgamma | dbeta column partials;
  // lnb_x = the norm's input, ln_gamma / ln_mean / ln_rstd its weight and saved statistics
  int tail;
  float ln_eps;
  const float* ln_gamma;
  const float* ln_beta;
  long ln_sg;                                  // gamma / beta group stride
  void* ln_y;
  float* ln_mean;
  float* ln_rstd;
  const void* lnb_x;
  const void* lnb_dy2;
  void* lnb_dxs;
  float* lnb_part;
};

// block id -> tile id, giving each of the 8 XCDs (hardware deals block b to XCD b % 8) a
// contiguous range of tiles so neighbouring tiles share an L2.  Bijective for any count.
__device__ __forceinline__ int xcd_tile(int b, int nt) {
  const int q = nt >> 3, r = nt & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// ---------------------------------------------------------------------------- epilogue
// bilinear taps of output row i in low-res map s: 4 element offsets (units of rows) + weights
struct UpTaps {
  long r00, r01, r10, r11;
  float w00, w01, w10, w11;
};
__device__ __forceinline__ UpTaps up_taps(const GemmArgs& p, int s, int i) {
  const int hw = p.uoH * p.uoW;
  const int n = i / hw, r = i - n * hw, y = r / p.uoW, x = r - y * p.uoW;
  const int h = p.uh[s], w = p.uw[s];
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  cmx_bilin_src(y, (float)h / p.uoH, h, y0, y1, ly0, ly1);
  cmx_bilin_src(x, (float)w / p.uoW, w, x0, x1, lx0, lx1);
  const long b = (long)n * h * w;
  return UpTaps{b + (long)y0 * w + x0, b + (long)y0 * w + x1, b + (long)y1 * w + x0, b + (long)y1 * w + x1,
                ly0 * lx0, ly0 * lx1, ly1 * lx0, ly1 * lx1};
}

// (the source loops are fully unrolled with `s < p.nup` guards: a runtime index into the
// argument struct's arrays would demote the whole struct to scratch memory)
template <typename T>
__device__ __forceinline__ float up_add1(const GemmArgs& p, int i, int j) {
  float v = 0.f;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (s < p.nup) {
      const UpTaps t = up_taps(p, s, i);
      const T* u = reinterpret_cast<const T*>(p.up[s]) + j;
      const long ld = p.N;
      v += t.w00 * to_f32(u[t.r00 * ld]) + t.w01 * to_f32(u[t.r01 * ld]) + t.w10 * to_f32(u[t.r10 * ld]) +
           t.w11 * to_f32(u[t.r11 * ld]);
    }
  }
  return v;
}

// 8 consecutive columns (16-B rows of the maps: N % 8 == 0 checked at launch)
template <typename T>
__device__ __forceinline__ void up_add8(const GemmArgs& p, int i, int j, float* v) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (s >= p.nup) continue;
    const UpTaps t = up_taps(p, s, i);
    const T* u = reinterpret_cast<const T*>(p.up[s]) + j;
    const long ld = p.N;
    float a[8], b[8], c[8], d[8];
    load_vec<T>(u + t.r00 * ld, a);
    load_vec<T>(u + t.r01 * ld, b);
    load_vec<T>(u + t.r10 * ld, c);
    load_vec<T>(u + t.r11 * ld, d);
    if constexpr (sizeof(T) == 4) {
      load_vec<T>(u + t.r00 * ld + 4, a + 4);
      load_vec<T>(u + t.r01 * ld + 4, b + 4);
      load_vec<T>(u + t.r10 * ld + 4, c + 4);
      load_vec<T>(u + t.r11 * ld + 4, d + 4);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t.w00 * a[e] + t.w01 * b[e] + t.w10 * c[e] + t.w11 * d[e];
  }
}

__device__ __forceinline__ long goff(const GemmArgs& p, int g, long s, long sh) {
  return p.gh > 1 ? (long)(g / p.gh) * s + (long)(g % p.gh) * sh : (long)g * s;
}

// element offset of C(g, i, j) under the patch scatter
__device__ __forceinline__ long scatter_offset(const GemmArgs& p, int g, int i, int j) {
  const int hw = p.scHo * p.scWo;
  const int n = i / hw, r = i - n * hw, oy = r / p.scWo, ox = r - oy * p.scWo;
  const int tap = j / p.scC, c = j - tap * p.scC, kh = tap / p.scR, kw = tap - kh * p.scR;
  return (long)g * p.sC + (((long)n * p.scH + oy * p.scR + kh) * p.scW + ox * p.scR + kw) * p.scC + c;
}

// element offset of C(g, i, j): row-major with ldc, or (EXT instantiations only) the patch scatter
template <bool EXT = true>
__device__ __forceinline__ long c_offset(const GemmArgs& p, int g, int i, int j) {
  if constexpr (EXT) {
    if (p.scatter) return scatter_offset(p, g, i, j);
  }
  return goff(p, g, p.sC, p.sCh) + (long)i * p.ldc + j;
}

// per-element epilogue of the generic (register-staged) kernel; the upsample-add and scatter
// extensions only in its EXT instantiations (inlined into the 16 x tiles unrolled epilogue
// loop they would spill the plain kernels' registers)
template <typename T, bool EXT = false>
__device__ __forceinline__ void epi_store(const GemmArgs& p, int g, int i, int j, float acc) {
  const float bj = p.bias ? p.bias[(long)g * p.sbias + j] : 0.f;
  if constexpr (EXT) {
    if (p.nup) acc += up_add1<T>(p, i, j);
  }
  float v = act_fwd(acc + bj, p.act);
  const long off = c_offset<EXT>(p, g, i, j);
  if (p.R) {
    const float sc = p.rscale ? p.rscale[((long)g * p.M + i) / p.rows_per_sample] : 1.f;
    v = to_f32(reinterpret_cast<const T*>(p.R)[off]) + sc * v;
  }
  if (p.mask && !(to_f32(reinterpret_cast<const T*>(p.mask)[off]) > 0.f)) v = 0.f;
  if (p.out_mode == 0) reinterpret_cast<T*>(p.C)[off] = from_f32<T>(v);
  else if (p.out_mode == 1) reinterpret_cast<float*>(p.C)[off] = v;
  else reinterpret_cast<float*>(p.C)[off] += v;
}

__device__ __forceinline__ void dbias_store(const GemmArgs& p, int g, int i, float v) {
  float* d = p.dbias + (long)g * p.sdb + i;
  *d = p.out_mode == 2 ? *d + v : v;
}

// 8 consecutive columns j..j+nv-1 of row i (nv <= 8).  p.vec8: C / R rows are 16-B aligned
// chunks, so a full group moves with one 16-B (bf16) or two 16-B (fp32) accesses
template <typename T>
__device__ __forceinline__ void epi_store8(const GemmArgs& p, int g, int i, int j, int nv, float* v) {
  if (nv < 8 || !p.cvec) {
    for (int e = 0; e < nv; ++e) epi_store<T, true>(p, g, i, j + e, v[e]);
    return;
  }
  if (p.bias) {
    const float* bp = p.bias + (long)g * p.sbias + j;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bp[e];
  }
  if (p.nup) up_add8<T>(p, i, j, v);
  if (p.act) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = act_fwd(v[e], p.act);
  }
  const long off = c_offset(p, g, i, j);
  if (p.R) {
    const float sc = p.rscale ? p.rscale[((long)g * p.M + i) / p.rows_per_sample] : 1.f;
    float rv[8];
    load_vec<T>(reinterpret_cast<const T*>(p.R) + off, rv);
    if constexpr (sizeof(T) == 4) load_vec<T>(reinterpret_cast<const T*>(p.R) + off + 4, rv + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rv[e] + sc * v[e];
  }
  if (p.mask) {
    float mv[8];
    load_vec<T>(reinterpret_cast<const T*>(p.mask) + off, mv);
    if constexpr (sizeof(T) == 4) load_vec<T>(reinterpret_cast<const T*>(p.mask) + off + 4, mv + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = mv[e] > 0.f ? v[e] : 0.f;
  }
  if (p.out_mode == 0) {
    store_vec<T>(reinterpret_cast<T*>(p.C) + off, v);
    if constexpr (sizeof(T) == 4) store_vec<T>(reinterpret_cast<T*>(p.C) + off + 4, v + 4);
  } else {
    float4* d = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + off);
    if (p.out_mode == 2) {
      const float4 o0 = d[0], o1 = d[1];
      v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w; v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
    }
    d[0] = make_float4(v[0], v[1], v[2], v[3]);
    d[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// split-K slabs: real columns ws[((g*S + z)*M + i)*Nr + j], bias-gradient column after them
// at ws[G*S*M*Nr + (g*S + z)*M + i]  (total G*S*M*N floats, N counting the ones column)
__device__ __forceinline__ float* slab(const GemmArgs& p, int g, int z) {
  const int Nr = p.ones_col ? p.N - 1 : p.N;
  return p.ws + (((long)g * p.nsplit + z) * p.M) * Nr;
}
__device__ __forceinline__ float* slab_db(const GemmArgs& p, int G, int g, int z) {
  const int Nr = p.N - 1;
  return p.ws + (long)G * p.nsplit * p.M * Nr + ((long)g * p.nsplit + z) * p.M;
}

// ============================================================================ bf16 fast path
constexpr int FBK = 64;                         // k per pipeline stage
// swizzle of the transposed image [64][ROWS]: 16-B chunk position of chunk c in k-row kk
template <int ROWS>
__device__ __forceinline__ int tr_swz(int kk) {
  if constexpr (ROWS == 128) return ((kk & 3) << 2) | ((kk >> 2) & 3);   // 256-B rows, 16 chunks
  else return ((kk >> 1) & 1) << 2;                                        // 128-B rows, 8 chunks
}

// k-contiguous operand tile -> image [ROWS][64] (128-B rows), chunk c of row r at position
// c ^ ((r >> 1) & 7).  ROWS / 32 LDS-DMA instructions per wave (8 rows each).
template <int ROWS>
__device__ __forceinline__ void stage_k(const i32x4 rsrc, char* img, long ld, int row0, int nrows, int k0, int kend,
                                        int w, int lane) {
  constexpr int NI = ROWS / 32;
#pragma unroll
  for (int n = 0; n < NI; ++n) {
    const int row = (w * NI + n) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int gr = row0 + row, gk = k0 + c * 8;
    const int off = (gr < nrows && gk < kend) ? (int)(((long)gr * ld + gk) * 2) : OOB;
    dma16(rsrc, lds_addr(img + (w * NI + n) * 1024), off);
  }
}

// row-contiguous operand tile -> image [64][ROWS] (ROWS*2-B k-rows), chunk c of k-row kk at
// position c ^ tr_swz(kk).  ROWS / 32 instructions per wave.
template <int ROWS>
__device__ __forceinline__ void stage_r(const i32x4 rsrc, char* img, long ld, int row0, int nrows, int k0, int kend,
                                        int w, int lane) {
  constexpr int NI = ROWS / 32;
  constexpr int CPR = ROWS / 8;                 // chunks per k-row
  constexpr int KPI = 64 / CPR;                 // k-rows per instruction
#pragma unroll
  for (int n = 0; n < NI; ++n) {
    const int kk = (w * NI + n) * KPI + lane / CPR;
    const int c = (lane % CPR) ^ tr_swz<ROWS>(kk);
    const int gk = k0 + kk, gr = row0 + c * 8;
    const int off = (gk < kend && gr < nrows) ? (int)(((long)gk * ld + gr) * 2) : OOB;
    dma16(rsrc, lds_addr(img + (w * NI + n) * 1024), off);
  }
}

template <typename E> using frag8 = typename MF<E>::frag;

// fragment of sub-tile rows [rb, rb + 32), k16-step s, from a [ROWS][64] image
template <typename E>
__device__ __forceinline__ frag8<E> frag_k(const char* img, int rb, int s, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int row = rb + r;
  const int pos = (2 * s + h) ^ ((row >> 1) & 7);
  return __builtin_bit_cast(frag8<E>, *reinterpret_cast<const uint4*>(img + row * 128 + pos * 16));
}

// same fragment from a transposed [64][ROWS] image: two ds_read_b64_tr_b16 (k 0-3, 4-7 of
// the lane's 8), each delivering column (16*g16 + i) of a 4 x 16 block
template <typename E, int ROWS>
__device__ __forceinline__ frag8<E> frag_r(const char* img, int rb, int s, int lane) {
  const int h = lane >> 5, g16 = (lane >> 4) & 1, i = lane & 15, q = i >> 2, pp = i & 3;
  const int col = rb + 16 * g16 + 4 * pp;
  const int chunk = col >> 3;
  s16x4 v[2];
#pragma unroll
  for (int rd = 0; rd < 2; ++rd) {
    const int kk = 16 * s + 8 * h + 4 * rd + q;
    const int off = kk * (ROWS * 2) + ((chunk ^ tr_swz<ROWS>(kk)) << 4) + ((pp & 1) << 3);
    v[rd] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4*>(reinterpret_cast<uintptr_t>(img + off)));
  }
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 c = __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8<E>, c);
}

// NS = LDS stages in the DMA ring: 2 for grids of >= 2 blocks per CU (the co-resident block
// hides the DMA latency), 4 for grids of at most one block per CU (the ring must hide it).
// LDS bytes of one block: the NS-stage DMA ring, reused by the fp32 epilogue tile
// KW = k-groups of 4 waves: KW = 2 runs 8 waves on one tile, group g multiplying the g-th 64-deep
// half of each 128-deep ring slot (twice the DMA and MFMA issue per tile: a small-grid GEMM
// with one 4-wave block per CU is bound by that issue rate, not by the CU's memory path)
template <int BM, int BN, int NS, int KW = 1>
constexpr int gemm_smem_bytes() {
  return NS * KW * (BM + BN) * FBK * 2 > KW * BM * (BN + 4) * 4 ? NS * KW * (BM + BN) * FBK * 2
                                                                 : KW * BM * (BN + 4) * 4;
}

// Row LayerNorm in the epilogue (GemmArgs::tail = 2): the tile spans the whole output row
// (tiles_n = 1, N <= BN), so the TPR lanes that store a row's 8-column chunks also normalise it:
// ln_y = LN(C row) * gamma + beta in C's dtype and layout, ln_mean / ln_rstd (fp32, g * M + i).
// The statistics are those of the stored (rounded) values, summed exactly as ln_fwd_kernel
// (layernorm.hip) sums a row of TPR 16-B chunks: 8 values per lane, then the xor tree over the
// TPR lanes -- so mean, rstd and the normalised row are bit-identical to the separate launch.
// Consumer norms of the residual Linears (Block.norm2 after proj, the next norm1 / stage norm
// after fc2, dual_segformer.py:168-169,382) at C <= 128 (stages 1-2) run here.
template <typename E, int TPR>
__device__ __forceinline__ void row_layernorm(const GemmArgs& p, int g, int i, int j, int jl, bool live,
                                              const float* v) {
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const cmx_f2 r = unpack2<E>(pack2<E>(v[e], v[e + 1]));
    x[e] = live ? r.x : 0.f;
    x[e + 1] = live ? r.y : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += x[e];
  s = group_sum(s, TPR);
  const int C = p.N;
  const float mu = s / C;
  float q = 0.f;
  if (live) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = x[e] - mu; q += d * d; }
  }
  q = group_sum(q, TPR);
  const float rs = rsqrtf(q / C + p.ln_eps);
  if (live) {
    const float* ga = p.ln_gamma + (long)g * p.ln_sg + j;
    const float* be = p.ln_beta + (long)g * p.ln_sg + j;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (x[e] - mu) * rs * ga[e] + be[e];
    store_vec<E>(reinterpret_cast<E*>(p.ln_y) + (long)g * p.sC + (long)i * p.ldc + j, o);
  }
  if (jl == 0) {
    p.ln_mean[(long)g * p.M + i] = mu;
    p.ln_rstd[(long)g * p.M + i] = rs;
  }
}

// LayerNorm backward in the epilogue (GemmArgs::tail = 3) of the dgrad that produces the norm's
// output gradient dy (Block.norm2's consumer fc1, dual_segformer.py:169): the TPR lanes of a row
// hold dy's 8-column chunks and finish the norm's backward without dy ever reaching HBM:
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) + dres,  g = dy * gamma,  xhat = (x - mu) rstd
// exactly as ln_bwd_kernel (layernorm.hip) computes a row of TPR 16-B chunks (dy rounded to the
// storage type first, as that kernel reads it), so dx and dxs are bit-identical to the separate
// launches whenever the separate dgrad sums k in the same order -- every shape but N = 128 on
// grids small enough for its 64 x 64 k-group blocks (two k-halves added at the end), where dy and
// so dx may differ by one rounding (tests/test_gpu_gemm.py::test_gemm_ln_bwd); the lane's dgamma /
// dbeta terms accumulate in dga / dba for the tile's partials.
// Under the patch scatter (cmx_conv_patch_dgrad_ln_bwd: the SR conv's input gradient, Attention.sr
// dual_segformer.py:95-96) a tile is one tap of 64 patches, i.e. 64 whole input-pixel rows of C =
// BN channels: the norm row is the scattered pixel, its statistics index the pixel.
template <typename E, int TPR>
__device__ __forceinline__ void row_layernorm_bwd(const GemmArgs& p, int g, int i, int j, int jl, bool live,
                                                  const float* v, float* dga, float* dba) {
  const int C = p.scatter ? p.scC : p.N;          // the norm's width
  const long off = c_offset(p, g, i, j);
  const long grow = p.scatter ? off / C : (long)g * p.M + i;
  const float mu = p.ln_mean[grow], rs = p.ln_rstd[grow];
  float dv[8], xh[8], gv[8];
  if (live) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const cmx_f2 r = unpack2<E>(pack2<E>(v[e], v[e + 1]));
      dv[e] = r.x;
      dv[e + 1] = r.y;
    }
    if (p.lnb_dy2) {
      float d2[8];
      load_vec<E>(reinterpret_cast<const E*>(p.lnb_dy2) + off, d2);
#pragma unroll
      for (int e = 0; e < 8; ++e) dv[e] += d2[e];
    }
    float xv[8];
    load_vec<E>(reinterpret_cast<const E*>(p.lnb_x) + off, xv);
    const float* ga = p.ln_gamma + (long)g * p.ln_sg + jl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[e] = (xv[e] - mu) * rs;
      gv[e] = dv[e] * ga[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) dv[e] = xh[e] = gv[e] = 0.f;
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1 += gv[e];
    s2 += gv[e] * xh[e];
  }
  s1 = group_sum(s1, TPR) / C;
  s2 = group_sum(s2, TPR) / C;
  if (!live) return;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    dga[e] += dv[e] * xh[e];
    dba[e] += dv[e];
    o[e] = rs * (gv[e] - s1 - xh[e] * s2);
  }
  if (p.R) {
    float rv[8];
    load_vec<E>(reinterpret_cast<const E*>(p.R) + off, rv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += rv[e];
  }
  store_vec<E>(reinterpret_cast<E*>(p.C) + off, o);
  if (p.lnb_dxs) {
    const float sc = p.rscale[grow / p.rows_per_sample];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= sc;
    store_vec<E>(reinterpret_cast<E*>(p.lnb_dxs) + off, o);
  }
}

// One output tile (of one split / group) of problem p.  `lin` = the block's linear index
// within the problem, in (split, group, tile) order; smem = gemm_smem_bytes<BM, BN, NS>().
// E = the 16-bit storage type (bf16 or f16: v_mfma_f32_32x32x16_bf16 / _f16, same tiles and rate)
template <int BM, int BN, bool TA, bool TB, int NS, int KW = 1, typename E = bf16, int EPI = 0>
__device__ __forceinline__ void gemm_bf16_body(const GemmArgs& p, const int lin, char* smem) {
  constexpr int A_BYTES = BM * FBK * 2, STAGE = (BM + BN) * FBK * 2, SLOT = KW * STAGE;
  constexpr int TM = BM / 64, TN = BN / 64;

  const int ntile = p.tiles_m * p.tiles_n;
  const int t = lin % ntile, g = (lin / ntile) % p.G, z = lin / (ntile * p.G);
  const int tm = t / p.tiles_n, tn = t % p.tiles_n;
  const E* Ag = reinterpret_cast<const E*>(p.A) + goff(p, g, p.sA, p.sAh);
  const E* A2g = p.A2 ? reinterpret_cast<const E*>(p.A2) + (long)g * p.sA2 : Ag;
  const E* Bg = reinterpret_cast<const E*>(p.B) + goff(p, g, p.sB, p.sBh);
  const i32x4 rA = make_rsrc(Ag), rA2 = make_rsrc(A2g), rB = make_rsrc(Bg);
  const int i0 = tm * BM, j0 = tn * BN;
  const int nreal = p.ones_col ? p.N - 1 : p.N;
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) & 3, kg = KW == 1 ? 0 : threadIdx.x >> 8;
  const int wm = w >> 1, wn = w & 1;
  const bool do_db = KW == 1 && p.ones_col && tn == 0 && wn == 0;   // this wave also sums its A rows

  f32x16 acc[TM][TN], accd[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    accd[a] = zero16();
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = zero16();
  }
  constexpr uint32_t one2 = (uint32_t)one_bits<E> * 0x10001u;
  const frag8<E> ones = __builtin_bit_cast(frag8<E>, make_uint4(one2, one2, one2, one2));

  const int nk = (p.K + FBK * KW - 1) / (FBK * KW);   // ring slots of KW x 64 k
  const int kt0 = z * p.kt_per_split;
  const int kt1 = min(nk, kt0 + p.kt_per_split);

  // conv = 1: this lane's output pixels (one per A-staging instruction), decoded once
  constexpr int NIA = BM / 32;
  int cv_y[NIA], cv_x[NIA], cv_base[NIA];
  if constexpr (!TA) {
    if (p.conv == 1) {
      const int hw = p.cHo * p.cWo;
#pragma unroll
      for (int n = 0; n < NIA; ++n) {
        const int gr = i0 + (w * NIA + n) * 8 + (lane >> 3);
        const int b = gr / hw, r2 = gr - b * hw, oy = r2 / p.cWo, ox = r2 - oy * p.cWo;
        cv_y[n] = gr < p.M ? oy * p.cst - p.cpad : -(1 << 28);   // out-of-range rows: never in bounds
        cv_x[n] = ox * p.cst - p.cpad;
        cv_base[n] = (b * p.cH + cv_y[n]) * p.cW + cv_x[n];
      }
    }
  }

  auto stage = [&](int kt, char* buf) {
    const int k0 = (kt * KW + kg) * FBK;
    buf += kg * STAGE;
    if constexpr (TA) {
      stage_r<BM>(rA, buf, p.lda, i0, p.M, k0, p.K, w, lane);
    } else {
      if (p.conv == 1) {
        // a 64-wide k-tile lies inside one tap (C % 64 == 0): tap uniform, 8 channels per chunk
        const int tap = k0 / p.cC, cb = k0 - tap * p.cC;
        const int kh = tap / p.cKW, kw = tap - kh * p.cKW;
#pragma unroll
        for (int n = 0; n < NIA; ++n) {
          const int row = (w * NIA + n) * 8 + (lane >> 3);
          const int c = (lane & 7) ^ ((row >> 1) & 7);
          const int iy = cv_y[n] + kh, ix = cv_x[n] + kw;
          const bool ok = k0 < p.K && iy >= 0 && iy < p.cH && ix >= 0 && ix < p.cW;
          const int off = ok ? ((cv_base[n] + kh * p.cW + kw) * p.cC + cb + c * 8) * 2 : OOB;
          dma16(rA, lds_addr(buf + (w * NIA + n) * 1024), off);
        }
      } else if (k0 < p.K1) {
        stage_k<BM>(rA, buf, p.lda, i0, p.M, k0, p.K1, w, lane);
      } else {
        stage_k<BM>(rA2, buf, p.lda2, i0, p.M, k0 - p.K1, p.K - p.K1, w, lane);
      }
    }
    if constexpr (TB) {
      if (p.conv == 2) {
        // B(j = channel, k = output pixel m) = x[pixel(m) at tap ctap][j]: rows of 8 channels
        constexpr int NI = BN / 32, CPR = BN / 8, KPI = 64 / CPR;
        const int hw = p.cHo * p.cWo;
        const int kh = p.ctap / p.cKW, kw = p.ctap - kh * p.cKW;
#pragma unroll
        for (int n = 0; n < NI; ++n) {
          const int kk = (w * NI + n) * KPI + lane / CPR;
          const int c = (lane % CPR) ^ tr_swz<BN>(kk);
          const int m = k0 + kk, gr = j0 + c * 8;
          int off = OOB;
          if (m < p.K && gr < nreal) {
            const int b = m / hw, r2 = m - b * hw, oy = r2 / p.cWo, ox = r2 - oy * p.cWo;
            const int iy = oy * p.cst - p.cpad + kh, ix = ox * p.cst - p.cpad + kw;
            if (iy >= 0 && iy < p.cH && ix >= 0 && ix < p.cW) off = (((b * p.cH + iy) * p.cW + ix) * p.cC + gr) * 2;
          }
          dma16(rB, lds_addr(buf + A_BYTES + (w * NI + n) * 1024), off);
        }
      } else {
        stage_r<BN>(rB, buf + A_BYTES, p.ldb, j0, nreal, k0, p.K, w, lane);
      }
    } else {
      stage_k<BN>(rB, buf + A_BYTES, p.ldb, j0, nreal, k0, p.K, w, lane);
    }
  };

  auto compute = [&](const char* buf) {
    buf += kg * STAGE;
    const char* ai = buf;
    const char* bi = buf + A_BYTES;
#pragma unroll
    for (int s = 0; s < FBK / 16; ++s) {
      frag8<E> fa[TM], fb[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int rb = wm * (BM / 2) + a * 32;
        if constexpr (TA) fa[a] = frag_r<E, BM>(ai, rb, s, lane);
        else fa[a] = frag_k<E>(ai, rb, s, lane);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int rb = wn * (BN / 2) + b * 32;
        if constexpr (TB) fb[b] = frag_r<E, BN>(bi, rb, s, lane);
        else fb[b] = frag_k<E>(bi, rb, s, lane);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = MF<E>::mma(fb[b], fa[a], acc[a][b]);
      if (do_db) {
#pragma unroll
        for (int a = 0; a < TM; ++a) accd[a] = MF<E>::mma(ones, fa[a], accd[a]);
      }
    }
  };

  // NS-deep ring of LDS stages: tile t + NS - 1 is issued before tile t is multiplied; the
  // counted wait before each barrier retires exactly the next tile (the DMA of the tiles after
  // it stays in flight across the barrier).  The WAR distance is one barrier: the stage being
  // refilled was last read in the previous iteration, which every wave has left.
  constexpr int PER = BM / 32 + BN / 32;        // LDS-DMA instructions per stage per wave
  auto wait_keep = [](int keep) {               // all but the `keep` most recent tiles landed
    if (NS > 7 && keep >= 7) vm_wait<7 * PER>();
    else if (NS > 6 && keep >= 6) vm_wait<6 * PER>();
    else if (NS > 5 && keep == 5) vm_wait<5 * PER>();
    else if (NS > 4 && keep == 4) vm_wait<4 * PER>();
    else if (NS > 3 && keep == 3) vm_wait<3 * PER>();
    else if (keep >= 2) vm_wait<2 * PER>();
    else if (keep == 1) vm_wait<PER>();
    else vm_wait<0>();
  };
  const int pro = min(NS - 1, kt1 - kt0);
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < pro) stage(kt0 + q, smem + q * SLOT);
  wait_keep(pro - 1);
  __syncthreads();
  int cur = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    const int nxt = cur == 0 ? NS - 1 : cur - 1;
    if (kt + NS - 1 < kt1) stage(kt + NS - 1, smem + nxt * SLOT);
    compute(smem + cur * SLOT);
    // tiles kt+1 .. kt+ahead are in flight; retire tile kt+1, keep the rest
    const int ahead = min(NS - 1, kt1 - 1 - kt);
    wait_keep(ahead - 1);
    __syncthreads();
    cur = cur + 1 == NS ? 0 : cur + 1;
  }

  // epilogue through LDS.  acc[a][b] holds C^T (B fragment fed as the MFMA's A operand), so
  // lane (r, h) register q is C(i = r, j = accrow(q, h)) of its 32x32 sub-tile and registers
  // 4g..4g+3 are 4 consecutive j: one ds_write_b128 each into a row-major fp32 tile (pitch
  // BN + 4 floats: the 8 lanes of a write group hit 8 distinct 4-bank slots).  The tile is
  // then read back 8 consecutive columns per thread and stored with 16-B (bf16) / 32-B
  // (fp32) row-contiguous stores, the epilogue applied on the way.
  const int r = lane & 31, h = lane >> 5;
  constexpr int CP = BN + 4;
  float* cs = reinterpret_cast<float*>(smem) + kg * BM * CP;     // one fp32 image per k-group
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int il = wm * (BM / 2) + a * 32 + r, jl = wn * (BN / 2) + b * 32 + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(cs + il * CP + jl) =
            make_float4(acc[a][b][4 * g4], acc[a][b][4 * g4 + 1], acc[a][b][4 * g4 + 2], acc[a][b][4 * g4 + 3]);
      }
  if (do_db && h == 0) {        // accd[a] = ones * A^T: every register of lane r is sum_k A(r, k)
    float* wd = p.nsplit > 1 ? slab_db(p, p.G, g, z) : nullptr;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int i = i0 + wm * (BM / 2) + a * 32 + r;
      if (i < p.M) {
        if (wd) wd[i] = accd[a][0];
        else dbias_store(p, g, i, accd[a][0]);
      }
    }
  }
  __syncthreads();
  cs = reinterpret_cast<float*>(smem);
  constexpr int TPR = BN / 8, RPP = 256 * KW / TPR, NPASS = (BM + RPP - 1) / RPP;
  const int jl = (threadIdx.x % TPR) * 8;
  const int j = j0 + jl;
  const bool live = j < nreal;
  if (EPI < 2 && !live) return;             // (row LayerNorm: every lane of a row takes part)
  const int nv = min(8, nreal - j);
  float* wsz = p.nsplit > 1 ? slab(p, g, z) : nullptr;
  float dga[8], dba[8];                      // (tail = 3: this lane's dgamma / dbeta column terms)
#pragma unroll
  for (int e = 0; e < 8; ++e) dga[e] = dba[e] = 0.f;
#pragma unroll 2
  for (int pass = 0; pass < NPASS; ++pass) {
    const int il = pass * RPP + threadIdx.x / TPR;
    const int i = i0 + il;
    if (il >= BM || i >= p.M) break;
    float v[8];
    const float4 u0 = *reinterpret_cast<const float4*>(cs + il * CP + jl);
    const float4 u1 = *reinterpret_cast<const float4*>(cs + il * CP + jl + 4);
    v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w; v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
#pragma unroll
    for (int q = 1; q < KW; ++q) {              // the other k-groups' partial images
      const float4 w0 = *reinterpret_cast<const float4*>(cs + q * BM * CP + il * CP + jl);
      const float4 w1 = *reinterpret_cast<const float4*>(cs + q * BM * CP + il * CP + jl + 4);
      v[0] += w0.x; v[1] += w0.y; v[2] += w0.z; v[3] += w0.w; v[4] += w1.x; v[5] += w1.y; v[6] += w1.z; v[7] += w1.w;
    }
    if constexpr (EPI == 2) {
      if (live) epi_store8<E>(p, g, i, j, 8, v);   // v: the stored row values before rounding
      row_layernorm<E, TPR>(p, g, i, j, jl, live, v);
    } else if constexpr (EPI == 3) {
      row_layernorm_bwd<E, TPR>(p, g, i, j, jl, live, v, dga, dba);
    } else if (wsz) {
      float* d = wsz + (long)i * nreal + j;
      if (nv == 8 && (nreal & 3) == 0) {
        reinterpret_cast<float4*>(d)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(d)[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        for (int e = 0; e < nv; ++e) d[e] = v[e];
      }
    } else {
      epi_store8<E>(p, g, i, j, nv, v);
    }
  }
  if constexpr (EPI == 3) {
    // the tile's dgamma | dbeta column partials: the RPP row slots' lane sums meet in LDS
    __syncthreads();                                  // every lane is done with the fp32 C image
    float* red = reinterpret_cast<float*>(smem);      // [RPP][2][BN]
    const int rsl = threadIdx.x / TPR;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rsl * 2) * BN + jl + e] = dga[e];
      red[(rsl * 2 + 1) * BN + jl + e] = dba[e];
    }
    __syncthreads();
    const int C = p.scatter ? p.scC : p.N;         // the norm's width (= BN under the scatter)
    for (int c = threadIdx.x; c < 2 * BN; c += 256 * KW) {
      const int which = c / BN, col = c - which * BN;
      if (col >= C || j0 + col >= nreal) continue;
      float a = 0.f;
      for (int q = 0; q < RPP; ++q) a += red[(q * 2 + which) * BN + col];
      p.lnb_part[(((long)g * p.tiles_m + tm) * p.tiles_n + tn) * 2 * C + which * C + col] = a;
    }
  }
}

// 1-D grid over (split, group, tile); each XCD gets a contiguous run of that order, i.e.
// neighbouring tiles of one (split, group): they share A row panels and the B k-slice in L2
// (64 x 64 two-stage blocks take 32 KB of LDS: five fit a CU when the kernel stays within 96
// VGPRs, which the launch bound asks of the register allocator -- at 97 only four are resident)
template <int BM, int BN, bool TA, bool TB, int NS, int KW = 1, typename E = bf16, int TAIL = 0>
__global__ __launch_bounds__(256 * KW, (BM == 64 && BN == 64 && NS == 2 && KW == 1) ? 5 : (KW == 4 ? 1 : 2))
void gemm_bf16_kernel(const GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[gemm_smem_bytes<BM, BN, NS, KW>()];
  const int lin = xcd_tile(blockIdx.x, p.tiles_m * p.tiles_n * p.G * p.nsplit);
  gemm_bf16_body<BM, BN, TA, TB, NS, KW, E, TAIL>(p, lin, smem);
}

// ============================================================================ streaming launch
// Tall products on 64 x 64 tiles (tens of thousands of rows, a few k-steps: the stage-1/2
// Linears and their input gradients, G = 2 modalities).  The one-tile block above is a latency
// chain -- DMA, MFMA, epilogue store, retire -- and the chip runs ~2-4 rounds of them.  Here a
// resident grid (CMX_STREAM_LB = 4 blocks per CU) walks the tiles, and each block's 2-slot LDS ring runs ACROSS
// tile boundaries: the next tile's first k-step is in flight while this tile's epilogue stores.
// Tiles are dealt to XCDs in contiguous ranges (block b sits on XCD b % 8), so the column tiles
// of one row panel share that XCD's L2.  The epilogue's fp32 image takes the slot just consumed
// (64 x 64 floats, 16-B chunks XOR-swizzled by row instead of padded: it fits one 16 KB stage).
// Epilogues: the plain one (bias / act / residual / mask / fp32 out) and the row LayerNorm
// (EPI = 2, N <= 64).  No split-K, transA, A2, implicit conv, bias column, upsample or scatter.
constexpr int STREAM_SLOT = 64 * FBK * 2 * 2;   // one stage: A + B images, 64 x 64 each (16 KB)
#ifndef CMX_STREAM_LB
#define CMX_STREAM_LB 4                          // resident blocks per CU the registers are sized for
#endif
template <bool TB, typename E, int EPI>
__global__ __launch_bounds__(256, CMX_STREAM_LB) void gemm_stream_kernel(const GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STREAM_SLOT];
  constexpr int A_BYTES = 64 * FBK * 2;
  const int ntile = p.tiles_m * p.tiles_n, total = ntile * p.G;
  const int nk = (p.K + FBK - 1) / FBK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int nreal = p.N;
  // XCD x = blockIdx.x % 8 takes tiles [lo, hi) round-robin over its nbx blocks
  const int nbx = gridDim.x >> 3, xb = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int per = (total + 7) >> 3, lo = xb * per, hi = min(total, lo + per);
  const int first = lo + bi;
  const int nq = first < hi ? (hi - first + nbx - 1) / nbx : 0;
  const int S = nq * nk;
  if (S == 0) return;
  auto tile_of = [&](int q, int& g, int& tm, int& tn) {
    const int lin = first + q * nbx;
    const int t = lin % ntile;
    g = lin / ntile;
    tm = t / p.tiles_n;
    tn = t - tm * p.tiles_n;
  };
  auto stage = [&](int st, char* buf) {
    const int q = st / nk, kt = st - q * nk;
    int g, tm, tn;
    tile_of(q, g, tm, tn);
    const i32x4 rA = make_rsrc(reinterpret_cast<const E*>(p.A) + goff(p, g, p.sA, p.sAh));
    const i32x4 rB = make_rsrc(reinterpret_cast<const E*>(p.B) + goff(p, g, p.sB, p.sBh));
    const int k0 = kt * FBK;
    stage_k<64>(rA, buf, p.lda, tm * 64, p.M, k0, p.K, w, lane);
    if constexpr (TB) stage_r<64>(rB, buf + A_BYTES, p.ldb, tn * 64, nreal, k0, p.K, w, lane);
    else stage_k<64>(rB, buf + A_BYTES, p.ldb, tn * 64, nreal, k0, p.K, w, lane);
  };
  f32x16 acc = zero16();
  auto compute = [&](const char* buf) {
    const char* ai = buf;
    const char* bi_ = buf + A_BYTES;
#pragma unroll
    for (int s = 0; s < FBK / 16; ++s) {
      const frag8<E> fa = frag_k<E>(ai, wm * 32, s, lane);
      frag8<E> fb;
      if constexpr (TB) fb = frag_r<E, 64>(bi_, wn * 32, s, lane);
      else fb = frag_k<E>(bi_, wn * 32, s, lane);
      acc = MF<E>::mma(fb, fa, acc);
    }
  };
  // image element (row il, column jl): 16-B chunk jl / 4 of the row at position chunk ^ (il & 15)
  auto img = [](float* cs, int il, int c4) { return cs + il * 64 + ((c4 ^ (il & 15)) << 2); };
  auto epilogue = [&](int q, float* cs) {
    int g, tm, tn;
    tile_of(q, g, tm, tn);
    const int i0 = tm * 64, j0 = tn * 64;
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int il = wm * 32 + r, c4 = wn * 8 + 2 * g4 + h;
      *reinterpret_cast<float4*>(img(cs, il, c4)) =
          make_float4(acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]);
    }
    __syncthreads();
    constexpr int TPR = 8, RPP = 256 / TPR;
    const int jl = (threadIdx.x % TPR) * 8, j = j0 + jl;
    const bool live = j < nreal;
    const int nv = min(8, nreal - j);
#pragma unroll
    for (int pass = 0; pass < 64 / RPP; ++pass) {
      const int il = pass * RPP + threadIdx.x / TPR;
      const int i = i0 + il;
      if (i >= p.M) break;
      const float4 u0 = *reinterpret_cast<const float4*>(img(cs, il, jl / 4));
      const float4 u1 = *reinterpret_cast<const float4*>(img(cs, il, jl / 4 + 1));
      float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      if constexpr (EPI == 2) {
        if (live) epi_store8<E>(p, g, i, j, 8, v);
        row_layernorm<E, TPR>(p, g, i, j, jl, live, v);
      } else {
        if (live) epi_store8<E>(p, g, i, j, nv, v);
      }
    }
  };
  stage(0, smem);
  vm_wait<0>();
  __syncthreads();
  int cur = 0;
  for (int st = 0; st < S; ++st) {
    if (st + 1 < S) stage(st + 1, smem + (cur ^ 1) * STREAM_SLOT);
    compute(smem + cur * STREAM_SLOT);
    const int q = st / nk;
    if (st - q * nk == nk - 1) {
      __syncthreads();                          // every wave has read its last fragments of slot cur
      epilogue(q, reinterpret_cast<float*>(smem + cur * STREAM_SLOT));
      acc = zero16();
    }
    vm_wait<0>();                               // the next stage has landed (and this tile's stores)
    __syncthreads();                            // ... and slot cur is free for the stage after it
    cur ^= 1;
  }
}

// ============================================================================ multi launch
// Up to four independent forward / dgrad problems (64 x 64 tiles, no split-K, same B layout) in
// ONE grid, records passed by value: e.g. Attention.q beside Attention.kv (dual_segformer.py:
// 114-121; both read norm1's output or its spatial reduction) and the decoder's four
// linear_c* projections (MLPDecoder.py:66-73).  Block b runs problem i with blk0[i] <= b.
constexpr int MULTI_MAX = 4;
struct GemmMulti {
  GemmArgs a[MULTI_MAX];
  int blk0[MULTI_MAX + 1];
  int n;
};

template <int NS, int KW, bool TB, typename E>
__global__ __launch_bounds__(256 * KW, (NS == 2 && KW == 1) ? 5 : 2) void gemm_multi_kernel(const GemmMulti m) {
  __shared__ __attribute__((aligned(1024))) char smem[gemm_smem_bytes<64, 64, NS, KW>()];
  const int b = blockIdx.x;
  int i = 0;
#pragma unroll
  for (int j = 1; j < MULTI_MAX; ++j)
    if (j < m.n && b >= m.blk0[j]) i = j;
  const int nb = m.blk0[i + 1] - m.blk0[i];
  gemm_bf16_body<64, 64, false, TB, NS, KW, E>(m.a[i], xcd_tile(b - m.blk0[i], nb), smem);
}

// ============================================================================ grouped launch
// Many independent problems in ONE launch (the weight gradients of a whole backward segment,
// which nothing reads before the optimizer): record r owns blocks [blk0, blk0 + nblk) of the
// grid.  The XCD remap runs over the whole grid, so each XCD takes a contiguous run of
// (problem, split, group, tile) and neighbouring tiles of one problem still share L2.  The
// tile shape is chosen per problem (the output's narrow side gets 64), so a 64 x 64 stage-1
// weight gradient and a 512 x 2048 decoder one share the launch without padding waste.
struct GroupRec {
  GemmArgs a;
  int bm, bn, blk0, nblk;
};

// chunked round-robin block -> tile map: runs of `ch` consecutive tiles (neighbours sharing
// operand panels in one L2) are dealt to the 8 XCDs in turn, so problems whose tiles cost very
// different k-loop lengths spread over every XCD instead of loading the one whose contiguous
// range they fall in (xcd_tile).  Tiles past the last whole round keep the identity map.
__device__ __forceinline__ int xcd_chunk_tile(int b, int nt, int ch) {
  const int full = nt / (8 * ch) * (8 * ch);
  if (b >= full) return b;
  const int x = b & 7, j = b >> 3;
  return ((j / ch) * 8 + x) * ch + j % ch;
}

// (two-stage DMA ring, two blocks per CU: deeper rings at one block per CU measured 2-17 %
// slower on the B2 step, round 3)
// one block's tile of the grouped launch: the record whose block range holds `lin`
template <typename E, int NS>
__device__ __forceinline__ void grouped_tile(const GroupRec* __restrict__ recs, int nrec, int lin, char* smem) {
  int lo = 0, hi = nrec - 1;                    // last record with blk0 <= lin
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (recs[mid].blk0 <= lin) lo = mid; else hi = mid - 1;
  }
  const GroupRec& r = recs[lo];
  const GemmArgs p = r.a;
  const int local = lin - r.blk0;
  if (r.bm == 128 && r.bn == 128) gemm_bf16_body<128, 128, true, true, NS, 1, E>(p, local, smem);
  else if (r.bm == 128) gemm_bf16_body<128, 64, true, true, NS, 1, E>(p, local, smem);
  else if (r.bn == 128) gemm_bf16_body<64, 128, true, true, NS, 1, E>(p, local, smem);
  else gemm_bf16_body<64, 64, true, true, NS, 1, E>(p, local, smem);
}

// LOOP: a grid smaller than `total` (a multiple of 8 workgroups: block b + k * gridDim.x stays on
// block b's XCD) walks the blocks b, b + gridDim.x, ... in turn (cmx_gemm_grouped_capped).  The
// one-tile-per-block instantiation stays separate: the loop around the k-loop body cost the
// full-grid launch 40 % (round 5: 522-570 us -> 770-850 us on the B2 step)
template <typename E, int NS = 2, bool LOOP = false>
__global__ __launch_bounds__(256, 2) void gemm_grouped_kernel(const GroupRec* __restrict__ recs, int nrec,
                                                                             int chunk, int total) {
  __shared__ __attribute__((aligned(1024))) char smem[gemm_smem_bytes<128, 128, NS>()];
  if constexpr (!LOOP) {
    const int b = blockIdx.x;
    grouped_tile<E, NS>(recs, nrec, chunk > 0 ? xcd_chunk_tile(b, total, chunk) : xcd_tile(b, total), smem);
  } else {
    for (int b = blockIdx.x; b < total; b += gridDim.x) {
      if (b != (int)blockIdx.x) __syncthreads();   // every wave is done with the previous tile's LDS
      grouped_tile<E, NS>(recs, nrec, chunk > 0 ? xcd_chunk_tile(b, total, chunk) : xcd_tile(b, total), smem);
    }
  }
}

// ============================================================================ generic path
constexpr int BK = 32;

template <typename T> struct Stage;
template <> struct Stage<bf16> { static constexpr int V = 8, PAD = 8; typedef uint4 raw; };
template <> struct Stage<f16> { static constexpr int V = 8, PAD = 8; typedef uint4 raw; };
template <> struct Stage<float> { static constexpr int V = 4, PAD = 4; typedef float4 raw; };

template <typename T, int ROWS>
struct TileLoader {
  // One operand tile: ROWS (i or j) x BK (k).  Per thread: CH chunks of V contiguous
  // elements along the operand's contiguous dim (element-wise when !vec: ragged dims).
  static constexpr int V = Stage<T>::V;
  static constexpr int CHUNKS = ROWS * BK / V;
  static constexpr int CH = CHUNKS / 256;
  static_assert(CHUNKS % 256 == 0, "tile must split evenly over 256 threads");
  typename Stage<T>::raw r[CH];

  // rows [row0, nrows) valid, k in [k0, k0 + BK) of a segment with kend valid k;
  // ones_row >= 0: that (virtual) row is all ones for valid k
  template <bool TRANS>
  __device__ __forceinline__ void load(const T* __restrict__ P, long ld, int row0, int nrows, int k0, int kend,
                                       int ones_row, bool vec) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int q = threadIdx.x + c * 256;
      int row, k;
      if (!TRANS) {              // chunk = V consecutive k of one row
        row = q / (BK / V);
        k = (q % (BK / V)) * V;
      } else {                   // chunk = V consecutive rows of one k
        k = q / (ROWS / V);
        row = (q % (ROWS / V)) * V;
      }
      const int gr = row0 + row, gk = k0 + k;
      r[c] = typename Stage<T>::raw{};
      if (vec) {
        if (gk < kend) {
          if (gr < nrows) {
            const T* p = !TRANS ? P + (long)gr * ld + gk : P + (long)gk * ld + gr;
            r[c] = *reinterpret_cast<const typename Stage<T>::raw*>(p);
          } else if (TRANS && gr == ones_row) {
            reinterpret_cast<T*>(&r[c])[0] = from_f32<T>(1.f);
          }
        }
      } else {
        T* e = reinterpret_cast<T*>(&r[c]);
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int rr = TRANS ? gr + v : gr, kk = TRANS ? gk : gk + v;
          if (kk < kend) {
            if (rr < nrows) e[v] = !TRANS ? P[(long)rr * ld + kk] : P[(long)kk * ld + rr];
            else if (TRANS && rr == ones_row) e[v] = from_f32<T>(1.f);
          }
        }
      }
    }
  }

  template <bool TRANS>
  __device__ __forceinline__ void store(T* __restrict__ S) {   // S: [ROWS][BK + PAD]
    constexpr int LD = BK + Stage<T>::PAD;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int q = threadIdx.x + c * 256;
      if (!TRANS) {
        const int row = q / (BK / V), k = (q % (BK / V)) * V;
        *reinterpret_cast<typename Stage<T>::raw*>(S + row * LD + k) = r[c];
      } else {
        const int k = q / (ROWS / V), row = (q % (ROWS / V)) * V;
        const T* e = reinterpret_cast<const T*>(&r[c]);
#pragma unroll
        for (int v = 0; v < V; ++v) S[(row + v) * LD + k] = e[v];
      }
    }
  }
};

template <typename T, int BM, int BN, bool TA, bool TB, bool EXT>
__global__ __launch_bounds__(256) void gemm_generic_kernel(const GemmArgs p) {
  typedef MF<T> mf;
  constexpr int LD = BK + Stage<T>::PAD;
  constexpr int TM = BM / 64, TN = BN / 64;     // 32x32 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) T As[2][BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LD];

  const int t = xcd_tile(blockIdx.x, p.tiles_m * p.tiles_n);
  const int tm = t / p.tiles_n, tn = t % p.tiles_n;
  const int g = blockIdx.y, z = blockIdx.z;
  const T* Ag = reinterpret_cast<const T*>(p.A) + goff(p, g, p.sA, p.sAh);
  const T* A2g = p.A2 ? reinterpret_cast<const T*>(p.A2) + (long)g * p.sA2 : nullptr;
  const T* Bg = reinterpret_cast<const T*>(p.B) + goff(p, g, p.sB, p.sBh);
  const int i0 = tm * BM, j0 = tn * BN;
  const int nreal = p.ones_col ? p.N - 1 : p.N;     // real B rows (the ones row is virtual)
  const int ones_row = p.ones_col ? p.N - 1 : -1;
  const bool vec = p.vec;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = zero16();

  TileLoader<T, BM> la;
  TileLoader<T, BN> lb;
  const int nk_all = (p.K + BK - 1) / BK;
  const int kt0 = z * p.kt_per_split;
  const int kt1 = min(nk_all, kt0 + p.kt_per_split);

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if (k0 < p.K1) la.template load<TA>(Ag, p.lda, i0, p.M, k0, p.K1, -1, vec);
    else la.template load<TA>(A2g, p.lda2, i0, p.M, k0 - p.K1, p.K - p.K1, -1, vec);
    lb.template load<TB>(Bg, p.ldb, j0, nreal, k0, p.K, ones_row, vec);
  };

  if (kt0 < kt1) {
    load_tile(kt0);
    la.template store<TA>(As[0]);
    lb.template store<TB>(Bs[0]);
  }
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    if (kt + 1 < kt1) load_tile(kt + 1);
    const T* as = As[cur];
    const T* bs = Bs[cur];
#pragma unroll
    for (int s = 0; s < BK / mf::KI; ++s) {
      typename mf::frag fa[TM], fb[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) fa[a] = mf::load(as + (wm * (BM / 2) + a * 32 + r) * LD + s * mf::KI + mf::E * h);
#pragma unroll
      for (int b = 0; b < TN; ++b) fb[b] = mf::load(bs + (wn * (BN / 2) + b * 32 + r) * LD + s * mf::KI + mf::E * h);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mf::mma(fa[a], fb[b], acc[a][b]);
    }
    if (kt + 1 < kt1) {
      la.template store<TA>(As[cur ^ 1]);
      lb.template store<TB>(Bs[cur ^ 1]);
    }
    __syncthreads();
  }

  // epilogue: MFMA operand A supplies rows (i), B supplies columns (j): accumulator
  // register q of lane (r, h) is C(i = tile row accrow(q, h), j = tile col r).
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int j = j0 + wn * (BN / 2) + b * 32 + r;
    if (j >= p.N) continue;
    const bool dbcol = j == ones_row;
    if (p.nsplit > 1) {
      float* wsz = dbcol ? slab_db(p, p.G, g, z) : slab(p, g, z);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = i0 + wm * (BM / 2) + a * 32 + accrow(q, h);
          if (i < p.M) {
            if (dbcol) wsz[i] = acc[a][b][q];
            else wsz[(long)i * nreal + j] = acc[a][b][q];
          }
        }
      continue;
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + wm * (BM / 2) + a * 32 + accrow(q, h);
        if (i >= p.M) continue;
        if (dbcol) dbias_store(p, g, i, acc[a][b][q]);
        else epi_store<T, EXT>(p, g, i, j, acc[a][b][q]);
      }
    }
  }
}

// ============================================================================ split-K reducer
// Sums the nsplit slabs and applies the full epilogue.  A thread owns one group of 8
// consecutive output columns and every ZL-th slab (ZL z-lanes per group: the wgrads carry up
// to 64 slabs, and a lone thread walking them serially is latency-bound); the z-lanes meet
// in LDS and lane 0 finishes the group.  Groups past M x ceil(Nr/8) are bias-gradient rows.
template <typename T, int ZL>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs p) {
  constexpr int GPB = 256 / ZL;                 // groups per block
  __shared__ float4 red[ZL > 1 ? ZL - 1 : 1][GPB][2];
  const int g = blockIdx.y;
  const int Nr = p.ones_col ? p.N - 1 : p.N;
  const int ng = (Nr + 7) >> 3;
  const long MN = (long)p.M * Nr;
  const long work = (long)p.M * ng;
  const int gl = threadIdx.x % GPB, zl = threadIdx.x / GPB;
  const long e = (long)blockIdx.x * GPB + gl;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0, j = 0, nv = 0;
  if (e < work) {
    i = (int)(e / ng); j = (int)(e % ng) * 8; nv = min(8, Nr - j);
    const float* src = slab(p, g, 0) + (long)i * Nr + j;
    if (nv == 8 && (Nr & 3) == 0) {
      int z = zl;
#pragma unroll 4
      for (; z < p.nsplit; z += ZL) {
        const float4 a = reinterpret_cast<const float4*>(src + (long)z * MN)[0];
        const float4 b = reinterpret_cast<const float4*>(src + (long)z * MN)[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
    } else {
      for (int z = zl; z < p.nsplit; z += ZL)
        for (int c = 0; c < nv; ++c) v[c] += src[(long)z * MN + c];
    }
  } else if (p.ones_col && e < work + p.M) {
    const float* src = slab_db(p, p.G, g, 0) + (e - work);
#pragma unroll 4
    for (int z = zl; z < p.nsplit; z += ZL) v[0] += src[(long)z * p.M];
  }
  if constexpr (ZL > 1) {
    if (zl > 0) {
      red[zl - 1][gl][0] = make_float4(v[0], v[1], v[2], v[3]);
      red[zl - 1][gl][1] = make_float4(v[4], v[5], v[6], v[7]);
    }
    __syncthreads();
    if (zl > 0) return;
#pragma unroll
    for (int q = 0; q < ZL - 1; ++q) {
      const float4 a = red[q][gl][0], b = red[q][gl][1];
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
  }
  if (e < work) epi_store8<T>(p, g, i, j, nv, v);
  else if (p.ones_col && e < work + p.M) dbias_store(p, g, (int)(e - work), v[0]);
}

template <typename T>
void launch_reduce(const GemmArgs& a, int G, long groups, hipStream_t s) {
  if (a.nsplit >= 32) hipLaunchKernelGGL((splitk_reduce_kernel<T, 16>), dim3(cdiv(groups, 16), G), dim3(256), 0, s, a);
  else if (a.nsplit >= 8) hipLaunchKernelGGL((splitk_reduce_kernel<T, 4>), dim3(cdiv(groups, 64), G), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((splitk_reduce_kernel<T, 1>), dim3(cdiv(groups, 256), G), dim3(256), 0, s, a);
}

// ============================================================================ host side
template <int BM, int BN, int NS, int KW = 1, typename E = bf16>
void launch_bf16(const GemmArgs& a, int G, int nsplit, int tA, int tB, hipStream_t s) {
  dim3 grid(a.tiles_m * a.tiles_n * G * nsplit);
  if constexpr (BM == 64 && (BN == 64 || (BN == 128 && KW == 1))) {
    if (a.tail == 2) {                // whole-row LayerNorm in the epilogue (forward layouts, tiles_n = 1)
      hipLaunchKernelGGL((gemm_bf16_kernel<64, BN, false, false, NS, KW, E, 2>), grid, dim3(256 * KW), 0, s, a);
      return;
    }
    if (a.tail == 3) {                // LayerNorm backward in a dgrad's epilogue (transB = 1, tiles_n = 1)
      hipLaunchKernelGGL((gemm_bf16_kernel<64, BN, false, true, NS, KW, E, 3>), grid, dim3(256 * KW), 0, s, a);
      return;
    }
  }
#define CMX_GEMM_LAUNCH(TA, TB) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, TA, TB, NS, KW, E>), grid, dim3(256 * KW), 0, s, a)
  if (!tA && !tB) CMX_GEMM_LAUNCH(false, false);
  else if (!tA && tB) CMX_GEMM_LAUNCH(false, true);
  else if (tA && tB) CMX_GEMM_LAUNCH(true, true);
  else CMX_GEMM_LAUNCH(true, false);
#undef CMX_GEMM_LAUNCH
}

template <int BM, int BN, typename E = bf16>
void launch_bf16_ns(const GemmArgs& a, int G, int nsplit, int tA, int tB, hipStream_t s) {
  const long blocks = (long)a.tiles_m * a.tiles_n * G * nsplit;
  // k-group blocks for 64 x 64 tiles without split-K or bias column (CMX_GEMM_KW = the largest
  // group count allowed, default 2; 1 = off).  Measured (scripts/gemm_sweep.py, G2 M600 N512):
  // K 2048 20.1 -> 11.9 us, K 512 7.5 -> 5.8 us at KW = 2; grids above 512 blocks and one-slot
  // problems are slower with it (M9600 N128 K512: 9.7 -> 10.4 us), so they keep 4 waves.
  static int& kw = cmx_knob("GEMM_KW", 2);
  if constexpr (BM == 64 && BN == 64) {
    const int nk64 = (a.K + FBK - 1) / FBK;
    if (kw >= 2 && nsplit == 1 && !a.ones_col && blocks <= 512 && nk64 >= 4) {
      GemmArgs b = a;
      if (kw >= 4 && blocks <= 256 && nk64 >= 16) {
        b.kt_per_split = (b.K + 4 * FBK - 1) / (4 * FBK);
        launch_bf16<64, 64, 2, 4, E>(b, G, nsplit, tA, tB, s);
        return;
      }
      b.kt_per_split = (b.K + 2 * FBK - 1) / (2 * FBK);
      if (blocks <= 256) launch_bf16<64, 64, 4, 2, E>(b, G, nsplit, tA, tB, s);
      else launch_bf16<64, 64, 2, 2, E>(b, G, nsplit, tA, tB, s);
      return;
    }
  }
  if (blocks <= 256) launch_bf16<BM, BN, 4, 1, E>(a, G, nsplit, tA, tB, s);
  else launch_bf16<BM, BN, 2, 1, E>(a, G, nsplit, tA, tB, s);
}

// the 16-bit fast path for one problem: tile shape (bm, bn), element type from dtype (1 bf16, 2 fp16)
template <typename E>
void launch_fast_t(const GemmArgs& a, int bm, int bn, int G, int nsplit, int tA, int tB, hipStream_t s) {
  if (bm == 64 && bn == 64) launch_bf16_ns<64, 64, E>(a, G, nsplit, tA, tB, s);
  else if (bm == 64) launch_bf16_ns<64, 128, E>(a, G, nsplit, tA, tB, s);
  else if (bn == 64) launch_bf16_ns<128, 64, E>(a, G, nsplit, tA, tB, s);
  else launch_bf16_ns<128, 128, E>(a, G, nsplit, tA, tB, s);
}
inline void launch_fast(const GemmArgs& a, int bm, int bn, int G, int nsplit, int tA, int tB, int dtype, hipStream_t s) {
  if (dtype == 2) launch_fast_t<f16>(a, bm, bn, G, nsplit, tA, tB, s);
  else launch_fast_t<bf16>(a, bm, bn, G, nsplit, tA, tB, s);
}

// one block per CU (queried once)
inline int cu_count() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess)
      c = 0;
    return c > 0 ? c : 256;
  }();
  return n;
}

template <typename E>
void launch_stream(const GemmArgs& a, int G, int tB, hipStream_t s) {
  const long total = (long)a.tiles_m * a.tiles_n * G;
  static int& bpc = cmx_knob("GEMM_STREAM_BPC", CMX_STREAM_LB);   // resident blocks per CU (VGPR-bound)
  long grid = (long)(bpc > 0 && bpc <= CMX_STREAM_LB ? bpc : CMX_STREAM_LB) * cu_count();
  if (grid > total) grid = total;
  grid = (grid + 7) / 8 * 8;
  if (a.tail == 2) {
    hipLaunchKernelGGL((gemm_stream_kernel<false, E, 2>), dim3((unsigned)grid), dim3(256), 0, s, a);
  } else if (tB) {
    hipLaunchKernelGGL((gemm_stream_kernel<true, E, 0>), dim3((unsigned)grid), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((gemm_stream_kernel<false, E, 0>), dim3((unsigned)grid), dim3(256), 0, s, a);
  }
}

template <typename T, int BM, int BN, bool EXT>
void launch_generic_x(const GemmArgs& a, int G, int nsplit, int tA, int tB, hipStream_t s) {
  dim3 grid(a.tiles_m * a.tiles_n, G, nsplit);
#define CMX_GEMM_LAUNCH(TA, TB) hipLaunchKernelGGL((gemm_generic_kernel<T, BM, BN, TA, TB, EXT>), grid, dim3(256), 0, s, a)
  if (!tA && !tB) CMX_GEMM_LAUNCH(false, false);
  else if (!tA && tB) CMX_GEMM_LAUNCH(false, true);
  else if (tA && tB) CMX_GEMM_LAUNCH(true, true);
  else CMX_GEMM_LAUNCH(true, false);
#undef CMX_GEMM_LAUNCH
}

template <typename T, int BM, int BN>
void launch_generic(const GemmArgs& a, int G, int nsplit, int tA, int tB, hipStream_t s) {
  if (a.nup || a.scatter) launch_generic_x<T, BM, BN, true>(a, G, nsplit, tA, tB, s);
  else launch_generic_x<T, BM, BN, false>(a, G, nsplit, tA, tB, s);
}

// the bf16 fast path needs every operand row to be whole 16-B chunks on 16-B boundaries
// and every per-group operand to be addressable with 31-bit byte offsets
inline bool fast_ok(const void* A, const void* A2, const void* B, int M, int N, int K, int K1, long lda, long lda2, long ldb,
             long sA, long sA2, long sB, int tA, int tB, int ones_col) {
  const int nb = ones_col ? N - 1 : N;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al(A) || !al(B) || (A2 && !al(A2))) return false;
  // a k-contiguous operand is staged in 8-element k chunks (K % 8 keeps the last chunk inside
  // the row); with both operands row-contiguous k is the row index and any K works
  // (FFM k^T v / u^T dout over 300-token stage-4 images)
  if (lda % 8 || ldb % 8 || sA % 8 || sB % 8 || (K % 8 && !(tA && tB))) return false;
  if (tA ? M % 8 : false) return false;
  if (tB ? nb % 8 : false) return false;
  if (A2 && (K1 % FBK || lda2 % 8 || sA2 % 8 || tA)) return false;
  const long extA = tA ? (long)K * lda : (long)M * lda;
  const long extB = tB ? (long)K * ldb : (long)nb * ldb;
  const long extA2 = A2 ? (long)M * lda2 : 0;
  const long lim = (1L << 30) - 64;             // elements (bf16) -> < 2^31 bytes
  return extA < lim && extB < lim && extA2 < lim;
}

inline int tile_dim(int n) { return n <= 64 ? 64 : 128; }

// Tile policy of the bf16 path (CMX_GEMM_TILES=0 restores the 128-wide-first policy, for A/B
// measurements).  Policy 1: when 128-wide tiles leave the chip under-filled (< 400 tiles),
// take 64 x 64 tiles -- 4x the tiles, a lighter per-block k-loop and no split-K combine --
// and split K only when even those leave it under-filled.
inline int tile_policy() {
  static int& p = cmx_knob("GEMM_TILES", 1);
  return p;
}

// Small-K policy (CMX_GEMM_SMALLK=k, default 256): problems with K <= k take 64 x 64 tiles
// whatever their tile count -- a block of one to four k-tiles is a latency chain (DMA, MFMA,
// epilogue), and the 128 x 128 tile's 67 KB epilogue image allows only two such chains per CU
// where 64 x 64 blocks (32 KB) run four or more.  Measured on the B2 step's GEMM census
// (profiles/r02_r_gemm_census.txt): the stage-1/2 MLP and decoder-input GEMMs
// (M 38400 / 9600, K 64-256) gain 10-25 % each, 2558 -> 2485 us per step at k = 640; the one
// 512 x 512 decoder GEMM (K 512) is the shape that keeps 128-wide tiles faster, hence 256.
// A narrow output (N <= 64, K 512: the decoder's class / c1 products) also takes 64 x 64.
inline int smallk_policy() {
  static int& p = cmx_knob("GEMM_SMALLK", 256);
  return p;
}

inline void plan_tiles(int G, int M, int nb, int K, int* bm, int* bn) {
  *bm = tile_dim(M);
  *bn = tile_dim(nb);
  if (tile_policy() == 1) {
    // (CMX_GEMM_T128, default 400: the stage-3 MLP GEMMs, 380 128-wide tiles, run 64 x 64;
    // measured +0.6 % per step over 240 in interleaved A/B)
    static int& t128min = cmx_knob("GEMM_T128", 400);
    const long t128 = (long)cdiv(M, *bm) * cdiv(nb, *bn) * G;
    if (t128 < t128min) *bm = *bn = 64;
  }
  if (K <= smallk_policy() || (nb <= 64 && smallk_policy() > 0)) *bm = *bn = 64;
}

// split factor for the bf16 path: one block per CU when the output has few tiles (each split
// keeps >= 4 k-tiles of 64; the slabs cost 8 B of HBM traffic per output element and split)
inline int auto_split(int G, int M, int N, int K, int ones_col) {
  const int nb = ones_col ? N - 1 : N;
  int bm, bn;
  plan_tiles(G, M, nb, K, &bm, &bn);
  const long tiles = (long)cdiv(M, bm) * cdiv(nb, bn) * G;
  const int nk = (K + FBK - 1) / FBK;
  const long full = tile_policy() == 1 ? 128 : 200;
  if (tiles >= full || nk < 8) return 1;
  // an under-filled 64 x 64 problem without a bias-gradient column runs as k-group blocks
  // (launch_bf16_ns, KW waves per tile) instead of split-K slabs + a reducer launch: measured
  // +1.2 % per step (interleaved A/B, 246.7 / 247.1 -> 249.5 / 250.5 img/s; CMX_GEMM_SPLITKW=0
  // restores split-K)
  static int& splitkw = cmx_knob("GEMM_SPLITKW", 1);
  // (short k-loops only: a k-group block walks nk / 2 ring slots serially, and the FFM context
  // products -- 64 x 64 over 19200 tokens, nk = 300 -- keep split-K: 10.8 vs 33 us)
  if (splitkw && bm == 64 && bn == 64 && !ones_col && nk <= 32) return 1;
  long s = (256 + tiles - 1) / tiles;
  s = s < nk / 4 ? s : nk / 4;
  if (s > 128) s = 128;
  if (s < 1) s = 1;
  const int per = (nk + (int)s - 1) / (int)s;
  return (nk + per - 1) / per;
}

}  // namespace gemmk

#define CMX_GEMM_GENERIC_SHAPES(X, T) X(T, 64, 64) X(T, 64, 128) X(T, 128, 64) X(T, 128, 128)
#define CMX_GEMM_GENERIC_INST(T, BM, BN) \
  template void gemmk::launch_generic<T, BM, BN>(const GemmArgs&, int, int, int, int, hipStream_t);
#define CMX_GEMM_GENERIC_EXTERN(T, BM, BN) \
  extern template void gemmk::launch_generic<T, BM, BN>(const GemmArgs&, int, int, int, int, hipStream_t);
#define CMX_GEMM_FAST_INST(E)                                                                         \
  template void gemmk::launch_fast_t<E>(const GemmArgs&, int, int, int, int, int, int, hipStream_t);
#define CMX_GEMM_FAST_EXTERN(E)                                                                              \
  extern template void gemmk::launch_fast_t<E>(const GemmArgs&, int, int, int, int, int, int, hipStream_t);

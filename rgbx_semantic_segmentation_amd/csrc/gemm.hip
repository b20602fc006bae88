// Batched MFMA GEMM with fused epilogues for every dense layer of the step.
//
//   C[g](i, j) = epi( sum_k A[g](i, k) * B[g](j, k) )          g < G, i < M, j < N, k < K
//
// A(i, k) is read from A[i*lda + k] (transA = 0, k contiguous) or A[k*lda + i] (transA = 1,
// i contiguous); likewise B.  The three GEMMs of a Linear / 1x1 conv / im2col conv are
//   forward   y  = x W^T   : A = x (M x K),  B = W (N x K)           transA = 0, transB = 0
//   dgrad     dx = dy W    : A = dy (M x N), B(j=k', k=n) = W[n][k']  transA = 0, transB = 1
//   wgrad     dW = dy^T x  : A(i=n, k=m) = dy[m][n], B(j=k', k=m) = x[m][k']   both 1
// (reference layers: dual_segformer.py Linear/Conv2d, net_utils.py 1x1 convs, MLPDecoder.py).
//
// Extras that remove whole passes / launches from the step:
//  * two-segment A along k (k < K1 from A, k >= K1 from A2): Linear on cat(x1, x2) without
//    the cat (CrossPath.end_proj, ChannelEmbed, net_utils.py:277-280, 323-326);
//  * `ones_col`: column N - 1 of the result is sum_k A(i, k) (the bias gradient of a wgrad,
//    sum over tokens of dy), routed to `dbias` -- no colsum launch;
//  * split-K over blockIdx.z into fp32 partial slabs + a reducer that applies the full
//    epilogue: the wgrads reduce over up to 76800 tokens into a 64 x 256 result, and the
//    stage-4 layers (600 tokens) have only ~20 output tiles; both need K parallelism.
//
// Epilogue (per output element, fp32):  v = acc + bias[j];  v = act(v);
//   out_mode 0: C = T(v)            out_mode 1: C = fp32(v)        out_mode 2: C += v (fp32)
//   residual R (same layout as C):  C = R + s[(g*M + i) / rows_per_sample] * v  (DropPath-scaled
//   residual, s may be NULL = 1) -- the Block's `x + drop_path(f(x))` (dual_segformer.py:168-169).
//
// Two kernels:
//  * gemm_bf16_kernel -- the bf16 path of the step.  256 threads = 4 waves (2 x 2) over a
//    BM x BN tile (64 or 128 each), v_mfma_f32_32x32x16_bf16, BK = 64.  Operand tiles move
//    HBM -> LDS by buffer_load_dwordx4 ... lds (LDS-DMA, no register staging), double
//    buffered: tile t+1 is in flight while tile t is multiplied.  Out-of-range rows / k come
//    back as zeros from the buffer descriptor's range check (offset 0x80000000), so ragged
//    edges need no branches.  A k-contiguous operand is imaged [rows][64] (128-B rows) and
//    read with ds_read_b128; a row-contiguous (transposed) operand is imaged [64][rows] and
//    read with gfx950's ds_read_b64_tr_b16, which transposes 4 x 16 blocks on the way to the
//    registers -- no transposing LDS writes.  Both images are XOR-swizzled on 16-B chunks so
//    every fragment read is bank-conflict-free; the LDS-DMA writes linearly, so the inverse
//    swizzle is applied to the per-lane global source address.
//  * gemm_generic_kernel -- fp32 parity mode (exact v_mfma_f32_32x32x2_f32) and any bf16
//    problem whose strides / dims do not allow 16-B chunks; register staged, BK = 32.
#include "gemm_kernels.h"
#include <string.h>
#include <stdlib.h>

using namespace gemmk;
CMX_GEMM_FAST_EXTERN(bf16)
CMX_GEMM_FAST_EXTERN(f16)
CMX_GEMM_GENERIC_SHAPES(CMX_GEMM_GENERIC_EXTERN, float)
CMX_GEMM_GENERIC_SHAPES(CMX_GEMM_GENERIC_EXTERN, bf16)
CMX_GEMM_GENERIC_SHAPES(CMX_GEMM_GENERIC_EXTERN, f16)

namespace {
// ============================================================================ grouped reduce
// out (+)= sum over nblk partial rows, for many reductions in one launch: the split-K slabs of
// the grouped weight gradients, the per-block dgamma / dbeta partials of LayerNorm backward and
// the dW / db partials of the depthwise conv backward.  Element w < rows * cols of group g is
// sum_b src[g*sg + b*sb + w]; it lands at dst[g*dg + r*ldd + c] (c < csplit) or
// dst2[g*dg2 + r*ldd2 + c - csplit] (r = w / cols, c = w % cols): e.g. LN's [dgamma | dbeta]
// rows, DWConv's [9 taps | bias] rows, a GEMM slab's row pitch vs the gradient view's ldc.
// zl threads share one output along b (long partial columns), meeting in LDS.
struct RedRec {
  const float* src; float* dst; float* dst2;
  long sg, sb, dg, dg2;
  int ldd, ldd2, G, nblk, rows, cols, csplit, accumulate, zl, cpg, blk0, pad;
};

__global__ __launch_bounds__(256) void reduce_grouped_kernel(const RedRec* __restrict__ recs, int nrec) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  int lo = 0, hi = nrec - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (recs[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const RedRec& r = recs[lo];
  const int zl = r.zl, opb = 256 / zl;
  const int local = b - r.blk0;
  const int g = local / r.cpg, ch = local % r.cpg;
  const int o = threadIdx.x % opb, sl = threadIdx.x / opb;
  const long W = (long)r.rows * r.cols;
  const long w = (long)ch * opb + o;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (w < W) {
    const float* p = r.src + (long)g * r.sg + w;
    const long sb = r.sb;
    int k = sl;
    for (; k + 3 * zl < r.nblk; k += 4 * zl) {
      s0 += p[(long)k * sb];
      s1 += p[(long)(k + zl) * sb];
      s2 += p[(long)(k + 2 * zl) * sb];
      s3 += p[(long)(k + 3 * zl) * sb];
    }
    for (; k < r.nblk; k += zl) s0 += p[(long)k * sb];
  }
  float v = (s0 + s1) + (s2 + s3);
  if (zl > 1) {
    red[threadIdx.x] = v;
    __syncthreads();
    if (sl) return;
    for (int q = 1; q < zl; ++q) v += red[o + q * opb];
  }
  if (w >= W) return;
  const int row = (int)(w / r.cols), c = (int)(w % r.cols);
  float* d = c < r.csplit ? r.dst + (long)g * r.dg + (long)row * r.ldd + c
                          : r.dst2 + (long)g * r.dg2 + (long)row * r.ldd2 + (c - r.csplit);
  *d = r.accumulate ? *d + v : v;
}

}  // namespace

extern "C" {

size_t cmx_gemm_workspace(int G, int M, int N, int splitk) {
  return splitk > 1 ? (size_t)G * splitk * M * N * sizeof(float) : 0;
}

int cmx_gemm_splitk(int G, int M, int N, int K, int ones_col, int dtype) {
  if (G <= 0 || M <= 0 || N <= 0 || K <= 0) return 1;
  if (dtype == 1 || dtype == 2) return auto_split(G, M, N, K, ones_col);
  // generic path: BK = 32, aim for ~1024 blocks with >= 8 k-tiles per split
  const int nb = ones_col ? N : N;
  const long tiles = (long)cdiv(M, M <= 64 ? 64 : 128) * cdiv(nb, nb <= 64 ? 64 : 128) * G;
  const int nk = (K + BK - 1) / BK;
  long s = 1024 / (tiles > 0 ? tiles : 1);
  if (s > nk / 8) s = nk / 8;
  if (s > 64) s = 64;
  return s < 1 ? 1 : (int)s;
}

}  // extern "C"

namespace {
// a planned problem for cmx_gemm_multi (host memory of cmx_gemm_plan_size() bytes)
struct GemmPlan {
  GemmArgs a;
  int tA, tB, dtype, nblk, nk64, pad;
};

// LayerNorm of the output rows in the epilogue (cmx_gemm_ln)
struct LnTail {
  const float* gamma; const float* beta; long sg; void* y; float* mean; float* rstd; float eps;
};

// LayerNorm backward of the epilogue (cmx_gemm_ln_bwd)
struct LnBwd {
  const void* x; const float* gamma; long sg; const float* mean; const float* rstd; const void* dy2; void* dxs;
  float* part;
};

// upsample-add sources of the epilogue (nup = 0: none)
struct UpSpec {
  const void* src[3];
  int h[3], w[3], n, oH, oW;
};

int gemm_impl(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R,
              const float* rscale, float* dbias, float* workspace, int G, int M, int N, int K, int K1, int64_t lda,
              int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias,
              int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode, int ones_col, int splitk,
              int dtype, hipStream_t s, const UpSpec* up, int scR = 0, int scH = 0, int scW = 0, int scC = 0,
              int scHo = 0, int scWo = 0, int gh = 1, int64_t sAh = 0, int64_t sBh = 0, int64_t sCh = 0,
              GemmPlan* plan = nullptr, const void* mask = nullptr, const LnTail* tail = nullptr,
              const LnBwd* lnb = nullptr) {
  CMX_REQUIRE(G > 0 && M > 0 && N > 0 && K > 0, CMX_ERR_SHAPE, "gemm: empty problem G=%d M=%d N=%d K=%d", G, M, N, K);
  CMX_REQUIRE(dtype >= 0 && dtype <= 2, CMX_ERR_DTYPE, "gemm: unsupported dtype %d", dtype);
  CMX_REQUIRE(out_mode >= 0 && out_mode <= 2 && act >= 0 && act <= 3, CMX_ERR_ARG, "gemm: out_mode/act");
  CMX_REQUIRE(!(R && out_mode == 2), CMX_ERR_ARG, "gemm: residual with accumulate");
  if (!A2) K1 = K;
  CMX_REQUIRE(K1 > 0 && K1 <= K && (K1 == K || !transA), CMX_ERR_SHAPE,
              "gemm: a second A segment needs transA = 0 (K1=%d K=%d)", K1, K);
  CMX_REQUIRE(!R || rows_per_sample > 0, CMX_ERR_ARG, "gemm: rows_per_sample");
  CMX_REQUIRE(!ones_col || (transB && dbias && N >= 2 && out_mode != 0 && !bias && !R && act == 0), CMX_ERR_ARG,
              "gemm: ones_col (bias gradient) needs transB, dbias, fp32 output and no epilogue");
  CMX_REQUIRE((long)M * N < (1L << 31) && (long)M * K < (1L << 40), CMX_ERR_SHAPE, "gemm: problem too large");
  const bool fast = dtype != 0 && fast_ok(A, A2, B, M, N, K, K1, lda, lda2, ldb, sA, sA2, sB, transA, transB, ones_col) &&
                    sAh % 8 == 0 && sBh % 8 == 0;
  const int V = dtype == 0 ? 4 : 8;
  const int nb = ones_col ? N - 1 : N;
  const bool vec = (transA ? M : K) % V == 0 && (transB ? nb : K) % V == 0 && (K - K1) % V == 0 && (K1 == K || K1 % V == 0) &&
                   lda % V == 0 && ldb % V == 0 && sA % V == 0 && sB % V == 0 && (!A2 || (lda2 % V == 0 && sA2 % V == 0)) &&
                   ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && (!A2 || (uintptr_t)A2 % 16 == 0);
  CMX_REQUIRE(fast || K1 == K || K1 % BK == 0, CMX_ERR_SHAPE, "gemm: second A segment needs K1 %% %d == 0", BK);
  if (splitk <= 0) splitk = fast ? auto_split(G, M, N, K, ones_col) : cmx_gemm_splitk(G, M, N, K, ones_col, 0);
  CMX_REQUIRE(splitk == 1 || workspace, CMX_ERR_ARG, "gemm: split-K needs a workspace");
  GemmArgs a{};
  a.A = A; a.A2 = A2; a.B = B; a.C = C; a.bias = bias; a.R = R; a.rscale = rscale; a.dbias = dbias; a.ws = workspace;
  a.G = G; a.M = M; a.N = N; a.K = K; a.K1 = K1; a.rows_per_sample = rows_per_sample > 0 ? rows_per_sample : 1;
  a.act = act; a.out_mode = out_mode; a.ones_col = ones_col; a.vec = vec;
  CMX_REQUIRE(!mask || (out_mode == 0 && !ones_col && (uintptr_t)mask % 16 == 0 && (!R || R != mask)), CMX_ERR_ARG,
              "gemm: a ReLU mask needs a plain store in C's layout");
  a.mask = mask;
  // 8-column epilogue groups as aligned vectors: C (and R) rows start on 16-B boundaries
  const long esz = out_mode == 0 ? (dtype != 0 ? 2 : 4) : 4;
  a.cvec = ((uintptr_t)C % 16 == 0) && (ldc * esz) % 16 == 0 && (sC * esz) % 16 == 0 &&
           (!R || (uintptr_t)R % 16 == 0);
  a.lda = lda; a.lda2 = lda2; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sA2 = sA2; a.sB = sB; a.sC = sC;
  a.sbias = sbias; a.sdb = sdb;
  CMX_REQUIRE(gh >= 1 && (gh == 1 || (G % gh == 0 && !A2 && !bias && !R && !ones_col && !(up && up->n) && !scR)),
              CMX_ERR_ARG, "gemm: a two-level batch (gh=%d) takes G %% gh == 0 and no A2 / bias / residual / "
              "bias-gradient / upsample / scatter", gh);
  a.gh = gh; a.sAh = sAh; a.sBh = sBh; a.sCh = sCh;
  if (up && up->n > 0) {
    CMX_REQUIRE(up->n <= 3 && G == 1 && !ones_col && N % 8 == 0 && (long)up->oH * up->oW > 0 &&
                M % (up->oH * up->oW) == 0, CMX_ERR_ARG, "gemm: upsample-add epilogue needs G = 1, N %% 8 == 0 and "
                "M a whole number of %d x %d grids", up->oH, up->oW);
    for (int q = 0; q < up->n; ++q) {
      CMX_REQUIRE(up->src[q] && ((uintptr_t)up->src[q] & 15) == 0 && up->h[q] > 0 && up->w[q] > 0, CMX_ERR_ARG,
                  "gemm: upsample-add source %d", q);
      a.up[q] = up->src[q]; a.uh[q] = up->h[q]; a.uw[q] = up->w[q];
    }
    a.nup = up->n; a.uoH = up->oH; a.uoW = up->oW;
  }
  if (scR > 0) {
    CMX_REQUIRE(G == 1 || sC > 0, CMX_ERR_ARG, "gemm: scatter");
    CMX_REQUIRE((!R || lnb) && out_mode == 0 && !ones_col && N == scR * scR * scC && M % (scHo * scWo) == 0,
                CMX_ERR_ARG, "gemm: patch scatter needs a plain store of N = R*R*C columns");
    a.scatter = 1; a.scH = scH; a.scW = scW; a.scC = scC; a.scR = scR; a.scHo = scHo; a.scWo = scWo;
  }
  const int kstep = fast ? FBK : BK;
  const int nk = (K + kstep - 1) / kstep;
  a.kt_per_split = (nk + splitk - 1) / splitk;
  splitk = (nk + a.kt_per_split - 1) / a.kt_per_split;      // no empty splits
  a.nsplit = splitk;
  // LayerNorm of C's rows in the same launch (tail = 2): N <= 128, one 64 x 64 / 64 x 128 tile
  // spans the row and the lanes that store it normalise it
  const bool row_ln = tail != nullptr;
  if (tail) {
    CMX_REQUIRE(fast && N <= 128 && N % 8 == 0 && splitk == 1 && !transA && !transB && out_mode == 0 && !ones_col &&
                    !a.nup && !a.scatter && gh == 1 && !mask && a.cvec && dtype != 0,
                CMX_ERR_ARG, "gemm_ln: the LayerNorm epilogue needs the 16-bit path without split-K, forward layouts, a "
                "plain aligned store and N <= 128, N %% 8 == 0 (G=%d M=%d N=%d K=%d)", G, M, N, K);
    CMX_REQUIRE(tail->gamma && tail->beta && tail->y && tail->mean && tail->rstd && ((uintptr_t)tail->y & 15) == 0 &&
                    tail->y != C, CMX_ERR_ARG, "gemm_ln: LayerNorm buffers");
    a.tail = 2; a.ln_gamma = tail->gamma; a.ln_beta = tail->beta; a.ln_sg = tail->sg; a.ln_y = tail->y;
    a.ln_mean = tail->mean; a.ln_rstd = tail->rstd; a.ln_eps = tail->eps;
  }
  if (lnb) {
    const bool al = ((uintptr_t)C & 15) == 0 && ((uintptr_t)lnb->x & 15) == 0 && ((uintptr_t)R & 15) == 0 &&
                    ((uintptr_t)lnb->dy2 & 15) == 0 && ((uintptr_t)lnb->dxs & 15) == 0;
    // (under the patch scatter a 64 x C tile is one tap of 64 patches: C must be a tile width)
    const bool rows_ok = a.scatter ? (scC == 64 || scC == 128) && scH == scHo * scR && scW == scWo * scR
                                   : N <= 128 && N % 8 == 0;
    CMX_REQUIRE(fast && splitk == 1 && !transA && transB && out_mode == 0 && !ones_col && !bias && act == 0 && !mask &&
                    !a.nup && gh == 1 && !A2 && a.cvec && al && rows_ok && dtype != 0 &&
                    !tail && lnb->x && lnb->gamma && lnb->mean && lnb->rstd && lnb->part && (!lnb->dxs || rscale),
                CMX_ERR_ARG, "gemm_ln_bwd: needs the 16-bit dgrad path (transB) without split-K, 16-B aligned rows, "
                "N <= 128 (N %% 8 == 0), no bias / activation (G=%d M=%d N=%d K=%d)", G, M, N, K);
    a.tail = 3; a.ln_gamma = lnb->gamma; a.ln_sg = lnb->sg; a.ln_mean = const_cast<float*>(lnb->mean); a.ln_rstd = const_cast<float*>(lnb->rstd);
    a.lnb_x = lnb->x; a.lnb_dy2 = lnb->dy2; a.lnb_dxs = lnb->dxs; a.lnb_part = lnb->part;
  }
  if (plan) {
    // planning only (cmx_gemm_plan): eligible for a multi launch = the 16-bit path on 64 x 64
    // tiles, no split-K, no bias-gradient column / upsample / scatter / two-level batch
    if (!fast || splitk != 1 || ones_col || a.nup || a.scatter || gh != 1 || transA) return 0;
    int bm, bn;
    plan_tiles(G, M, nb, K, &bm, &bn);
    if (bm != 64 || bn != 64) return 0;
    a.tiles_m = cdiv(M, 64); a.tiles_n = cdiv(nb, 64);
    memset(plan, 0, sizeof(*plan));
    plan->a = a; plan->tA = transA; plan->tB = transB; plan->dtype = dtype;
    plan->nblk = a.tiles_m * a.tiles_n * G;
    plan->nk64 = (K + FBK - 1) / FBK;
    return plan->nblk;
  }
  if (fast) {
    int bm, bn;
    plan_tiles(G, M, nb, K, &bm, &bn);
    if (row_ln || lnb) bm = 64, bn = N <= 64 ? 64 : 128;   // one tile spans the row
    if (lnb && a.scatter) bn = scC;                         // (one tap's C channels)
    // 64 x 64 tiles that overflow one round of resident blocks by less than CMX_GEMM_MID percent
    // (5 per CU) take 64 x 128 tiles instead: one round of blocks twice as long, not a second
    // partial round (0 = off; default 50: GEMM census 1380 -> 1361 us, stage-3 fc1 14.3 -> 13.0 us)
    static int& mid = cmx_knob("GEMM_MID", 50);
    if (mid > 0 && bm == 64 && bn == 64 && !row_ln && !lnb && !a.scatter && !a.nup && splitk == 1 && nb >= 128) {
      const long t64 = (long)cdiv(M, 64) * cdiv(nb, 64) * G, slots = 5L * cu_count();
      if (t64 > slots && t64 * 100 <= slots * (100 + mid)) bn = 128;
    }
    a.tiles_m = cdiv(M, bm); a.tiles_n = cdiv(nb, bn);
    // tall 64 x 64 problems of at least CMX_GEMM_STREAM tiles (0 = off) and K <= CMX_GEMM_STREAM_K:
    // the resident streaming grid (gemm_stream_kernel) instead of one block per tile
    static int& stream_min = cmx_knob("GEMM_STREAM", 1024);
    static int& stream_k = cmx_knob("GEMM_STREAM_K", 128);
    const long tiles = (long)a.tiles_m * a.tiles_n * G;
    if (stream_min > 0 && tiles >= stream_min && K <= stream_k && bm == 64 && bn == 64 && splitk == 1 && !transA && !A2 &&
        !ones_col && !a.nup && !a.scatter && gh == 1 && !lnb && (!tail || (row_ln && N <= 64))) {
      if (dtype == 2) launch_stream<f16>(a, G, transB, s);
      else launch_stream<bf16>(a, G, transB, s);
    } else {
      launch_fast(a, bm, bn, G, splitk, transA, transB, dtype, s);
    }
  } else {
    // tile shape: the output's narrow side gets 64 (stage-1 C = 64 outputs, 64-row wgrads)
    const bool m64 = M <= 64, n64 = N <= 64;
    a.tiles_m = cdiv(M, m64 ? 64 : 128); a.tiles_n = cdiv(N, n64 ? 64 : 128);
    if (dtype == 1) {
      if (m64 && n64) launch_generic<bf16, 64, 64>(a, G, splitk, transA, transB, s);
      else if (m64) launch_generic<bf16, 64, 128>(a, G, splitk, transA, transB, s);
      else if (n64) launch_generic<bf16, 128, 64>(a, G, splitk, transA, transB, s);
      else launch_generic<bf16, 128, 128>(a, G, splitk, transA, transB, s);
    } else if (dtype == 2) {
      if (m64 && n64) launch_generic<f16, 64, 64>(a, G, splitk, transA, transB, s);
      else if (m64) launch_generic<f16, 64, 128>(a, G, splitk, transA, transB, s);
      else if (n64) launch_generic<f16, 128, 64>(a, G, splitk, transA, transB, s);
      else launch_generic<f16, 128, 128>(a, G, splitk, transA, transB, s);
    } else {
      if (m64 && n64) launch_generic<float, 64, 64>(a, G, splitk, transA, transB, s);
      else if (m64) launch_generic<float, 64, 128>(a, G, splitk, transA, transB, s);
      else if (n64) launch_generic<float, 128, 64>(a, G, splitk, transA, transB, s);
      else launch_generic<float, 128, 128>(a, G, splitk, transA, transB, s);
    }
  }
  if (splitk > 1) {
    const long work = (long)M * ((nb + 7) / 8) + (ones_col ? M : 0);
    if (dtype == 1) launch_reduce<bf16>(a, G, work, s);
    else if (dtype == 2) launch_reduce<f16>(a, G, work, s);
    else launch_reduce<float>(a, G, work, s);
  }
  return cmx_check_launch("gemm");
}
}  // namespace

extern "C" {

int cmx_gemm(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R,
             const float* rscale, const void* mask, float* dbias, float* workspace, int G, int M, int N, int K, int K1,
             int64_t lda, int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC,
             int64_t sbias, int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode,
             int ones_col, int splitk, int dtype, hipStream_t s) {
  return gemm_impl(A, A2, B, C, bias, R, rscale, dbias, workspace, G, M, N, K, K1, lda, lda2, ldb, ldc, sA, sA2, sB,
                   sC, sbias, sdb, rows_per_sample, transA, transB, act, out_mode, ones_col, splitk, dtype, s, nullptr,
                   0, 0, 0, 0, 0, 0, 1, 0, 0, 0, nullptr, mask);
}

int cmx_gemm_ln(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R,
                const float* rscale, int G, int M, int N, int K, int K1, int64_t lda, int64_t lda2, int64_t ldb,
                int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias, int rows_per_sample,
                int act, const float* ln_gamma, const float* ln_beta, int64_t ln_sg, float ln_eps, void* ln_y,
                float* ln_mean, float* ln_rstd, int dtype, hipStream_t s) {
  const LnTail t{ln_gamma, ln_beta, (long)ln_sg, ln_y, ln_mean, ln_rstd, ln_eps};
  return gemm_impl(A, A2, B, C, bias, R, rscale, nullptr, nullptr, G, M, N, K, K1, lda, lda2, ldb, ldc, sA, sA2, sB,
                   sC, sbias, 0, rows_per_sample, 0, 0, act, 0, 0, 1, dtype, s, nullptr, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0,
                   nullptr, nullptr, &t);
}


int cmx_gemm_ln_bwd(const void* A, const void* B, void* dx, int G, int M, int N, int K, int64_t lda, int64_t ldb,
                    int64_t ldc, int64_t sA, int64_t sB, int64_t sC, const void* x, const float* gamma, int64_t sg,
                    const float* mean, const float* rstd, const void* dres, const void* dy2, const float* sscale,
                    int rows_per_sample, void* dxs, float* partials, int dtype, hipStream_t s) {
  const LnBwd l{x, gamma, (long)sg, mean, rstd, dy2, dxs, partials};
  return gemm_impl(A, nullptr, B, dx, nullptr, dres, sscale, nullptr, nullptr, G, M, N, K, K, lda, 0, ldb, ldc, sA, 0,
                   sB, sC, 0, 0, rows_per_sample, 0, 1, 0, 0, 0, 1, dtype, s, nullptr, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0,
                   nullptr, nullptr, nullptr, &l);
}

size_t cmx_gemm_ln_bwd_partials(int G, int M, int N) { return (size_t)G * ((M + 63) / 64) * 2 * N * sizeof(float); }

// cmx_conv_patch_dgrad with the backward of the LayerNorm that produced the conv's input in the
// epilogue: dx = LN'(col2im(dy W) [+ dy2]) + dres (the norm's input gradient), never storing the conv's
int cmx_conv_patch_dgrad_ln_bwd(const void* dy, const void* Wt, void* dx, int G, int NIg, int H, int Wd, int C, int R,
                                int Ho, int Wo, int N, int64_t sdy, int64_t sW, int64_t sdx, const void* x,
                                const float* gamma, int64_t sg, const float* mean, const float* rstd, const void* dres,
                                const void* dy2, const float* sscale, int rows_per_sample, void* dxs, float* partials,
                                int dtype, hipStream_t s) {
  CMX_REQUIRE(G > 0 && NIg > 0 && (C == 64 || C == 128) && R > 0 && Ho * R == H && Wo * R == Wd, CMX_ERR_SHAPE,
              "conv_patch_dgrad_ln_bwd: H=%d W=%d R=%d Ho=%d Wo=%d C=%d (exact patches, C 64 / 128)", H, Wd, R, Ho, Wo,
              C);
  const int M = NIg * Ho * Wo, Kc = R * R * C;
  const LnBwd l{x, gamma, (long)sg, mean, rstd, dy2, dxs, partials};
  return gemm_impl(dy, nullptr, Wt, dx, nullptr, dres, sscale, nullptr, nullptr, G, M, Kc, N, N, N, 0, Kc, Kc, sdy, 0,
                   sW, sdx, 0, 0, rows_per_sample, 0, 1, 0, 0, 0, 1, dtype, s, nullptr, R, H, Wd, C, Ho, Wo, 1, 0, 0, 0,
                   nullptr, nullptr, nullptr, &l);
}

size_t cmx_conv_patch_dgrad_ln_bwd_partials(int G, int NIg, int Ho, int Wo, int C, int R) {
  return (size_t)G * ((NIg * Ho * Wo + 63) / 64) * R * R * 2 * C * sizeof(float);
}

size_t cmx_gemm_plan_size(void) { return sizeof(GemmPlan); }

// cmx_gemm's arguments, planned instead of launched: > 0 = the problem's block count (eligible
// for cmx_gemm_multi), 0 = not eligible (run it with cmx_gemm), < 0 = invalid arguments
int cmx_gemm_plan(void* plan, const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R,
                  const float* rscale, const void* mask, float* dbias, float* workspace, int G, int M, int N, int K,
                  int K1, int64_t lda,
                  int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC,
                  int64_t sbias, int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode,
                  int ones_col, int splitk, int dtype) {
  CMX_REQUIRE(plan, CMX_ERR_ARG, "gemm_plan: null plan");
  return gemm_impl(A, A2, B, C, bias, R, rscale, dbias, workspace, G, M, N, K, K1, lda, lda2, ldb, ldc, sA, sA2, sB,
                   sC, sbias, sdb, rows_per_sample, transA, transB, act, out_mode, ones_col, splitk, dtype, nullptr,
                   nullptr, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, reinterpret_cast<GemmPlan*>(plan), mask);
}

// n <= 4 planned problems (same dtype and B layout) in ONE launch; waves / ring depth chosen for
// the combined grid as a single problem's launch would be (launch_bf16_ns)
int cmx_gemm_multi(const void* plans, int n, hipStream_t s) {
  CMX_REQUIRE(plans && n >= 1 && n <= MULTI_MAX, CMX_ERR_ARG, "gemm_multi: 1..%d problems (got %d)", MULTI_MAX, n);
  const GemmPlan* pl = reinterpret_cast<const GemmPlan*>(plans);
  GemmMulti m{};
  m.n = n;
  int total = 0, nk64 = 1 << 30;
  for (int i = 0; i < n; ++i) {
    CMX_REQUIRE(pl[i].nblk > 0 && pl[i].tA == 0 && pl[i].tB == pl[0].tB && pl[i].dtype == pl[0].dtype &&
                (pl[i].dtype == 1 || pl[i].dtype == 2), CMX_ERR_ARG, "gemm_multi: plan %d does not match plan 0", i);
    m.a[i] = pl[i].a;
    m.blk0[i] = total;
    total += pl[i].nblk;
    nk64 = nk64 < pl[i].nk64 ? nk64 : pl[i].nk64;
  }
  m.blk0[n] = total;
  for (int i = n + 1; i <= MULTI_MAX; ++i) m.blk0[i] = total;
  static int& kwk = cmx_knob("GEMM_KW", 2);
  const bool kw2 = kwk >= 2 && total <= 512 && nk64 >= 4;
  if (kw2)
    for (int i = 0; i < n; ++i) m.a[i].kt_per_split = (m.a[i].K + 2 * FBK - 1) / (2 * FBK);
  const bool ns4 = total <= 256;
  const bool tB = pl[0].tB != 0, h = pl[0].dtype == 2;
#define CMX_MULTI(NS_, KW_, TB_, E_) \
  hipLaunchKernelGGL((gemm_multi_kernel<NS_, KW_, TB_, E_>), dim3(total), dim3(256 * KW_), 0, s, m)
#define CMX_MULTI_E(NS_, KW_, TB_) \
  do { if (h) CMX_MULTI(NS_, KW_, TB_, f16); else CMX_MULTI(NS_, KW_, TB_, bf16); } while (0)
#define CMX_MULTI_TB(NS_, KW_) do { if (tB) CMX_MULTI_E(NS_, KW_, true); else CMX_MULTI_E(NS_, KW_, false); } while (0)
  if (kw2 && ns4) CMX_MULTI_TB(4, 2);
  else if (kw2) CMX_MULTI_TB(2, 2);
  else if (ns4) CMX_MULTI_TB(4, 1);
  else CMX_MULTI_TB(2, 1);
#undef CMX_MULTI_TB
#undef CMX_MULTI_E
#undef CMX_MULTI
  return cmx_check_launch("gemm_multi");
}

// dx of a non-overlapping patchify conv (stride == kernel == R, pad 0: Attention.sr,
// dual_segformer.py:95-96) in ONE launch: dx[g] = col2im(dy[g] @ W[g]) with the col2im folded
// into the GEMM epilogue as an address remap (every input pixel belongs to at most one patch,
// so there is no overlap to sum).  dy (G, NIg*Ho*Wo, N), W (G, N, R*R*C) tap-major, dx
// (G*NIg, H, W, C) NHWC.  Pixels outside the Ho*R x Wo*R window (H or W not a multiple of R)
// are not written: the caller zeroes dx for such shapes.
// cmx_gemm over a two-level batch: G = Go * gh problems, problem g = (g / gh, g % gh) at operand
// offsets (g / gh) * sX + (g % gh) * sXh (per-head products of the FFM cross attention:
// net_utils.py:206-212, (image x modality, head) pairs with the heads a column slice of a row)
int cmx_gemm_h2(const void* A, const void* B, void* C, float* workspace, int G, int gh, int M, int N, int K,
                int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sAh, int64_t sB, int64_t sBh, int64_t sC,
                int64_t sCh, int transA, int transB, int out_mode, int splitk, int dtype, hipStream_t s) {
  return gemm_impl(A, nullptr, B, C, nullptr, nullptr, nullptr, nullptr, workspace, G, M, N, K, K, lda, 0, ldb, ldc, sA,
                   0, sB, sC, 0, 0, 1, transA, transB, 0, out_mode, 0, splitk, dtype, s, nullptr, 0, 0, 0, 0, 0, 0, gh,
                   sAh, sBh, sCh);
}

int cmx_conv_patch_dgrad(const void* dy, const void* Wt, void* dx, int G, int NIg, int H, int Wd, int C, int R, int Ho,
                         int Wo, int N, int64_t sdy, int64_t sW, int64_t sdx, int dtype, hipStream_t s) {
  CMX_REQUIRE(G > 0 && NIg > 0 && C % 8 == 0 && R > 0 && Ho == H / R && Wo == Wd / R && Ho > 0 && Wo > 0, CMX_ERR_SHAPE,
              "conv_patch_dgrad: H=%d W=%d R=%d Ho=%d Wo=%d C=%d", H, Wd, R, Ho, Wo, C);
  const int M = NIg * Ho * Wo, Kc = R * R * C;
  return gemm_impl(dy, nullptr, Wt, dx, nullptr, nullptr, nullptr, nullptr, nullptr, G, M, Kc, N, N, N, 0, Kc, Kc, sdy,
                   0, sW, sdx, 0, 0, 1, 0, 1, 0, 0, 0, 1, dtype, s, nullptr, R, H, Wd, C, Ho, Wo);
}

// DecoderHead.linear_fuse on the restructured decoder (MLPDecoder.py:66-77):
//   Z = e1 @ Wf[:, 3E:4E]^T + bias + up(z4) + up(z3) + up(z2)
// where z_i = e_i @ Wf[:, slot_i]^T are the low-resolution products of the upsampled branches
// (bilinear interpolation is linear with weights summing to 1, so it commutes with the 1x1
// conv: W up(e) = up(W e)).  e1 (B*H1*W1, K) row stride lda, z_i (B, h_i, w_i, E), Wf_c1 (E, K)
// row stride ldw: the c1 slice of the conv (K = E, DecoderFuseF) or, with linear_c1 folded in,
// the composed M_1 = Wf_c1 Wc_1 (K = C1, e1 = the stage-1 features; decoder_fold.hip).
// Z (B*H1*W1, E).  The (B, N1, 4E) concat of the reference is never formed.
int cmx_decoder_fuse_fwd(const void* e1, const void* Wf_c1, void* Z, const float* bias, const void* z4, const void* z3,
                         const void* z2, int B, int H1, int W1, int h4, int w4, int h3, int w3, int h2, int w2, int E,
                         int K, int64_t lda, int64_t ldw, int dtype, hipStream_t s) {
  CMX_REQUIRE(B > 0 && H1 > 0 && W1 > 0 && E > 0 && E % 8 == 0 && K > 0 && lda >= K && ldw >= K, CMX_ERR_SHAPE,
              "decoder_fuse_fwd: B=%d E=%d K=%d", B, E, K);
  UpSpec up{};
  const void* src[3] = {z4, z3, z2};
  const int hh[3] = {h4, h3, h2}, ww[3] = {w4, w3, w2};
  for (int q = 0; q < 3; ++q) {
    if (!src[q]) continue;
    up.src[up.n] = src[q]; up.h[up.n] = hh[q]; up.w[up.n] = ww[q]; ++up.n;
  }
  up.oH = H1; up.oW = W1;
  const int M = B * H1 * W1;
  return gemm_impl(e1, nullptr, Wf_c1, Z, bias, nullptr, nullptr, nullptr, nullptr, 1, M, E, K, K, lda, 0, ldw, E, 0, 0,
                   0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, dtype, s, &up);
}


// ---------------------------------------------------------------- grouped (deferred) launches
size_t cmx_gemm_group_record_size(void) { return sizeof(GroupRec); }

// split for a problem inside a grouped launch: the launch is filled by many problems, so a
// split only bounds the k-loop of one block (<= 48 k-tiles of 64 = 3072 tokens per block)
int cmx_gemm_grouped_splitk(int G, int M, int N, int K, int ones_col) {
  if (G <= 0 || M <= 0 || N <= 0 || K <= 0) return 1;
  // <= 48 k-tiles of 64 tokens per block (CMX_GROUPED_KT): measured against 16 / 24 / 32 / 64
  // on the B2 step (interleaved A/B: 32 -> 48 is +1.5 %, 64 no better; fewer slabs to reduce)
  static int& kt = cmx_knob("GROUPED_KT", 48);
  const int nk = (K + FBK - 1) / FBK;
  int s = (nk + kt - 1) / kt;
  if (s > 64) s = 64;
  const int per = (nk + s - 1) / s;
  return (nk + per - 1) / per;
}

int cmx_gemm_group_pack(void* rec, const void* A, const void* B, void* C, float* dbias, float* workspace, int G, int M,
                        int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC,
                        int64_t sdb, int transA, int transB, int out_mode, int ones_col, int splitk, int blk0) {
  CMX_REQUIRE(rec && G > 0 && M > 0 && N > 0 && K > 0 && blk0 >= 0, CMX_ERR_SHAPE, "gemm_group_pack: bad problem");
  CMX_REQUIRE(transA && transB, CMX_ERR_ARG, "gemm_group_pack: grouped launches take transA = transB = 1 (weight gradients)");
  CMX_REQUIRE(out_mode == 1 || out_mode == 2, CMX_ERR_ARG, "gemm_group_pack: fp32 output only");
  CMX_REQUIRE(!ones_col || (dbias && N >= 2), CMX_ERR_ARG, "gemm_group_pack: ones_col needs dbias");
  CMX_REQUIRE((long)M * N < (1L << 31), CMX_ERR_SHAPE, "gemm_group_pack: problem too large");
  CMX_REQUIRE(fast_ok(A, nullptr, B, M, N, K, K, lda, 0, ldb, sA, 0, sB, transA, transB, ones_col), CMX_ERR_ARG,
              "gemm_group_pack: operands not eligible for the bf16 LDS-DMA path");
  if (splitk <= 0) splitk = cmx_gemm_grouped_splitk(G, M, N, K, ones_col);
  CMX_REQUIRE(splitk == 1 || workspace, CMX_ERR_ARG, "gemm_group_pack: split-K needs a workspace");
  GroupRec r{};
  GemmArgs& a = r.a;
  a.A = A; a.A2 = nullptr; a.B = B; a.C = C; a.dbias = dbias; a.ws = workspace;
  a.G = G; a.M = M; a.N = N; a.K = K; a.K1 = K; a.rows_per_sample = 1;
  a.act = 0; a.out_mode = out_mode; a.ones_col = ones_col; a.vec = 1;
  a.cvec = ((uintptr_t)C % 16 == 0) && (ldc * 4) % 16 == 0 && (sC * 4) % 16 == 0;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC; a.sdb = sdb;
  const int nk = (K + FBK - 1) / FBK;
  a.kt_per_split = (nk + splitk - 1) / splitk;
  a.nsplit = (nk + a.kt_per_split - 1) / a.kt_per_split;
  const int nb = ones_col ? N - 1 : N;
  r.bm = tile_dim(M); r.bn = tile_dim(nb);
  a.tiles_m = cdiv(M, r.bm); a.tiles_n = cdiv(nb, r.bn);
  r.blk0 = blk0;
  r.nblk = a.tiles_m * a.tiles_n * G * a.nsplit;
  memcpy(rec, &r, sizeof(r));
  return r.nblk;
}

// weight gradient of ONE tap of an NHWC convolution as a grouped-GEMM record:
// dW[g][n][tap*C + c] (row pitch K = KH*KW*C) = sum_m dy[g][m][n] * x[g][pixel(m) at tap][c]
int cmx_gemm_group_pack_conv_wgrad(void* rec, const void* dy, const void* x, float* dW, float* dbias, float* workspace,
                                   int G, int NIg, int H, int Wd, int C, int KH, int KW, int stride, int pad, int Ho,
                                   int Wo, int N, int tap, int64_t sdy, int64_t sx, int64_t sdW, int64_t sdb,
                                   int splitk, int blk0) {
  const int M = NIg * Ho * Wo;                  // reduction length (output pixels)
  CMX_REQUIRE(rec && G > 0 && N > 0 && C % 8 == 0 && N % 8 == 0 && M % 8 == 0 && tap >= 0 && tap < KH * KW,
              CMX_ERR_SHAPE, "gemm_group_pack_conv_wgrad: bad problem");
  CMX_REQUIRE(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && sdy % 8 == 0 && sx % 8 == 0, CMX_ERR_ARG,
              "gemm_group_pack_conv_wgrad: alignment");
  CMX_REQUIRE((long)NIg * H * Wd * C < (1L << 30) && (long)M * N < (1L << 30), CMX_ERR_SHAPE,
              "gemm_group_pack_conv_wgrad: too large for 31-bit offsets");
  const int ones = dbias ? 1 : 0;
  const int Nk = C + ones;                      // output columns (+ bias-gradient column)
  if (splitk <= 0) splitk = cmx_gemm_grouped_splitk(G, N, Nk, M, ones);
  CMX_REQUIRE(splitk == 1 || workspace, CMX_ERR_ARG, "gemm_group_pack_conv_wgrad: split-K needs a workspace");
  GroupRec r{};
  GemmArgs& a = r.a;
  a.A = dy; a.B = x; a.C = dW + (long)tap * C; a.dbias = dbias; a.ws = workspace;
  a.G = G; a.M = N; a.N = Nk; a.K = M; a.K1 = M; a.rows_per_sample = 1;
  a.out_mode = 1; a.ones_col = ones; a.vec = 1;
  a.lda = N; a.sA = sdy; a.ldb = 0; a.sB = sx; a.ldc = (long)KH * KW * C; a.sC = sdW; a.sdb = sdb;
  a.cvec = (((uintptr_t)a.C % 16) == 0) && (a.ldc * 4) % 16 == 0 && (sdW * 4) % 16 == 0;
  a.conv = 2; a.cH = H; a.cW = Wd; a.cC = C; a.cKW = KW; a.cst = stride; a.cpad = pad; a.cHo = Ho; a.cWo = Wo;
  a.ctap = tap;
  const int nk = (M + FBK - 1) / FBK;
  a.kt_per_split = (nk + splitk - 1) / splitk;
  a.nsplit = (nk + a.kt_per_split - 1) / a.kt_per_split;
  r.bm = tile_dim(N); r.bn = tile_dim(C);
  a.tiles_m = cdiv(N, r.bm); a.tiles_n = cdiv(C, r.bn);
  r.blk0 = blk0;
  r.nblk = a.tiles_m * a.tiles_n * G * a.nsplit;
  memcpy(rec, &r, sizeof(r));
  return r.nblk;
}

// y[g] (NIg*Ho*Wo, N) = conv(x[g]) + bias[g] with the im2col done by the GEMM's operand DMA
// (OverlapPatchEmbed.proj k3 s2 p1, dual_segformer.py:196-197; Attention.sr kR sR, :95-96).
// bf16, NHWC x with C % 64 == 0, weights (N, KH, KW, C).
int cmx_conv_implicit_fwd(const void* x, const void* Wt, void* y, const float* bias, float* workspace, int G, int NIg,
                          int H, int Wd, int C, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int64_t sx,
                          int64_t sW, int64_t sy, int64_t sbias, int splitk, int dtype, hipStream_t s) {
  CMX_REQUIRE((dtype == 1 || dtype == 2) && C % 64 == 0 && N % 8 == 0 && G > 0 && NIg > 0, CMX_ERR_SHAPE,
              "conv_implicit_fwd: bf16 / fp16 with C %% 64 == 0 only (C=%d, N=%d)", C, N);
  CMX_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)Wt & 15) == 0 && ((uintptr_t)y & 15) == 0 && sx % 8 == 0 &&
              sW % 8 == 0 && sy % 8 == 0, CMX_ERR_ARG, "conv_implicit_fwd: alignment");
  const long M = (long)NIg * Ho * Wo, K = (long)KH * KW * C;
  CMX_REQUIRE((long)NIg * H * Wd * C < (1L << 30) && M * N < (1L << 31) && (long)N * K < (1L << 30), CMX_ERR_SHAPE,
              "conv_implicit_fwd: too large for 31-bit offsets");
  GemmArgs a{};
  a.A = x; a.B = Wt; a.C = y; a.bias = bias;
  a.G = G; a.M = (int)M; a.N = N; a.K = (int)K; a.K1 = (int)K; a.rows_per_sample = 1; a.vec = 1;
  a.lda = 0; a.sA = sx; a.ldb = K; a.sB = sW; a.ldc = N; a.sC = sy; a.sbias = sbias;
  a.cvec = (N * 2) % 16 == 0 && (sy * 2) % 16 == 0;
  a.conv = 1; a.cH = H; a.cW = Wd; a.cC = C; a.cKW = KW; a.cst = stride; a.cpad = pad; a.cHo = Ho; a.cWo = Wo;
  // the SR conv has few output pixels and a long K (stage 1: 600 x 64 x 4096): split K like a
  // plain GEMM (splitk <= 0: the library's choice, cmx_gemm_splitk(G, M, N, K, 0, 1))
  if (splitk <= 0) splitk = auto_split(G, (int)M, N, (int)K, 0);
  CMX_REQUIRE(splitk == 1 || workspace, CMX_ERR_ARG, "conv_implicit_fwd: split-K needs a workspace");
  a.ws = workspace;
  const int nk = (int)((K + FBK - 1) / FBK);
  a.kt_per_split = (nk + splitk - 1) / splitk;
  splitk = (nk + a.kt_per_split - 1) / a.kt_per_split;
  a.nsplit = splitk;
  int bm, bn;
  plan_tiles(G, (int)M, N, (int)K, &bm, &bn);
  a.tiles_m = cdiv(M, bm); a.tiles_n = cdiv(N, bn);
  launch_fast(a, bm, bn, G, splitk, 0, 0, dtype, s);
  if (splitk > 1) {
    if (dtype == 2) launch_reduce<f16>(a, G, (long)M * ((N + 7) / 8), s);
    else launch_reduce<bf16>(a, G, (long)M * ((N + 7) / 8), s);
  }
  return cmx_check_launch("conv_implicit_fwd");
}

int cmx_gemm_grouped(const void* recs, int nrec, int total_blocks, int dtype, hipStream_t s) {
  CMX_REQUIRE(dtype == 1 || dtype == 2, CMX_ERR_DTYPE, "gemm_grouped: operands bf16 (1) or fp16 (2), got %d", dtype);
  CMX_REQUIRE(recs && nrec > 0 && total_blocks > 0, CMX_ERR_ARG, "gemm_grouped: empty launch");
  // XCD map of the grouped grid: chunked round-robin with 64-tile runs (CMX_GROUPED_CHUNK=n to
  // change the run, 0 = the contiguous xcd_tile map).  Measured on the B2 step's 8174-block
  // launch: 695-702 us contiguous, 624-633 us for runs of 4..128 tiles
  // (scripts/grouped_chunk_sweep.sh); PMC HBM bytes per launch 3.13 GB at 16-tile runs,
  // 2.48 GB at 64 (contiguous: 2.43 GB), so 64 keeps the L2 reuse of neighbouring tiles
  return cmx_gemm_grouped_capped(recs, nrec, total_blocks, 0, dtype, s);
}

int cmx_gemm_grouped_capped(const void* recs, int nrec, int total_blocks, int max_blocks, int dtype, hipStream_t s) {
  CMX_REQUIRE(dtype == 1 || dtype == 2, CMX_ERR_DTYPE, "gemm_grouped: operands bf16 (1) or fp16 (2), got %d", dtype);
  CMX_REQUIRE(recs && nrec > 0 && total_blocks > 0, CMX_ERR_ARG, "gemm_grouped: empty launch");
  CMX_REQUIRE(max_blocks <= 0 || max_blocks % 8 == 0, CMX_ERR_ARG, "gemm_grouped: max_blocks %d not a multiple of 8",
              max_blocks);
  static int& chunk = cmx_knob("GROUPED_CHUNK", 64);
  const GroupRec* rr = (const GroupRec*)recs;
  const int grid = max_blocks > 0 && max_blocks < total_blocks ? max_blocks : total_blocks;
  if (grid < total_blocks) {
    if (dtype == 2)
      hipLaunchKernelGGL((gemm_grouped_kernel<f16, 2, true>), dim3(grid), dim3(256), 0, s, rr, nrec, chunk, total_blocks);
    else
      hipLaunchKernelGGL((gemm_grouped_kernel<bf16, 2, true>), dim3(grid), dim3(256), 0, s, rr, nrec, chunk, total_blocks);
  } else if (dtype == 2) {
    hipLaunchKernelGGL((gemm_grouped_kernel<f16>), dim3(grid), dim3(256), 0, s, rr, nrec, chunk, total_blocks);
  } else {
    hipLaunchKernelGGL((gemm_grouped_kernel<bf16>), dim3(grid), dim3(256), 0, s, rr, nrec, chunk, total_blocks);
  }
  return cmx_check_launch("gemm_grouped");
}

size_t cmx_reduce_record_size(void) { return sizeof(RedRec); }

int cmx_reduce_pack(void* rec, const float* src, float* dst, float* dst2, int G, int nblk, int64_t sg, int64_t sb,
                    int rows, int cols, int csplit, int64_t dg, int ldd, int64_t dg2, int ldd2, int accumulate,
                    int blk0) {
  CMX_REQUIRE(rec && src && dst && G > 0 && nblk > 0 && rows > 0 && cols > 0 && blk0 >= 0, CMX_ERR_SHAPE,
              "reduce_pack: bad reduction");
  CMX_REQUIRE(csplit >= cols || (dst2 && csplit >= 0), CMX_ERR_ARG, "reduce_pack: columns past csplit need dst2");
  RedRec r{};
  r.src = src; r.dst = dst; r.dst2 = dst2; r.sg = sg; r.sb = sb; r.dg = dg; r.dg2 = dg2;
  r.ldd = ldd; r.ldd2 = ldd2; r.G = G; r.nblk = nblk; r.rows = rows; r.cols = cols; r.csplit = csplit;
  r.accumulate = accumulate;
  r.zl = nblk <= 8 ? 1 : (nblk <= 64 ? 4 : 16);
  r.cpg = (int)cdiv((long)rows * cols, 256 / r.zl);
  r.blk0 = blk0;
  memcpy(rec, &r, sizeof(r));
  return r.cpg * G;
}

int cmx_reduce_grouped(const void* recs, int nrec, int total_blocks, hipStream_t s) {
  CMX_REQUIRE(recs && nrec > 0 && total_blocks > 0, CMX_ERR_ARG, "reduce_grouped: empty launch");
  hipLaunchKernelGGL(reduce_grouped_kernel, dim3(total_blocks), dim3(256), 0, s, (const RedRec*)recs, nrec);
  return cmx_check_launch("reduce_grouped");
}

}  // extern "C"

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
//  * `ones_col`: B gets a virtual column j = N - 1 of ones, so the wgrad's last output
//    column is sum_m dy[m][n] = the bias gradient, routed to `dbias` (no colsum launch);
//  * split-K over blockIdx.z into fp32 partial slabs + a reducer that writes the (possibly
//    strided, possibly accumulating) fp32 output: the wgrad reduces over up to 76800 tokens
//    into a 64 x 256 result, which has no parallelism without it.
//
// Epilogue (per output element, fp32):  v = acc + bias[j];  v = act(v);
//   out_mode 0: C = T(v)            out_mode 1: C = fp32(v)        out_mode 2: C += v (fp32)
//   residual R (same layout as C):  C = R + s[(g*M + i) / rows_per_sample] * v  (DropPath-scaled
//   residual, s may be NULL = 1) -- the Block's `x + drop_path(f(x))` (dual_segformer.py:168-169).
//
// Tiling (gfx950, wave64): 256 threads = 4 waves in a 2 x 2 grid over a BM x BN block tile;
// each wave owns (BM/2) x (BN/2) as 32x32 MFMA tiles (v_mfma_f32_32x32x16_bf16, or the exact
// fp32 v_mfma_f32_32x32x2_f32 in fp32 parity mode).  BK = 32 per stage, two LDS buffers;
// the next stage's global loads are issued into registers before the current stage's
// MFMAs and written to LDS after them (one barrier per stage).  Transposed operands are
// transposed during the LDS write.  Block -> tile mapping is XCD-aware: consecutive block
// ids land on different XCDs, so each XCD's L2 sees consecutive tiles of one A row-panel.
#include "cmx_mfma.h"

namespace {

constexpr int BK = 32;

template <typename T> struct Stage;
template <> struct Stage<bf16> { static constexpr int V = 8, PAD = 8; typedef uint4 raw; };
template <> struct Stage<float> { static constexpr int V = 4, PAD = 4; typedef float4 raw; };

template <typename T>
__device__ __forceinline__ typename Stage<T>::raw ones_first() {   // {1, 0, 0, ...}
  typename Stage<T>::raw v{};
  if constexpr (sizeof(T) == 4) v.x = 1.f;
  else v.x = 0x3f80u;                                              // bf16(1.0) in the low half
  return v;
}

struct GemmArgs {
  const void* A; const void* A2; const void* B; void* C; const float* bias; const void* R; const float* rscale;
  float* dbias; float* ws;
  int M, N, K, K1, kt_per_split, rows_per_sample, act, out_mode, tiles_m, tiles_n, ones_col, nsplit;
  long lda, lda2, ldb, ldc, sA, sA2, sB, sC, sbias, sdb;
};

template <typename T, int ROWS>
struct TileLoader {
  // One operand tile: ROWS (i or j) x BK (k).  Per thread: CH chunks of V contiguous
  // elements along the operand's contiguous dim.
  static constexpr int V = Stage<T>::V;
  static constexpr int CHUNKS = ROWS * BK / V;
  static constexpr int CH = CHUNKS / 256;
  static_assert(CHUNKS % 256 == 0, "tile must split evenly over 256 threads");
  typename Stage<T>::raw r[CH];

  // rows [row0, nrows) valid, k in [k0, k0 + BK) of a segment with kend valid k;
  // ones_row >= 0: that (virtual) row is all ones for valid k
  template <bool TRANS>
  __device__ __forceinline__ void load(const T* __restrict__ P, long ld, int row0, int nrows, int k0, int kend,
                                       int ones_row) {
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
      if (gk < kend) {
        if (gr < nrows) {
          const T* p = !TRANS ? P + (long)gr * ld + gk : P + (long)gk * ld + gr;
          r[c] = *reinterpret_cast<const typename Stage<T>::raw*>(p);
        } else if (TRANS && gr == ones_row) {
          r[c] = ones_first<T>();
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

template <typename T, int BM, int BN, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs p) {
  typedef MF<T> mf;
  constexpr int LD = BK + Stage<T>::PAD;
  constexpr int TM = BM / 64, TN = BN / 64;     // 32x32 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) T As[2][BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LD];

  // XCD-aware tile order: hardware dispatches block b to XCD b % 8; give XCD x the
  // contiguous tile range [x * per, (x + 1) * per) so one XCD walks one A row-panel.
  const int ntiles = p.tiles_m * p.tiles_n;
  int t = blockIdx.x;
  if (ntiles % 8 == 0) t = (t % 8) * (ntiles / 8) + t / 8;
  const int tm = t / p.tiles_n, tn = t % p.tiles_n;
  const int g = blockIdx.y, z = blockIdx.z;
  const T* Ag = reinterpret_cast<const T*>(p.A) + (long)g * p.sA;
  const T* A2g = p.A2 ? reinterpret_cast<const T*>(p.A2) + (long)g * p.sA2 : nullptr;
  const T* Bg = reinterpret_cast<const T*>(p.B) + (long)g * p.sB;
  const int i0 = tm * BM, j0 = tn * BN;
  const int nreal = p.ones_col ? p.N - 1 : p.N;     // real B rows (the ones row is virtual)
  const int ones_row = p.ones_col ? p.N - 1 : -1;

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
    if (k0 < p.K1) la.template load<TA>(Ag, p.lda, i0, p.M, k0, p.K1, -1);
    else la.template load<TA>(A2g, p.lda2, i0, p.M, k0 - p.K1, p.K - p.K1, -1);
    lb.template load<TB>(Bg, p.ldb, j0, nreal, k0, p.K, ones_row);
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
    if (p.nsplit > 1) {        // raw fp32 partial slab (g, z, i, j), N columns incl. ones column
      float* wsz = p.ws + (((long)g * p.nsplit + z) * p.M) * p.N;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = i0 + wm * (BM / 2) + a * 32 + accrow(q, h);
          if (i < p.M) wsz[(long)i * p.N + j] = acc[a][b][q];
        }
      continue;
    }
    if (j == ones_row) {       // bias gradient column
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = i0 + wm * (BM / 2) + a * 32 + accrow(q, h);
          if (i < p.M) {
            float* d = p.dbias + (long)g * p.sdb + i;
            *d = p.out_mode == 2 ? *d + acc[a][b][q] : acc[a][b][q];
          }
        }
      continue;
    }
    const float bj = p.bias ? p.bias[(long)g * p.sbias + j] : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + wm * (BM / 2) + a * 32 + accrow(q, h);
        if (i >= p.M) continue;
        float v = act_fwd(acc[a][b][q] + bj, p.act);
        const long off = (long)g * p.sC + (long)i * p.ldc + j;
        if (p.R) {
          const float sc = p.rscale ? p.rscale[((long)g * p.M + i) / p.rows_per_sample] : 1.f;
          v = to_f32(reinterpret_cast<const T*>(p.R)[off]) + sc * v;
        }
        if (p.out_mode == 0) {
          reinterpret_cast<T*>(p.C)[off] = from_f32<T>(v);
        } else if (p.out_mode == 1) {
          reinterpret_cast<float*>(p.C)[off] = v;
        } else {
          reinterpret_cast<float*>(p.C)[off] += v;
        }
      }
    }
  }
}

// sum the nsplit partial slabs; fp32 output (out_mode 1 store / 2 accumulate), strided C;
// column N-1 goes to dbias when ones_col.  4 columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs p) {
  const int g = blockIdx.y;
  const long MN = (long)p.M * p.N;
  const long e = ((long)blockIdx.x * 256 + threadIdx.x);
  if (e >= MN) return;
  const float* src = p.ws + (long)g * p.nsplit * MN + e;
  float s = 0.f;
  for (int z = 0; z < p.nsplit; ++z) s += src[(long)z * MN];
  const int i = (int)(e / p.N), j = (int)(e % p.N);
  float* d;
  if (p.ones_col && j == p.N - 1) d = p.dbias + (long)g * p.sdb + i;
  else d = reinterpret_cast<float*>(p.C) + (long)g * p.sC + (long)i * p.ldc + j;
  *d = p.out_mode == 2 ? *d + s : s;
}

template <typename T, int BM, int BN>
void launch(const GemmArgs& a, int G, int nsplit, int transA, int transB, hipStream_t s) {
  dim3 grid(a.tiles_m * a.tiles_n, G, nsplit);
#define CMX_GEMM_LAUNCH(TA, TB) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, TA, TB>), grid, dim3(256), 0, s, a)
  if (!transA && !transB) CMX_GEMM_LAUNCH(false, false);
  else if (!transA && transB) CMX_GEMM_LAUNCH(false, true);
  else if (transA && transB) CMX_GEMM_LAUNCH(true, true);
  else CMX_GEMM_LAUNCH(true, false);
#undef CMX_GEMM_LAUNCH
}

template <typename T>
void dispatch_tile(GemmArgs& a, int G, int nsplit, int transA, int transB, hipStream_t s) {
  // tile shape: the output's narrow side gets 64 (stage-1 C = 64 outputs, 64-row wgrads)
  const bool m64 = a.M <= 64, n64 = a.N <= 64;
  if (m64 && n64) {
    a.tiles_m = (a.M + 63) / 64; a.tiles_n = (a.N + 63) / 64;
    launch<T, 64, 64>(a, G, nsplit, transA, transB, s);
  } else if (m64) {
    a.tiles_m = (a.M + 63) / 64; a.tiles_n = (a.N + 127) / 128;
    launch<T, 64, 128>(a, G, nsplit, transA, transB, s);
  } else if (n64) {
    a.tiles_m = (a.M + 127) / 128; a.tiles_n = (a.N + 63) / 64;
    launch<T, 128, 64>(a, G, nsplit, transA, transB, s);
  } else {
    a.tiles_m = (a.M + 127) / 128; a.tiles_n = (a.N + 127) / 128;
    launch<T, 128, 128>(a, G, nsplit, transA, transB, s);
  }
}

}  // namespace

extern "C" {

size_t cmx_gemm_workspace(int G, int M, int N, int splitk) {
  return splitk > 1 ? (size_t)G * splitk * M * N * sizeof(float) : 0;
}

int cmx_gemm(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R,
             const float* rscale, float* dbias, float* workspace, int G, int M, int N, int K, int K1, int64_t lda,
             int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias,
             int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode, int ones_col, int splitk,
             int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(G > 0 && M > 0 && N > 0 && K > 0, CMX_ERR_SHAPE, "gemm: empty problem G=%d M=%d N=%d K=%d", G, M, N, K);
  CMX_REQUIRE(out_mode >= 0 && out_mode <= 2 && act >= 0 && act <= 3, CMX_ERR_ARG, "gemm: out_mode/act");
  CMX_REQUIRE(!(R && out_mode == 2), CMX_ERR_ARG, "gemm: residual with accumulate");
  if (!A2) K1 = K;
  CMX_REQUIRE(K1 > 0 && K1 <= K && (K1 == K || (K1 % BK == 0 && !transA)), CMX_ERR_SHAPE,
              "gemm: second A segment needs K1 %% %d == 0 and transA = 0 (K1=%d K=%d)", BK, K1, K);
  // vector staging: the contiguous dim of each operand moves in chunks of V elements
  const int nb = ones_col ? N - 1 : N;
  CMX_REQUIRE((transA ? M : K) % V == 0 && (transB ? nb : K) % V == 0 && (K - K1) % V == 0, CMX_ERR_SHAPE,
              "gemm: contiguous operand dims must be multiples of %d (M=%d N=%d K=%d tA=%d tB=%d)", V, M, N, K,
              transA, transB);
  CMX_REQUIRE(lda % V == 0 && ldb % V == 0 && sA % V == 0 && sB % V == 0 && (!A2 || (lda2 % V == 0 && sA2 % V == 0)),
              CMX_ERR_SHAPE, "gemm: operand strides must be multiples of %d", V);
  CMX_REQUIRE(!R || rows_per_sample > 0, CMX_ERR_ARG, "gemm: rows_per_sample");
  CMX_REQUIRE(!ones_col || (transB && dbias && N >= 2 && out_mode != 0 && !bias && !R && act == 0), CMX_ERR_ARG,
              "gemm: ones_col (bias gradient) needs transB, dbias, fp32 output and no epilogue");
  CMX_REQUIRE(splitk >= 1 && (splitk == 1 || (workspace && out_mode != 0 && !bias && !R && act == 0)), CMX_ERR_ARG,
              "gemm: split-K needs a workspace, fp32 output and no epilogue");
  CMX_REQUIRE((long)M * N < (1L << 31) && (long)M * K < (1L << 40), CMX_ERR_SHAPE, "gemm: problem too large");
  GemmArgs a{};
  a.A = A; a.A2 = A2; a.B = B; a.C = C; a.bias = bias; a.R = R; a.rscale = rscale; a.dbias = dbias; a.ws = workspace;
  a.M = M; a.N = N; a.K = K; a.K1 = K1; a.rows_per_sample = rows_per_sample > 0 ? rows_per_sample : 1;
  a.act = act; a.out_mode = out_mode; a.ones_col = ones_col; a.nsplit = splitk;
  a.lda = lda; a.lda2 = lda2; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sA2 = sA2; a.sB = sB; a.sC = sC;
  a.sbias = sbias; a.sdb = sdb;
  const int nk = (K + BK - 1) / BK;
  a.kt_per_split = (nk + splitk - 1) / splitk;
  if (dtype == 1) dispatch_tile<bf16>(a, G, splitk, transA, transB, s);
  else if (dtype == 0) dispatch_tile<float>(a, G, splitk, transA, transB, s);
  else { cmx_set_error("gemm: unsupported dtype %d", dtype); return CMX_ERR_DTYPE; }
  if (splitk > 1) {
    const long MN = (long)M * N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(cdiv(MN, 256), G), dim3(256), 0, s, a);
  }
  return cmx_check_launch("gemm");
}

}  // extern "C"

// Stage-1 OverlapPatchEmbed conv (Conv2d 3 -> N, k7 s4 p3, dual_segformer.py:196-197,219) on the
// fp32 NCHW input images, WITHOUT materialising im2col columns.
//
// Tile = 64 consecutive output pixels of one output row (oy, ox0 .. ox0 + 63).  Its input
// footprint (3 channels x 7 rows x 259 columns, fp32, zeros outside the image) is staged in
// LDS with coalesced row loads; the tile's 64 x 147 patch matrix (columns in the reference's
// (c, kh, kw) weight-flatten order, zero-padded to 192) is gathered LDS -> LDS as a bf16 / f16
// MFMA operand image, and multiplied by v_mfma_f32_32x32x16 against the weight image.
//   forward  y[g] (pixels x N)  = patches x W[g]^T + b[g]       (W (N, Kp): the ParamStore's
//            16-bit shadow, Kp = 152 = 147 padded to 16-B rows; k >= Kp reads as zero)
//   wgrad    dW[g] (N x Kp), db[g] = sum over pixels of dy^T [patches | 1]: one fp32 partial
//            slab (N, Kp + 1) per workgroup (several tiles each), summed by the caller's
//            reduction (the deferred grouped reduce).  The input images need no gradient.
// Both modality streams in one launch: g = 0 reads img0 (RGB), g = 1 img1 (the X modality).
#include "gemm_kernels.h"

using namespace gemmk;

namespace {

constexpr int PE_C = 3, PE_K = 7, PE_S = 4, PE_P = 3;
constexpr int PE_KR = PE_C * PE_K * PE_K;      // 147 real columns
constexpr int TW = 64;                          // output pixels per tile
constexpr int PW = (TW - 1) * PE_S + PE_K;      // 259 input columns per tile row
constexpr int PWP = 260;                        // LDS pitch of a patch row (floats)
constexpr int IMG = 64 * 64 * 2;                // one 64 x 64 16-bit operand image (8 KB)
constexpr int PROWS = PE_C * PE_K + 1;          // 21 footprint rows + one zero row (columns k >= 147)
constexpr int KPAD = 192;                       // patch-matrix columns of the three 64-wide k images
constexpr int PATCH_BYTES = PROWS * PWP * 4 + KPAD * 4;   // footprint (22.9 KB) + column offset table

// the tile's input footprint: rows iy0 .. iy0 + 6, columns ix0 .. ix0 + 258 of the 3 planes,
// PL values per thread (consecutive threads -> consecutive columns: coalesced).  Every load is
// issued (an out-of-image element reads the plane's first value and is zeroed on the way in),
// so all PL are in flight together and a thread has exactly PL loads outstanding -- the weight
// gradient prefetches the next tile's footprint during this tile's MFMAs and waits on
// vmcnt(PL) for its own DMA (a serial load-then-store loop had one load in flight per thread:
// ~40 us per tile of latency).
constexpr int PATCH_N = PE_C * PE_K * PW;       // 5439
constexpr int PL = (PATCH_N + 255) / 256;       // 22 values per thread
struct PatchRegs {
  float v[PL];
};

__device__ __forceinline__ void load_patch(const float* __restrict__ img, PatchRegs& r, int H, int W, int iy0,
                                           int ix0) {
#pragma unroll
  for (int u = 0; u < PL; ++u) {
    const int e = threadIdx.x + u * 256;
    const int cr = e / PW, col = e - cr * PW;   // cr = c * 7 + r
    const int c = cr / PE_K, kr = cr - c * PE_K;
    const int iy = iy0 + kr, ix = ix0 + col;
    const bool in = e < PATCH_N && iy >= 0 && iy < H && ix >= 0 && ix < W;
    const long off = in ? ((long)c * H + iy) * W + ix : 0;
    const float v = img[off];
    r.v[u] = in ? v : 0.f;
  }
}

__device__ __forceinline__ void store_patch(float* patch, const PatchRegs& r) {
#pragma unroll
  for (int u = 0; u < PL; ++u) {
    const int e = threadIdx.x + u * 256;
    if (e < PATCH_N) {
      const int cr = e / PW, col = e - cr * PW;
      patch[cr * PWP + col] = r.v[u];
    }
  }
}

// once per workgroup: the zero row, and koff[k] = LDS offset of patch-matrix column k at pixel 0
// (column k = (c, kh, kw) reads footprint row c*7 + kh at column 4 px + kw; k >= 147 reads the
// zero row), so a chunk of 8 columns is two table reads and 8 adds -- no index arithmetic.
// Pixels past the tile's last output column need no masking: their dy rows are zero (weight
// gradient) or their outputs are not stored (forward), and the footprint there is finite data.
__device__ __forceinline__ void init_patch_consts(float* patch, int* koff) {
  for (int i = threadIdx.x; i < PWP; i += 256) patch[(PROWS - 1) * PWP + i] = 0.f;
  for (int k = threadIdx.x; k < KPAD; k += 256) {
    int o = (PROWS - 1) * PWP;
    if (k < PE_KR) {
      const int c = k / (PE_K * PE_K), rr = k - c * (PE_K * PE_K), kh = rr / PE_K, kw = rr - kh * PE_K;
      o = (c * PE_K + kh) * PWP + kw;
    }
    koff[k] = o;
  }
}

// 8 patch-matrix entries (pixel px, columns k0 .. k0 + 7) as packed 16-bit values
template <typename E>
__device__ __forceinline__ uint4 patch_chunk(const float* patch, const int* koff, int px, int k0) {
  const int4 o0 = *reinterpret_cast<const int4*>(koff + k0);
  const int4 o1 = *reinterpret_cast<const int4*>(koff + k0 + 4);
  const float* pp = patch + px * PE_S;
  return make_uint4(pack2<E>(pp[o0.x], pp[o0.y]), pack2<E>(pp[o0.z], pp[o0.w]), pack2<E>(pp[o1.x], pp[o1.y]),
                    pack2<E>(pp[o1.z], pp[o1.w]));
}

// forward operand: three k-contiguous images [64 px][64 k] (gemm_kernels.h stage_k layout:
// chunk c of row r at position c ^ ((r >> 1) & 7)), read with frag_k
template <typename E>
__device__ __forceinline__ void build_patches_k(const float* patch, const int* koff, char* img) {
#pragma unroll
  for (int j = 0; j < TW * 24 / 256; ++j) {
    const int it = threadIdx.x + j * 256;
    const int px = it / 24, cc = it - px * 24, kc = cc >> 3, c8 = cc & 7;
    *reinterpret_cast<uint4*>(img + kc * IMG + px * 128 + ((c8 ^ ((px >> 1) & 7)) << 4)) =
        patch_chunk<E>(patch, koff, px, cc * 8);
  }
}

// weight-gradient operand: three pixel-row images [64 px][64 k] in the transposed layout
// (stage_r: chunk c of k-row px at position c ^ tr_swz<64>(px)), read with frag_r
template <typename E>
__device__ __forceinline__ void build_patches_r(const float* patch, const int* koff, char* img) {
#pragma unroll
  for (int j = 0; j < TW * 24 / 256; ++j) {
    const int it = threadIdx.x + j * 256;
    const int px = it / 24, cc = it - px * 24, kc = cc >> 3, c8 = cc & 7;
    *reinterpret_cast<uint4*>(img + kc * IMG + px * 128 + ((c8 ^ tr_swz<64>(px)) << 4)) =
        patch_chunk<E>(patch, koff, px, cc * 8);
  }
}

// LN (optional, gamma != nullptr): OverlapPatchEmbed.norm (dual_segformer.py:198,219) on the
// conv output in the same epilogue -- a row's N <= 64 channels are 8 consecutive lanes' values,
// so the row statistics are an 8-lane shuffle sum.  The statistics are taken on the stored
// (16-bit rounded) conv output, in the LayerNorm kernel's order (per-lane sums of 8, then the
// lane shuffle), so y_ln / mean / rstd are those cmx_layernorm_fwd computes from y.
struct Pe1Norm {
  const float* gamma;
  const float* beta;
  void* y;
  float* mean;
  float* rstd;
  long sgb;                                     // gamma / beta group stride
  float eps;
};

template <typename E>
__global__ __launch_bounds__(256) void pe1_fwd_kernel(const float* __restrict__ img0, const float* __restrict__ img1,
                                                      const E* __restrict__ Wt, const float* __restrict__ bias,
                                                      E* __restrict__ y, int H, int W, int Ho, int Wo, int N, int Kp,
                                                      long sW, long sbias, long sy, const Pe1Norm ln) {
  __shared__ __attribute__((aligned(1024))) char smem[6 * IMG + PATCH_BYTES];
  char* pimg = smem;                            // 3 patch images
  char* wimg = smem + 3 * IMG;                  // 3 weight images
  float* patch = reinterpret_cast<float*>(smem + 6 * IMG);
  int* koff = reinterpret_cast<int*>(patch + PROWS * PWP);
  init_patch_consts(patch, koff);
  const int g = blockIdx.z, b = blockIdx.y;
  const int tpr = (Wo + TW - 1) / TW;
  const int oy = blockIdx.x / tpr, ox0 = (blockIdx.x - oy * tpr) * TW;
  const int npx = min(TW, Wo - ox0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const float* img = (g == 0 ? img0 : img1) + (long)b * PE_C * H * W;
  const i32x4 rW = make_rsrc(Wt + (long)g * sW);
#pragma unroll
  for (int kc = 0; kc < 3; ++kc) stage_k<64>(rW, wimg + kc * IMG, Kp, 0, N, kc * 64, Kp, w, lane);
  {
    PatchRegs pr;
    load_patch(img, pr, H, W, oy * PE_S - PE_P, ox0 * PE_S - PE_P);
    store_patch(patch, pr);
  }
  __syncthreads();
  build_patches_k<E>(patch, koff, pimg);
  vm_wait<0>();
  __syncthreads();
  f32x16 acc = zero16();
#pragma unroll
  for (int kc = 0; kc < 3; ++kc)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = MF<E>::mma(frag_k<E>(wimg + kc * IMG, wn * 32, s, lane), frag_k<E>(pimg + kc * IMG, wm * 32, s, lane), acc);
  __syncthreads();
  // epilogue through an fp32 LDS tile: lane (r, h) register q holds C(px = r, n = accrow(q, h))
  constexpr int CP = 68;
  float* cs = reinterpret_cast<float*>(smem);
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4)
    *reinterpret_cast<float4*>(cs + (wm * 32 + r) * CP + wn * 32 + 8 * g4 + 4 * h) =
        make_float4(acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]);
  __syncthreads();
  const int jl = (threadIdx.x & 7) * 8;
  if (jl >= N) return;
  const float* bb = bias ? bias + (long)g * sbias + jl : nullptr;
  const long row0 = (long)b * Ho * Wo + (long)oy * Wo + ox0;     // row of the tile's first pixel in group g
  E* yrow = y + (long)g * sy + row0 * N + jl;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int il = pass * 32 + (threadIdx.x >> 3);
    if (il >= npx) break;
    float v[8];
    const float4 u0 = *reinterpret_cast<const float4*>(cs + il * CP + jl);
    const float4 u1 = *reinterpret_cast<const float4*>(cs + il * CP + jl + 4);
    v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w; v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
    if (bb) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bb[e];
    }
    store_vec<E>(yrow + (long)il * N, v);
    if (ln.gamma) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[e] = to_f32(from_f32<E>(v[e])); s += v[e]; }
      s = group_sum(s, N >> 3);
      const float mu = s / N;
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[e] - mu; q += d * d; }
      q = group_sum(q, N >> 3);
      const float rstd = rsqrtf(q / N + ln.eps);
      const float* gm = ln.gamma + (long)g * ln.sgb + jl;
      const float* bt = ln.beta + (long)g * ln.sgb + jl;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (v[e] - mu) * rstd * gm[e] + bt[e];
      store_vec<E>(reinterpret_cast<E*>(ln.y) + (long)g * sy + (row0 + il) * N + jl, v);
      if (jl == 0) {
        const long grow = (long)g * ((long)gridDim.y * Ho * Wo) + row0 + il;
        ln.mean[grow] = mu;
        ln.rstd[grow] = rstd;
      }
    }
  }
}

// one workgroup: tiles [blk * tpb, (blk + 1) * tpb) of group g (tile = (image, oy, ox0));
// dy (G, B*Ho*Wo, N) rows of a tile are contiguous, DMA'd as the A image [64 px][64 n]
template <typename E>
__global__ __launch_bounds__(256) void pe1_wgrad_kernel(const E* __restrict__ dy, const float* __restrict__ img0,
                                                        const float* __restrict__ img1, float* __restrict__ ws, int B,
                                                        int H, int W, int Ho, int Wo, int N, int Kp, long sdy,
                                                        int tpb) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * IMG + PATCH_BYTES];
  char* aimg = smem;                            // dy tile, transposed layout
  char* pimg = smem + IMG;                      // 3 patch images, transposed layout
  float* patch = reinterpret_cast<float*>(smem + 4 * IMG);
  int* koff = reinterpret_cast<int*>(patch + PROWS * PWP);
  init_patch_consts(patch, koff);
  const int g = blockIdx.y, nblk = gridDim.x;
  const int tpr = (Wo + TW - 1) / TW, tpi = Ho * tpr, ntile = B * tpi;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 31, h = lane >> 5;
  const i32x4 rdy = make_rsrc(dy + (long)g * sdy);
  const float* imgs = g == 0 ? img0 : img1;
  constexpr uint32_t one2 = (uint32_t)one_bits<E> * 0x10001u;
  const frag8<E> ones = __builtin_bit_cast(frag8<E>, make_uint4(one2, one2, one2, one2));
  f32x16 acc[3], accd = zero16();
#pragma unroll
  for (int kc = 0; kc < 3; ++kc) acc[kc] = zero16();
  const int t0 = blockIdx.x * tpb, t1 = min(ntile, t0 + tpb);
  auto tile_of = [&](int t, int& b, int& oy, int& ox0) {
    b = t / tpi;
    const int rem = t - b * tpi;
    oy = rem / tpr;
    ox0 = (rem - oy * tpr) * TW;
  };
  PatchRegs pr;                                 // the footprint of the tile being staged next
  if (t0 < t1) {
    int b, oy, ox0;
    tile_of(t0, b, oy, ox0);
    load_patch(imgs + (long)b * PE_C * H * W, pr, H, W, oy * PE_S - PE_P, ox0 * PE_S - PE_P);
  }
  for (int t = t0; t < t1; ++t) {
    int b, oy, ox0;
    tile_of(t, b, oy, ox0);
    const int npx = min(TW, Wo - ox0);
    const int m0 = (b * Ho + oy) * Wo + ox0;
    store_patch(patch, pr);                     // waits for this tile's footprint loads
    stage_r<64>(rdy, aimg, N, 0, N, m0, m0 + npx, w, lane);
    __syncthreads();
    if (t + 1 < t1) {                           // next tile's footprint in flight during this one
      int b2, oy2, ox2;
      tile_of(t + 1, b2, oy2, ox2);
      load_patch(imgs + (long)b2 * PE_C * H * W, pr, H, W, oy2 * PE_S - PE_P, ox2 * PE_S - PE_P);
      build_patches_r<E>(patch, koff, pimg);
      vm_wait<PL>();                            // the dy DMA (issued before the PL prefetch loads)
    } else {
      build_patches_r<E>(patch, koff, pimg);
      vm_wait<0>();
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const frag8<E> fa = frag_r<E, 64>(aimg, wm * 32, s, lane);
#pragma unroll
      for (int kc = 0; kc < 3; ++kc) acc[kc] = MF<E>::mma(frag_r<E, 64>(pimg + kc * IMG, wn * 32, s, lane), fa, acc[kc]);
      if (wn == 0) accd = MF<E>::mma(ones, fa, accd);
    }
    __syncthreads();                            // the images are refilled by the next tile
  }
  // slab (N, Kp + 1): lane (r, h) register q holds C(n = wm*32 + r, k = kc*64 + wn*32 + accrow(q, h));
  // staged through LDS so the slab rows leave as contiguous stores
  constexpr int CP = 196;
  float* cs = reinterpret_cast<float*>(smem);   // 64 x 196 fp32 = 50 KB (images + patch region)
#pragma unroll
  for (int kc = 0; kc < 3; ++kc)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *reinterpret_cast<float4*>(cs + (wm * 32 + r) * CP + kc * 64 + wn * 32 + 8 * g4 + 4 * h) =
          make_float4(acc[kc][4 * g4], acc[kc][4 * g4 + 1], acc[kc][4 * g4 + 2], acc[kc][4 * g4 + 3]);
  if (wn == 0 && h == 0) cs[(wm * 32 + r) * CP + 192] = accd[0];   // every register: sum_px dy(px, n)
  __syncthreads();
  float* out = ws + (long)(g * nblk + blockIdx.x) * N * (Kp + 1);
  for (int e = threadIdx.x; e < N * (Kp + 1); e += 256) {
    const int n = e / (Kp + 1), k = e - n * (Kp + 1);
    out[e] = cs[n * CP + (k == Kp ? 192 : k)];
  }
}

constexpr int PE1_TPB = 4;                      // tiles per weight-gradient workgroup (360 at B2 480 x 640: one round, two per CU)

int pe1_check(int N, int Kp, int KH, int KW, int stride, int pad, int C) {
  CMX_REQUIRE(C == PE_C && KH == PE_K && KW == PE_K && stride == PE_S && pad == PE_P, CMX_ERR_SHAPE,
              "pe1: the stage-1 patch embed (C 3, k 7, s 4, p 3) only (C=%d k=%dx%d s=%d p=%d)", C, KH, KW, stride, pad);
  CMX_REQUIRE(N > 0 && N <= 64 && N % 8 == 0 && Kp >= PE_KR && Kp <= 192 && Kp % 8 == 0, CMX_ERR_SHAPE,
              "pe1: N=%d (<= 64, %% 8) Kp=%d (147..192, %% 8)", N, Kp);
  return CMX_OK;
}

}  // namespace

extern "C" {

int cmx_pe1_conv_fwd(const float* img0, const float* img1, const void* Wt, const float* bias, void* y, int G, int B,
                     int C, int H, int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int Kp, int64_t sW,
                     int64_t sbias, int64_t sy, const float* gamma, const float* beta, void* y_ln, float* mean,
                     float* rstd, int64_t sgb, float eps, int dtype, hipStream_t s) {
  const int st = pe1_check(N, Kp, KH, KW, stride, pad, C);
  if (st != CMX_OK) return st;
  CMX_REQUIRE(!gamma || (beta && y_ln && mean && rstd && (N == 32 || N == 64) && ((uintptr_t)y_ln & 15) == 0),
              CMX_ERR_ARG, "pe1_conv_fwd: the LayerNorm epilogue needs beta / y_ln / mean / rstd and N 32 or 64 (N=%d)",
              N);
  const Pe1Norm ln{gamma, beta, y_ln, mean, rstd, (long)sgb, eps};
  CMX_REQUIRE((dtype == 1 || dtype == 2) && (G == 1 || G == 2) && B > 0 && img0 && (G == 1 || img1), CMX_ERR_ARG,
              "pe1_conv_fwd: 16-bit, G 1 or 2 (dtype %d, G %d)", dtype, G);
  CMX_REQUIRE(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1, CMX_ERR_SHAPE,
              "pe1_conv_fwd: output grid");
  CMX_REQUIRE(((uintptr_t)Wt & 15) == 0 && ((uintptr_t)y & 15) == 0 && sW % 8 == 0 && sy % 8 == 0 &&
              (long)N * Kp < (1L << 28), CMX_ERR_ARG, "pe1_conv_fwd: alignment");
  const dim3 grid(Ho * ((Wo + TW - 1) / TW), B, G);
  if (dtype == 2)
    hipLaunchKernelGGL(pe1_fwd_kernel<f16>, grid, dim3(256), 0, s, img0, img1, (const f16*)Wt, bias, (f16*)y, H, W, Ho,
                       Wo, N, Kp, (long)sW, (long)sbias, (long)sy, ln);
  else
    hipLaunchKernelGGL(pe1_fwd_kernel<bf16>, grid, dim3(256), 0, s, img0, img1, (const bf16*)Wt, bias, (bf16*)y, H, W,
                       Ho, Wo, N, Kp, (long)sW, (long)sbias, (long)sy, ln);
  return cmx_check_launch("pe1_conv_fwd");
}

int cmx_pe1_conv_wgrad_nblk(int B, int Ho, int Wo) {
  const long ntile = (long)B * Ho * ((Wo + TW - 1) / TW);
  return (int)((ntile + PE1_TPB - 1) / PE1_TPB);
}

int cmx_pe1_conv_wgrad(const void* dy, const float* img0, const float* img1, float* ws, int G, int B, int C, int H,
                       int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int Kp, int64_t sdy, int dtype,
                       hipStream_t s) {
  const int st = pe1_check(N, Kp, KH, KW, stride, pad, C);
  if (st != CMX_OK) return st;
  CMX_REQUIRE((dtype == 1 || dtype == 2) && (G == 1 || G == 2) && B > 0 && img0 && (G == 1 || img1) && ws, CMX_ERR_ARG,
              "pe1_conv_wgrad: 16-bit, G 1 or 2 (dtype %d, G %d)", dtype, G);
  CMX_REQUIRE(((uintptr_t)dy & 15) == 0 && sdy % 8 == 0 && (long)B * Ho * Wo * N < (1L << 30), CMX_ERR_ARG,
              "pe1_conv_wgrad: alignment / size");
  const int nblk = cmx_pe1_conv_wgrad_nblk(B, Ho, Wo);
  if (dtype == 2)
    hipLaunchKernelGGL(pe1_wgrad_kernel<f16>, dim3(nblk, G), dim3(256), 0, s, (const f16*)dy, img0, img1, ws, B, H, W,
                       Ho, Wo, N, Kp, (long)sdy, PE1_TPB);
  else
    hipLaunchKernelGGL(pe1_wgrad_kernel<bf16>, dim3(nblk, G), dim3(256), 0, s, (const bf16*)dy, img0, img1, ws, B, H,
                       W, Ho, Wo, N, Kp, (long)sdy, PE1_TPB);
  return cmx_check_launch("pe1_conv_wgrad");
}

}  // extern "C"

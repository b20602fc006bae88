// Mix-FFN band kernels: fc1 + DWConv3x3 + GELU as ONE launch (forward), fc2's input gradient +
// the DWConv / GELU backward as ONE launch (backward), for the short-sequence stages (3 / 4).
//
// Reference: Mlp.forward (dual_segformer.py:67-74): x = fc1(x); x = dwconv(x, H, W) (3x3
// depthwise, pad 1, + bias, :27-33); x = GELU(x); x = fc2(x).  Separate launches leave the
// fc1 output h to go through HBM once more and pay two launch boundaries; at stages 3 / 4 each
// launch is a 10-20 us latency chain (the stage-3/4 blocks at 3-5 % of MFMA).
//
// A workgroup owns one 64-channel slab of the hidden dim for a BAND of R image rows of one image:
//   forward:  h = x W1^T + b1 on the band's rows plus one halo row above and below (those rows'
//             fc1 recomputed: (R + 2) / R of fc1's MFMA work), h rounded to the storage type in
//             LDS, then z = DW(h) + bdw on the band's own pixels, a = GELU(z), act'(z) -- exactly
//             the operations and rounding points of gemm (fc1) + dw2_fwd_kernel, so h, a and
//             act'(z) are bit-identical to the separate launches;
//   backward: da = dz2 W2 (fc2's input gradient) on the band's rows plus the halo, rounded, times
//             the saved act'(z) (rounded: dz), then dh = DW^T(dz) on the band's pixels and the
//             partial dW / db sums h . dz over them (one fp32 slab per (band tile, slab) for the
//             deferred grouped reduce, the layout of dw2_bwdg_kernel's partials).
// Band rows R = 256 / W - 2 (the extended band fits the 256-row MFMA tile).  Wide images (R < 4:
// stages 1-2, W = 160 / 80) take 2-D tiles instead: TH x TW = 12 x 16 pixels, extended 14 x 18 =
// 252 rows (fc1 recomputed on 1.31x the pixels, K = C = 64 / 128: one or two k-tiles), so a tile's
// rows are gathered pixel segments rather than one contiguous token range.  The GEMM part is the
// MFMA tile loop of gemm_kernels.h (LDS-DMA ring of 2 stages, 4 waves 2 x 2, 32x32x16 MFMA) on a
// 256 x 64 tile; the DW part is dw2_fwd_kernel's channel-fast mapping (16 lanes x 4 channels per
// pixel) on the LDS image.
#include "gemm_kernels.h"

namespace {
using namespace gemmk;

constexpr int MB = 256;                  // extended-band rows per tile (MFMA rows)
constexpr int SL = 64;                   // hidden channels per slab
constexpr int STG = (MB + SL) * FBK * 2; // one ring stage: A 256 x 64 + B 64 x 64 (bf16)
constexpr int MIX_SMEM = 2 * STG;        // 80 KB: two stages (the bf16 band image reuses it)

constexpr int TH2 = 12, TW2 = 16;          // 2-D tile (interior pixels) of the wide stages

struct MixArgs {
  const void* A;       // fwd: x (G, M, C) (norm2 output); bwd: dz2 (G, M, C) (fc2's output gradient)
  const void* B;       // fwd: W1 (G, Ch, C) k-contiguous; bwd: W2 (G, C, Ch): B(j, k) = W2[k][j]
  const float* bias;   // fwd: b1 (G, Ch); bwd: unused
  const float* wdw;    // (G, Ch, 9)
  const float* bdw;    // (G, Ch)
  void* h;             // fwd: out; bwd: in -- fc1 output (G, M, Ch)
  void* gp;            // fwd: out; bwd: in -- act'(z) (G, M, Ch)
  void* a;             // fwd: out -- GELU(z) (G, M, Ch)
  void* dh;            // bwd: out (G, M, Ch)
  float* part;         // bwd: out, dW / db partials (G, nsp, Ch * 10), nsp = ipg * nbands
  int G, ipg, H, W, C, Ch, R, nbands, nslab;
  int TW, ntx;         // tile width (= W for bands) and tiles across; R = tile height, nbands = tiles down
  long sA, sB, sbias;  // group strides (elements)
};

// tile of block `lin`: (g, image, tile, slab); interior [y0, y1) x [x0, x1), extended (one halo
// pixel each side, clipped to the image) [ey0, ey1) x [ex0, ex0 + ecols): LDS / MFMA row r of the
// tile is extended pixel (ey0 + r / ecols, ex0 + r % ecols).  A band is a tile of full rows
// (TW = W, ntx = 1): its extended rows are one contiguous token range.
struct Band {
  int g, img, band, slab, y0, y1, x0, x1, ey0, ex0, ecols, erows;
};
__device__ __forceinline__ Band band_of(const MixArgs& p, int lin) {
  Band b;
  b.slab = lin % p.nslab;
  int r = lin / p.nslab;
  b.band = r % (p.nbands * p.ntx); r /= p.nbands * p.ntx;
  b.img = r % p.ipg;
  b.g = r / p.ipg;
  const int ty = b.band / p.ntx, tx = b.band - ty * p.ntx;
  b.y0 = ty * p.R;
  b.y1 = min(p.H, b.y0 + p.R);
  b.x0 = tx * p.TW;
  b.x1 = min(p.W, b.x0 + p.TW);
  b.ey0 = max(0, b.y0 - 1);
  b.ex0 = max(0, b.x0 - 1);
  b.ecols = min(p.W, b.x1 + 1) - b.ex0;
  b.erows = min(p.H, b.y1 + 1) - b.ey0;
  return b;
}
// group-local token of extended row r (-1: past the tile)
__device__ __forceinline__ int ext_token(const MixArgs& p, const Band& t, int r) {
  if (r >= t.erows * t.ecols) return -1;
  const int yy = t.ey0 + r / t.ecols, xx = t.ex0 + r % t.ecols;
  return (t.img * p.H + yy) * p.W + xx;
}
// LDS / MFMA row of image pixel (yy, xx) of the extended tile
__device__ __forceinline__ int ext_row(const Band& t, int yy, int xx) { return (yy - t.ey0) * t.ecols + (xx - t.ex0); }

// LDS image of the extended band: [row][64 ch] 16-bit, 16-B chunk c of row r at c ^ (r & 7)
__device__ __forceinline__ int img_off(int row, int ch) {       // byte offset of channel ch (multiple of 4)
  return row * 128 + ((((ch >> 3) ^ (row & 7))) << 4) + ((ch & 7) << 1);
}

// h / da tile (rows e0 .. e0 + 255, hidden slab) with MFMA; acc[a] = C^T sub-tiles (see
// gemm_bf16_body): lane (r, hh) register q = C(row = 128 wm + 32 a + r, col = 32 wn + accrow(q, hh))
template <typename E, bool TB>
__device__ __forceinline__ void band_gemm(const MixArgs& p, const Band& t, char* smem, f32x16 (&acc)[4]) {
  constexpr int A_BYTES = MB * FBK * 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const E* Ag = reinterpret_cast<const E*>(p.A) + (long)t.g * p.sA;
  const E* Bg = reinterpret_cast<const E*>(p.B) + (long)t.g * p.sB;
  const i32x4 rA = make_rsrc(Ag), rB = make_rsrc(Bg);
  const int j0 = t.slab * SL;
#pragma unroll
  for (int a = 0; a < 4; ++a) acc[a] = zero16();
  const int nk = (p.C + FBK - 1) / FBK;
  // the lane's A rows (one per staging instruction, the order of stage_k<MB>): tokens decoded once
  constexpr int NIA = MB / 32;
  int tok[NIA];
#pragma unroll
  for (int n = 0; n < NIA; ++n) tok[n] = ext_token(p, t, (w * NIA + n) * 8 + (lane >> 3));
  auto stage = [&](int kt, char* buf) {
    const int k0 = kt * FBK;
#pragma unroll
    for (int n = 0; n < NIA; ++n) {
      const int row = (w * NIA + n) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int gk = k0 + c * 8;
      const int off = (tok[n] >= 0 && gk < p.C) ? (int)(((long)tok[n] * p.C + gk) * 2) : OOB;
      dma16(rA, lds_addr(buf + (w * NIA + n) * 1024), off);
    }
    if constexpr (TB) stage_r<SL>(rB, buf + A_BYTES, p.Ch, j0, p.Ch, k0, p.C, w, lane);
    else stage_k<SL>(rB, buf + A_BYTES, p.C, j0, p.Ch, k0, p.C, w, lane);
  };
  auto compute = [&](const char* buf) {
    const char* ai = buf;
    const char* bi = buf + A_BYTES;
#pragma unroll
    for (int s = 0; s < FBK / 16; ++s) {
      frag8<E> fb;
      if constexpr (TB) fb = frag_r<E, SL>(bi, wn * 32, s, lane);
      else fb = frag_k<E>(bi, wn * 32, s, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[a] = MF<E>::mma(fb, frag_k<E>(ai, wm * 128 + a * 32, s, lane), acc[a]);
    }
  };
  constexpr int PER = MB / 32 + SL / 32;        // LDS-DMA instructions per stage per wave
  stage(0, smem);
  if (nk > 1) stage(1, smem + STG);
  if (nk > 1) vm_wait<PER>(); else vm_wait<0>();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    compute(smem + cur * STG);
    __syncthreads();                                // every wave is done with stage `cur`
    if (kt + 2 < nk) stage(kt + 2, smem + cur * STG);
    if (kt + 1 < nk) {
      if (kt + 2 < nk) vm_wait<PER>(); else vm_wait<0>();
      __syncthreads();                              // stage kt + 1 landed for every wave
    }
  }
}

// acc (+ bias) -> 16-bit image in LDS (rows past e1 - e0 are never read)
template <typename E>
__device__ __forceinline__ void acc_to_image(const f32x16 (&acc)[4], const float* bias, char* img) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int row = wm * 128 + a * 32 + r;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int col = wn * 32 + 8 * g4 + 4 * hh;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[a][4 * g4 + e] + (bias ? bias[col + e] : 0.f);
      *reinterpret_cast<uint2*>(img + img_off(row, col)) = make_uint2(pack2<E>(v[0], v[1]), pack2<E>(v[2], v[3]));
    }
  }
}

__device__ __forceinline__ void load_w36m(const float* wg, cmx_f2 (&w2)[2][9]) {
  const float4* q = reinterpret_cast<const float4*>(wg);
  float w[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 a = q[i];
    w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    w2[0][k] = (cmx_f2){w[k], w[9 + k]};
    w2[1][k] = (cmx_f2){w[18 + k], w[27 + k]};
  }
}

template <typename E>
__device__ __forceinline__ void img_ld4(const char* img, int row, int ch, cmx_f2 (&v)[2]) {
  const uint2 u = *reinterpret_cast<const uint2*>(img + img_off(row, ch));
  v[0] = unpack2<E>(u.x);
  v[1] = unpack2<E>(u.y);
}
template <typename E>
__device__ __forceinline__ void st4g(E* p, const cmx_f2 (&v)[2]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2<E>(v[0].x, v[0].y), pack2<E>(v[1].x, v[1].y));
}

// ------------------------------------------------------------------------------ forward
template <typename E>
__global__ __launch_bounds__(256, 2) void mixffn_fwd_band(const MixArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[MIX_SMEM];
  const int ntile = p.G * p.ipg * p.nbands * p.ntx * p.nslab;
  const Band t = band_of(p, xcd_tile(blockIdx.x, ntile));
  f32x16 acc[4];
  band_gemm<E, false>(p, t, smem, acc);
  const int j0 = t.slab * SL;
  acc_to_image<E>(acc, p.bias + (long)t.g * p.sbias + j0, smem);   // h, rounded as stored
  __syncthreads();
  // DW 3x3 + bias + GELU on the band's own pixels (channel-fast: 16 lanes x 4 channels a pixel)
  const int cq = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int ch = cq * 4;
  cmx_f2 wr[2][9], bias[2];
  load_w36m(p.wdw + ((long)t.g * p.Ch + j0 + ch) * 9, wr);
  {
    const float4 b0 = *reinterpret_cast<const float4*>(p.bdw + (long)t.g * p.Ch + j0 + ch);
    bias[0] = (cmx_f2){b0.x, b0.y};
    bias[1] = (cmx_f2){b0.z, b0.w};
  }
  const long gbase = (long)t.g * p.sA / p.C * p.Ch;           // group base of the (G, M, Ch) tensors
  E* hg = reinterpret_cast<E*>(p.h) + gbase;
  E* ag = reinterpret_cast<E*>(p.a) + gbase;
  E* gg = reinterpret_cast<E*>(p.gp) + gbase;
  const int N = p.H * p.W;
  const int tw = t.x1 - t.x0;
  const int npx = (t.y1 - t.y0) * tw;
  for (int q = pl; q < npx; q += 16) {
    const int y = t.y0 + q / tw, x = t.x0 + q % tw;
    cmx_f2 z[2] = {bias[0], bias[1]};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int yy = y + i - 1, xx = x + j - 1;
        cmx_f2 v[2] = {pk_splat(0.f), pk_splat(0.f)};
        if (yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) img_ld4<E>(smem, ext_row(t, yy, xx), ch, v);
#pragma unroll
        for (int u = 0; u < 2; ++u) z[u] = pk_fma(wr[u][i * 3 + j], v[u], z[u]);
      }
    const long o = ((long)t.img * N + (long)y * p.W + x) * p.Ch + j0 + ch;
    cmx_f2 hv[2];
    img_ld4<E>(smem, ext_row(t, y, x), ch, hv);
    st4g<E>(hg + o, hv);
    cmx_f2 gd[2], av[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gd[u] = act2_grad<1>(z[u]);
      av[u] = act2_fwd<1>(z[u]);
    }
    st4g<E>(gg + o, gd);
    st4g<E>(ag + o, av);
  }
}

// ------------------------------------------------------------------------------ backward
template <typename E>
__global__ __launch_bounds__(256, 2) void mixffn_bwd_band(const MixArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[MIX_SMEM];
  const int ntile = p.G * p.ipg * p.nbands * p.ntx * p.nslab;
  const Band t = band_of(p, xcd_tile(blockIdx.x, ntile));
  f32x16 acc[4];
  band_gemm<E, true>(p, t, smem, acc);
  const int j0 = t.slab * SL;
  acc_to_image<E>(acc, nullptr, smem);                       // da, rounded as stored
  __syncthreads();
  const long gbase = (long)t.g * p.sA / p.C * p.Ch;
  const E* gpg = reinterpret_cast<const E*>(p.gp) + gbase;
  const E* hgl = reinterpret_cast<const E*>(p.h) + gbase;
  // dz = da * act'(z) on the extended band, rounded as stored, in place (16-B chunks: every
  // act' load of the thread issued before the first multiply)
  const int erows = t.erows * t.ecols;
  {
    constexpr int IT = MB * 8 / 256;                         // 8 chunks of 8 channels a row
    uint4 gv[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int it = threadIdx.x + k * 256, row = it >> 3, c8 = it & 7;
      const int tk = ext_token(p, t, row);
      gv[k] = tk >= 0 ? *reinterpret_cast<const uint4*>(gpg + (long)tk * p.Ch + j0 + c8 * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int it = threadIdx.x + k * 256, row = it >> 3, c8 = it & 7;
      if (row >= erows) continue;
      uint4* cp = reinterpret_cast<uint4*>(smem + row * 128 + ((c8 ^ (row & 7)) << 4));
      const uint4 d = *cp;
      const uint32_t dw4[4] = {d.x, d.y, d.z, d.w}, gw4[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
      uint32_t o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const cmx_f2 a = unpack2<E>(dw4[q]) * unpack2<E>(gw4[q]);
        o4[q] = pack2<E>(a.x, a.y);
      }
      *cp = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
  }
  __syncthreads();
  // dh = DW^T(dz) on the band's pixels; dW[tap] += h . dz[p + (1 - i, 1 - j)], db += dz[p]
  const int cq = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int ch = cq * 4;
  cmx_f2 wr[2][9];
  load_w36m(p.wdw + ((long)t.g * p.Ch + j0 + ch) * 9, wr);
  cmx_f2 pacc[2][10];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) pacc[u][k] = pk_splat(0.f);
  E* dhg = reinterpret_cast<E*>(p.dh) + gbase;
  const int N = p.H * p.W;
  const int tw = t.x1 - t.x0;
  const int npx = (t.y1 - t.y0) * tw;
  for (int q = pl; q < npx; q += 16) {
    const int y = t.y0 + q / tw, x = t.x0 + q % tw;
    const long o = ((long)t.img * N + (long)y * p.W + x) * p.Ch + j0 + ch;
    cmx_f2 hv[2];
    {
      const uint2 u2 = *reinterpret_cast<const uint2*>(hgl + o);
      hv[0] = unpack2<E>(u2.x);
      hv[1] = unpack2<E>(u2.y);
    }
    cmx_f2 gsum[2] = {pk_splat(0.f), pk_splat(0.f)};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int yy = y + 1 - i, xx = x + 1 - j;
        cmx_f2 dv[2] = {pk_splat(0.f), pk_splat(0.f)};
        if (yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) img_ld4<E>(smem, ext_row(t, yy, xx), ch, dv);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          gsum[u] = pk_fma(wr[u][i * 3 + j], dv[u], gsum[u]);
          pacc[u][i * 3 + j] = pk_fma(hv[u], dv[u], pacc[u][i * 3 + j]);
        }
        if (i == 1 && j == 1) {
#pragma unroll
          for (int u = 0; u < 2; ++u) pacc[u][9] += dv[u];
        }
      }
    st4g<E>(dhg + o, gsum);
  }
  // partial dW / db of this tile: the 16 pixel lanes of each channel quad summed through LDS
  __syncthreads();                                           // every wave is done with the dz image
  float* red = reinterpret_cast<float*>(smem);               // [16 pl][64 ch][10]
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      red[(pl * 64 + ch + 2 * u) * 10 + k] = pacc[u][k].x;
      red[(pl * 64 + ch + 2 * u + 1) * 10 + k] = pacc[u][k].y;
    }
  __syncthreads();
  const int nsp = p.ipg * p.nbands * p.ntx, sp = t.img * p.nbands * p.ntx + t.band;
  float* out = p.part + ((long)t.g * nsp + sp) * p.Ch * 10 + (long)j0 * 10;
  for (int e = threadIdx.x; e < SL * 10; e += 256) {
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) s += red[l * SL * 10 + e];
    out[e] = s;
  }
}

int mix_check(const MixArgs& a, int dtype) {
  CMX_REQUIRE(dtype == 1 || dtype == 2, CMX_ERR_DTYPE, "mixffn: bf16 / fp16 only (dtype %d)", dtype);
  CMX_REQUIRE(a.G > 0 && a.ipg > 0 && a.H > 0 && a.W > 0 && a.C % 8 == 0 && a.C > 0 && a.Ch % SL == 0, CMX_ERR_SHAPE,
              "mixffn: C %% 8, hidden %% 64 (C=%d Ch=%d)", a.C, a.Ch);
  CMX_REQUIRE(a.R >= 1 && a.TW >= 1 && (a.R + 2) * (a.TW == a.W ? a.W : a.TW + 2) <= MB, CMX_ERR_SHAPE,
              "mixffn: a tile of %d x %d pixels + halo does not fit %d tokens (W=%d)", a.R, a.TW, MB, a.W);
  CMX_REQUIRE(((uintptr_t)a.A & 15) == 0 && ((uintptr_t)a.B & 15) == 0 && a.sA == (long)a.ipg * a.H * a.W * a.C &&
                  a.sB % 8 == 0, CMX_ERR_ARG, "mixffn: contiguous (G, M, C) activations, 16-B aligned operands");
  return CMX_OK;
}

// tiling of an H x W image: bands of R full rows when R = 256 / W - 2 >= 4, else TH2 x TW2 tiles
void mix_tiling(MixArgs& p) {
  const int R = p.W > 0 ? MB / p.W - 2 : 0;
  if (R >= 4) {
    p.R = R; p.TW = p.W;
  } else {
    p.R = TH2; p.TW = TW2;
  }
  p.nbands = (p.H + p.R - 1) / p.R;
  p.ntx = (p.W + p.TW - 1) / p.TW;
}

}  // namespace

extern "C" {

int cmx_mixffn_band_rows(int W) { return W > 0 && MB / W - 2 >= 1 ? MB / W - 2 : 0; }

int cmx_mixffn_mode(int W) { return W > 0 && MB / W - 2 >= 4 ? 1 : 2; }

size_t cmx_mixffn_bwd_workspace(int G, int ipg, int H, int W, int Ch) {
  MixArgs p{};
  p.H = H; p.W = W;
  if (H <= 0 || W <= 0) return 0;
  mix_tiling(p);
  return (size_t)G * ipg * p.nbands * p.ntx * Ch * 10 * sizeof(float);
}

int cmx_mixffn_fwd(const void* x, const void* W1, const float* b1, const float* wdw, const float* bdw, void* h,
                   void* gprime, void* a, int G, int ipg, int H, int W, int C, int Ch, int64_t sW, int64_t sb,
                   int64_t sdw, int dtype, hipStream_t s) {
  MixArgs p{};
  p.A = x; p.B = W1; p.bias = b1; p.wdw = wdw; p.bdw = bdw; p.h = h; p.gp = gprime; p.a = a;
  p.G = G; p.ipg = ipg; p.H = H; p.W = W; p.C = C; p.Ch = Ch;
  mix_tiling(p);
  p.sA = (long)ipg * H * W * C; p.sB = sW; p.sbias = sb;
  const int st = mix_check(p, dtype);
  if (st) return st;
  CMX_REQUIRE(b1 && wdw && bdw && h && gprime && a && sdw == (long)Ch * 9 && sb == Ch, CMX_ERR_ARG,
              "mixffn_fwd: buffers / (G, Ch) bias and (G, Ch, 9) DW weight layouts");
  p.nslab = Ch / SL;
  const unsigned grid = (unsigned)(G * ipg * p.nbands * p.ntx * p.nslab);
  if (dtype == 2) hipLaunchKernelGGL(mixffn_fwd_band<f16>, dim3(grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(mixffn_fwd_band<bf16>, dim3(grid), dim3(256), 0, s, p);
  return cmx_check_launch("mixffn_fwd");
}

int cmx_mixffn_bwd(const void* dz2, const void* W2, const float* wdw, const void* h, const void* gprime, void* dh,
                   float* workspace, int G, int ipg, int H, int W, int C, int Ch, int64_t sW, int64_t sdw, int dtype,
                   hipStream_t s) {
  MixArgs p{};
  p.A = dz2; p.B = W2; p.wdw = wdw; p.h = const_cast<void*>(h); p.gp = const_cast<void*>(gprime); p.dh = dh;
  p.part = workspace;
  p.G = G; p.ipg = ipg; p.H = H; p.W = W; p.C = C; p.Ch = Ch;
  mix_tiling(p);
  p.sA = (long)ipg * H * W * C; p.sB = sW;
  const int st = mix_check(p, dtype);
  if (st) return st;
  CMX_REQUIRE(wdw && h && gprime && dh && workspace && sdw == (long)Ch * 9, CMX_ERR_ARG,
              "mixffn_bwd: buffers / (G, Ch, 9) DW weight layout");
  p.nslab = Ch / SL;
  const unsigned grid = (unsigned)(G * ipg * p.nbands * p.ntx * p.nslab);
  if (dtype == 2) hipLaunchKernelGGL(mixffn_bwd_band<f16>, dim3(grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(mixffn_bwd_band<bf16>, dim3(grid), dim3(256), 0, s, p);
  return cmx_check_launch("mixffn_bwd");
}

}  // extern "C"

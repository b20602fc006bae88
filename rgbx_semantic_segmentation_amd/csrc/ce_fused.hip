// Final upsample + CrossEntropyLoss, tiled through LDS (forward loss and fused backward).
//
// Same math as upsample_ce.hip (builder.py:233,249; train.py:72-73: bilinear x4 upsample,
// align_corners=False, then mean CE over pixels != ignore_index), re-tiled so that neither
// the full-resolution logits NOR their gradient ever reach HBM:
//  * forward: a block owns a 16 x 16 full-res tile, stages the low-res logits it reads
//    (<= 6 x 6 x K, fp32) in LDS once, and each thread does one pixel's interpolation +
//    log-softmax + NLL.  Only per-block loss / count partials are written.
//  * backward: a block owns a TY x TX low-res tile of dlogits.  It recomputes the softmax
//    gradient g = (p - onehot) * dloss / n_valid of every full-res pixel whose bilinear
//    footprint touches the tile (<= 20 x 20 pixels at scale 4) into LDS, then applies the
//    separable bilinear adjoint (x, then y) in LDS and writes the tile once.  The 2-pass
//    adjoint of a materialised (B, H, W, K) gradient (49 MB at 480 x 640, K = 40) is gone.
#include "cmx_common.h"

namespace {

__device__ __forceinline__ void src_idx(int dst, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  float s = (dst + 0.5f) * scale - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

constexpr int KF = 40;                  // classes held in LDS (NYUv2 40, Cityscapes 19, MFNet 9)
constexpr int FT = 16;                  // forward full-res tile edge
constexpr int LRF = FT / 4 + 3;         // low-res rows / cols a forward tile can read (scale <= 4)
constexpr int TY = 4, TX = 4;           // backward low-res tile
constexpr int RY = 4 * TY + 4, RX = 4 * TX + 4;   // full-res footprint rows / cols (scale 4)

// ------------------------------------------------------------------------ forward (loss only)
template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_tiled(const T* __restrict__ logits, const int64_t* __restrict__ label,
                                                    float* __restrict__ part, int h, int w, int H, int W, int K,
                                                    int ignore, int tiles_x, int tiles_y) {
  __shared__ float lg[LRF * LRF * KF];
  __shared__ float red[2][256];
  const int bx = blockIdx.x % tiles_x, by = (blockIdx.x / tiles_x) % tiles_y, b = blockIdx.x / (tiles_x * tiles_y);
  const float sh = (float)h / H, sw = (float)w / W;
  const int Y0 = by * FT, X0 = bx * FT;
  int ly0, lx0, t1;
  float f0, f1;
  src_idx(Y0, sh, h, ly0, t1, f0, f1);
  src_idx(X0, sw, w, lx0, t1, f0, f1);
  const T* base = logits + (long)b * h * w * K;
  const int Y = Y0 + threadIdx.x / FT, X = X0 + threadIdx.x % FT;
  // every global load of the thread (its label, its share of the logits tile) is issued
  // before the first LDS store: one memory latency per block instead of one per 256 items
  const long lab = (Y < H && X < W) ? label[((long)b * H + Y) * W + X] : (long)ignore;
  constexpr int NL = (LRF * LRF * KF + 255) / 256;
  float v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = threadIdx.x + i * 256;
    const int k = e % K, px = e / K;
    const int yy = ly0 + px / LRF, xx = lx0 + px % LRF;
    v[i] = (e < LRF * LRF * K && yy < h && xx < w) ? to_f32(base[((long)yy * w + xx) * K + k]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = threadIdx.x + i * 256;
    if (e < LRF * LRF * K) lg[(e % K) * (LRF * LRF) + e / K] = v[i];   // class-major (see the backward)
  }
  __syncthreads();
  float ls = 0.f, lc = 0.f;
  if (Y < H && X < W) {
    if (!(lab == ignore || lab < 0 || lab >= K)) {
      int y0, y1, x0, x1;
      float wy0, wy1, wx0, wx1;
      src_idx(Y, sh, h, y0, y1, wy0, wy1);
      src_idx(X, sw, w, x0, x1, wx0, wx1);
      // class-major image [k][px] (49 pixels per class): the lanes of a wave read at most 10
      // distinct words per class, on distinct banks (a pixel-major [px][k] image put the wave's
      // low-res pixels 40 words apart: 1.7 bank conflicts per LDS read)
      constexpr int LP = LRF * LRF;
      const float* pa = lg + (y0 - ly0) * LRF + (x0 - lx0);
      const float* pb = lg + (y0 - ly0) * LRF + (x1 - lx0);
      const float* pc = lg + (y1 - ly0) * LRF + (x0 - lx0);
      const float* pd = lg + (y1 - ly0) * LRF + (x1 - lx0);
      // compile-time trip counts predicated on k < K: the LDS reads of all classes are in
      // flight together and z stays in registers (a runtime-bound loop waits on each read)
      float z[KF];
      float m = -INFINITY, zl = 0.f;
#pragma unroll
      for (int k = 0; k < KF; ++k) {
        z[k] = k < K ? wy0 * (wx0 * pa[k * LP] + wx1 * pb[k * LP]) + wy1 * (wx0 * pc[k * LP] + wx1 * pd[k * LP])
                     : -INFINITY;
        m = fmaxf(m, z[k]);
        if (k == lab) zl = z[k];
      }
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < KF; ++k) se += __expf(z[k] - m);
      ls = m + __logf(se) - zl;
      lc = 1.f;
    }
  }
  red[0][threadIdx.x] = ls;
  red[1][threadIdx.x] = lc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2] = red[0][0];
    part[blockIdx.x * 2 + 1] = red[1][0];
  }
}

// ------------------------------------------------------------------------ backward (fused)
// full-res rows contributing to low-res rows [y0, y0 + n): the interval of Y whose bilinear
// source pair (i0, i1) meets it (monotone in Y)
__device__ __forceinline__ void footprint(int y0, int n, float scale, int in, int out, int& Ya, int& Yb) {
  int a = (int)floorf((y0 - 1 + 0.5f) / scale - 0.5f) - 2;
  if (a < 0) a = 0;
  int i0, i1;
  float l0, l1;
  for (;; ++a) {
    src_idx(a, scale, in, i0, i1, l0, l1);
    if (i1 >= y0 || a >= out - 1) break;
  }
  int bb = (int)ceilf((y0 + n + 0.5f) / scale - 0.5f) + 2;
  if (bb > out - 1) bb = out - 1;
  for (;; --bb) {
    src_idx(bb, scale, in, i0, i1, l0, l1);
    if (i0 <= y0 + n - 1 || bb <= a) break;
  }
  Ya = a;
  Yb = bb;
}

// eight waves per workgroup: the 400 footprint pixels of phase A take one pass, and 3 resident
// workgroups (LDS-bound) give six waves per SIMD to hide the LDS / exp latency
constexpr int CE_BWD_NT = 512;
template <typename T>
__global__ __launch_bounds__(CE_BWD_NT) void ce_bwd_fused(const T* __restrict__ logits, const int64_t* __restrict__ label,
                                                    const float* __restrict__ dloss, const float* __restrict__ stats,
                                                    T* __restrict__ dlogits, int h, int w, int H, int W, int K,
                                                    int ignore, int tiles_x, int tiles_y) {
  // every LDS image is class-major ([k][pixel]): lanes on consecutive pixels touch consecutive
  // words (a pixel-major [pixel][k] image with K = 40 put 8 lanes on each bank)
  constexpr int LW = TX + 2, LP = (TY + 2) * LW;
  __shared__ float lg[KF * LP];                     // low-res logits: tile + 1-pixel halo
  __shared__ T g[KF * RY * RX];                     // full-res softmax gradient of the footprint
  constexpr int KP = KF + 1;                        // odd pitch: phase C lanes on consecutive k
  __shared__ float t1[RY * TX * KP];                // x-adjoint: (full-res row, low-res col, class)
  __shared__ float wy[TY * RY], wx[TX * RX];        // bilinear adjoint weights of the tile
  const int bx = blockIdx.x % tiles_x, by = (blockIdx.x / tiles_x) % tiles_y, b = blockIdx.x / (tiles_x * tiles_y);
  const int y0 = by * TY, x0 = bx * TX;
  const int ny = min(TY, h - y0), nx = min(TX, w - x0);
  const float sh = (float)h / H, sw = (float)w / W;
  const float gs = dloss[0] * stats[1];               // dloss / n_valid
  int Ya, Yb, Xa, Xb;
  footprint(y0, ny, sh, h, H, Ya, Yb);
  footprint(x0, nx, sw, w, W, Xa, Xb);
  const int ry = Yb - Ya + 1, rx = Xb - Xa + 1;       // <= RY, RX (exact x4, host-checked)
  const int np = ry * rx;
  const T* base = logits + (long)b * h * w * K;
  // all global loads first (logits tile + halo, the labels of the thread's footprint pixels),
  // then the LDS stores: one memory latency per block instead of one per 256 items
  constexpr int NL = (LP * KF + CE_BWD_NT - 1) / CE_BWD_NT, NPX = (RY * RX + CE_BWD_NT - 1) / CE_BWD_NT;
  float v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = threadIdx.x + i * CE_BWD_NT;
    const int k = e % K, px = e / K;                  // coalesced global reads along k
    const int yy = y0 - 1 + px / LW, xx = x0 - 1 + px % LW;
    v[i] = (e < LP * K && yy >= 0 && yy < h && xx >= 0 && xx < w) ? to_f32(base[((long)yy * w + xx) * K + k]) : 0.f;
  }
  long labs[NPX];
#pragma unroll
  for (int i = 0; i < NPX; ++i) {
    const int pi = threadIdx.x + i * CE_BWD_NT;
    labs[i] = pi < np ? label[((long)b * H + Ya + pi / rx) * W + Xa + pi % rx] : (long)ignore;
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = threadIdx.x + i * CE_BWD_NT;
    if (e < LP * K) lg[(e % K) * LP + e / K] = v[i];
  }
  for (int e = threadIdx.x; e < TY * RY + TX * RX; e += CE_BWD_NT) {
    const bool isy = e < TY * RY;
    const int q = isy ? e : e - TY * RY;
    const int R = isy ? RY : RX;
    const int tl = q / R, j = q % R;                  // low-res index within the tile, footprint index
    float wgt = 0.f;
    if (j < (isy ? ry : rx)) {
      int i0, i1;
      float l0, l1;
      src_idx((isy ? Ya : Xa) + j, isy ? sh : sw, isy ? h : w, i0, i1, l0, l1);
      const int t = (isy ? y0 : x0) + tl;
      if (i0 == t) wgt += l0;
      if (i1 == t) wgt += l1;
    }
    (isy ? wy : wx)[q] = wgt;
  }
  __syncthreads();
  // phase A: g for every footprint pixel (one pixel per lane)
#pragma unroll
  for (int i = 0; i < NPX; ++i) {
    const int pi = threadIdx.x + i * CE_BWD_NT;
    if (pi >= np) break;
    const int Y = Ya + pi / rx, X = Xa + pi % rx;
    const long lab = labs[i];
    if (lab == ignore || lab < 0 || lab >= K) {
      for (int k = 0; k < K; ++k) g[k * RY * RX + pi] = from_f32<T>(0.f);
      continue;
    }
    int ya, yb, xa, xb;
    float wy0, wy1, wx0, wx1;
    src_idx(Y, sh, h, ya, yb, wy0, wy1);
    src_idx(X, sw, w, xa, xb, wx0, wx1);
    const int pa = (ya - y0 + 1) * LW + (xa - x0 + 1), pb = (ya - y0 + 1) * LW + (xb - x0 + 1);
    const int pc = (yb - y0 + 1) * LW + (xa - x0 + 1), pd = (yb - y0 + 1) * LW + (xb - x0 + 1);
    const float c00 = wy0 * wx0, c01 = wy0 * wx1, c10 = wy1 * wx0, c11 = wy1 * wx1;
    // compile-time trip counts (predicated on k < K): z stays in registers (a runtime-bound
    // loop over a register array would spill it to scratch)
    float z[KF];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < KF; ++k) {
      const float* l = lg + k * LP;
      z[k] = k < K ? c00 * l[pa] + c01 * l[pb] + c10 * l[pc] + c11 * l[pd] : -INFINITY;
      m = fmaxf(m, z[k]);
    }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < KF; ++k) {
      z[k] = __expf(z[k] - m);
      se += z[k];
    }
    const float inv = gs / se;
#pragma unroll
    for (int k = 0; k < KF; ++k)
      if (k < K) g[k * RY * RX + pi] = from_f32<T>(z[k] * inv - (k == lab ? gs : 0.f));
  }
  __syncthreads();
  // phase B: x-adjoint t1[k][row][xl] = sum_X wx[xl][X] g[k][row][X].  The item index runs over
  // the compile-time box (KF, RY, TX) -- constant divisors -- and skips what the tile lacks; the
  // 8 taps are unchecked when they lie inside the footprint (every column but the image borders')
  for (int e = threadIdx.x; e < KF * RY * TX; e += CE_BWD_NT) {
    const int xl = e % TX, row = (e / TX) % RY, k = e / (TX * RY);
    if (k >= K || row >= ry || xl >= nx) continue;
    const T* gr = g + k * RY * RX + row * rx;
    const float* wr = wx + xl * RX;
    // exact x4 (align_corners=False): low-res column x takes full-res X in [4x - 2, 4x + 6)
    // only (the borders' clamped taps included); the other footprint weights are zero
    const int jb = 4 * (x0 + xl) - 2 - Xa;
    float acc = 0.f;
    if (jb >= 0 && jb + 8 <= rx) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc += wr[jb + jj] * to_f32(gr[jb + jj]);
    } else {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = jb + jj;
        acc += (j >= 0 && j < rx) ? wr[j] * to_f32(gr[j]) : 0.f;
      }
    }
    t1[(row * TX + xl) * KP + k] = acc;
  }
  __syncthreads();
  // phase C: y-adjoint, write the tile (k fastest: coalesced along the NHWC row)
  for (int e = threadIdx.x; e < TY * TX * KF; e += CE_BWD_NT) {
    const int k = e % KF, xl = (e / KF) % TX, yl = e / (KF * TX);
    if (k >= K || xl >= nx || yl >= ny) continue;
    const float* wr = wy + yl * RY;
    const int jb = 4 * (y0 + yl) - 2 - Ya;              // rows [4y - 2, 4y + 6), as above
    float acc = 0.f;
    if (jb >= 0 && jb + 8 <= ry) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc += wr[jb + jj] * t1[((jb + jj) * TX + xl) * KP + k];
    } else {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = jb + jj;
        acc += (j >= 0 && j < ry) ? wr[j] * t1[(j * TX + xl) * KP + k] : 0.f;
      }
    }
    dlogits[((long)b * h * w + (long)(y0 + yl) * w + x0 + xl) * K + k] = from_f32<T>(acc);
  }
}

}  // namespace

// tiled forward (loss partials only); part: (B * tiles) x 2 floats
int ce_fwd_tiled_nblk(int B, int H, int W) { return B * ((H + FT - 1) / FT) * ((W + FT - 1) / FT); }

// the tiles are sized for the decoder's exact x4 upsampling (MLPDecoder output at 1/4 res)
bool ce_tiled_ok(int h, int w, int H, int W, int K) { return K > 0 && K <= KF && H == 4 * h && W == 4 * w; }

int ce_fwd_tiled_launch(const void* logits, const int64_t* label, float* part, int B, int h, int w, int H, int W,
                        int K, int ignore, int dtype, hipStream_t s) {
  const int tx = (W + FT - 1) / FT, ty = (H + FT - 1) / FT;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(ce_fwd_tiled<T>, dim3(B * tx * ty), dim3(256), 0, s, (const T*)logits, label, part, h, w, H, W,
                       K, ignore, tx, ty);
  });
  return CMX_OK;
}

extern "C" {

// dlogits (B, h, w, K) = bilinear-adjoint of (softmax - onehot) * dloss[0] * stats[1], with
// stats = cmx_upsample_ce_fwd's out ([loss, 1/n_valid, n_valid]).  H = 4h, W = 4w, K <= 40
// (every CMX dataset); otherwise use the grad output of cmx_upsample_ce_fwd and
// cmx_bilinear_adjoint_1d.
int cmx_upsample_ce_bwd(const void* logits, const int64_t* label, const float* dloss, const float* stats,
                        void* dlogits, int B, int h, int w, int H, int W, int K, int ignore_index, int dtype,
                        hipStream_t s) {
  CMX_REQUIRE(B > 0 && ce_tiled_ok(h, w, H, W, K), CMX_ERR_SHAPE,
              "upsample_ce_bwd: needs K <= %d and an exact x4 upsampling (K=%d, %dx%d -> %dx%d)", KF, K, h, w, H, W);
  const int tx = (w + TX - 1) / TX, ty = (h + TY - 1) / TY;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(ce_bwd_fused<T>, dim3(B * tx * ty), dim3(CE_BWD_NT), 0, s, (const T*)logits, label, dloss, stats,
                       (T*)dlogits, h, w, H, W, K, ignore_index, tx, ty);
  });
  return cmx_check_launch("upsample_ce_bwd");
}

}  // extern "C"

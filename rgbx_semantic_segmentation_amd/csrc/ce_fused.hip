// Final upsample + CrossEntropyLoss, tiled through LDS (forward loss and fused backward).
//
// Same math as upsample_ce.hip (builder.py:233,249; train.py:72-73: bilinear x4 upsample,
// align_corners=False, then mean CE over pixels != ignore_index), re-tiled so that neither
// the full-resolution logits NOR their gradient ever reach HBM:
//  * forward: a block owns a 16 x 16 full-res tile, stages the low-res logits it reads
//    (<= 6 x 6 x K, fp32) in LDS once, and each thread does one pixel's interpolation +
//    log-softmax + NLL.  Only per-block loss / count partials are written.
//  * gradient (ce_cells): a block owns a CT_Y x CT_X low-res tile of dlogits and recomputes
//    the softmax gradient of every full-res pixel whose bilinear footprint touches it, a run
//    of 4 pixels per thread that share their two low-res columns, then applies the separable
//    bilinear adjoint (x in registers, y through LDS) and writes the tile once.  In training
//    the forward runs it (with the loss partials) and the backward only scales its fp32
//    result by dloss / n_valid; cmx_upsample_ce_bwd is the recompute-in-backward form.  The
//    2-pass adjoint of a materialised (B, H, W, K) gradient (49 MB at 480 x 640, K = 40) is gone.
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

// ------------------------------------------------------------------------ cells (gradient)
// Exact x4, align_corners=False: full-res X = 4x + r interpolates low-res columns (x - 1, x) for
// r = 0, 1 and (x, x + 1) for r = 2, 3, so the run X in [4c - 2, 4c + 2) reads columns c - 1 and
// c only (at the image borders the clamped taps put all weight on one of them) -- and, by the
// same weights, the adjoint of the x-interpolation sends the run's gradient to those two columns
// only.  A thread takes one such run of 4 pixels on one full-res row: 4 LDS reads per class give
// the run's two row-interpolated columns (registers, log2 units), from which the 4 pixels'
// logits, softmax and gradient follow; the softmax is shifted by the larger of the two columns'
// maxima (every pixel's logit is a convex combination of the two: an upper bound, no max pass),
// and the run's x-adjoint is its two column sums.  A workgroup owns a CT_Y x CT_X low-res tile
// of the output: the runs of full-res rows [4 y0 - 2, 4 y0 + 4 CT_Y + 2) and cells
// c = x0 .. x0 + CT_X (recompute (CT_X + 1) / CT_X x (CT_Y + 1) / CT_Y of the tile's own pixels);
// the column sums meet in LDS (the right column's first, the left column's added after a
// barrier: one fixed summation order), and the y-adjoint (8 full-res rows per low-res row)
// writes the tile.
//   FWD = true:  loss partials of the pixels the tile owns, and the unscaled adjoint of
//                (softmax - onehot) in fp32 (the backward only scales it: cmx_upsample_ce_bwd_scale)
//   FWD = false: the adjoint of (softmax - onehot) * dloss[0] * stats[1] in T (recompute backward)
constexpr int CT_Y = 6, CT_X = 8;
constexpr int CT_R = 4 * CT_Y + 4;                // full-res footprint rows
constexpr int CT_C = CT_X + 1;                    // runs per footprint row
constexpr int CT_NT = 256;
static_assert(CT_R * CT_C <= CT_NT, "one run per thread");
constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.69314718055994531f;

template <typename T, bool FWD>
__global__ __launch_bounds__(CT_NT) void ce_cells(const T* __restrict__ logits, const int64_t* __restrict__ label,
                                                  const float* __restrict__ dloss, const float* __restrict__ stats,
                                                  void* __restrict__ dst, float* __restrict__ part, int h, int w, int H,
                                                  int W, int K, int ignore, int tiles_x, int tiles_y) {
  constexpr int LH = CT_Y + 2, LW = CT_X + 2, LP = LH * LW;   // low-res tile + 1-pixel halo
  constexpr int KP = KF + 1;                                   // odd pitch of the column sums
  __shared__ float lg[KF * LP];                                // class-major [k][row][col]
  __shared__ float t1[CT_R * CT_X * KP + KP];                  // x-adjoint [row][col][k] + a spare row
  __shared__ float wtab[CT_Y][8];                              // y-adjoint weights
  __shared__ float red[2][CT_NT / 64];
  const int t = threadIdx.x;
  const int bx = blockIdx.x % tiles_x, by = (blockIdx.x / tiles_x) % tiles_y, b = blockIdx.x / (tiles_x * tiles_y);
  const int y0 = by * CT_Y, x0 = bx * CT_X;
  const int ny = min(CT_Y, h - y0), nx = min(CT_X, w - x0);
  const float sh = (float)h / H, sw = (float)w / W;
  const int ri = t / CT_C, c = t % CT_C;          // the thread's run: footprint row, cell
  const bool act = ri < CT_R;
  const int Y = 4 * y0 - 2 + ri, X0 = 4 * (x0 + c) - 2;
  const bool rowin = act && Y >= 0 && Y < H;
  // global loads first: the run's labels, the thread's share of the logits tile -- all of them
  // unconditional (an out-of-range element reads the tile's first one and is replaced by a
  // select), so they are in flight together: a load under `cond ? load : 0` was sunk into its
  // branch and waited for there, 4 + NL round trips one after another
  long lab[4];
  bool labok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int X = X0 + j;
    labok[j] = rowin && X >= 0 && X < W;
    lab[j] = label[labok[j] ? ((long)b * H + Y) * W + X : (long)b * H * W];
  }
  const T* base = logits + (long)b * h * w * K;
  constexpr int NL = (LP * KF + CT_NT - 1) / CT_NT;
  float v[NL];
  bool vok[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = t + i * CT_NT;
    const int k = e % K, px = e / K;                // coalesced along k
    const int yy = y0 - 1 + px / LW, xx = x0 - 1 + px % LW;
    vok[i] = e < LP * K && yy >= 0 && yy < h && xx >= 0 && xx < w;
    v[i] = to_f32(base[vok[i] ? ((long)yy * w + xx) * K + k : 0]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) lab[j] = labok[j] ? lab[j] : -1L;
#pragma unroll
  for (int i = 0; i < NL; ++i) v[i] = vok[i] ? v[i] : 0.f;
  if (t < CT_Y * 8) {                             // low-res row y0 + yl from footprint row 4 yl + jj
    const int yl = t >> 3, r = 4 * yl + (t & 7);
    int ya, yb;
    float wa, wb;
    src_idx(4 * y0 - 2 + r, sh, h, ya, yb, wa, wb);
    wtab[yl][t & 7] = (4 * y0 - 2 + r >= 0 && 4 * y0 - 2 + r < H)
                          ? (ya == y0 + yl ? wa : 0.f) + (yb == y0 + yl ? wb : 0.f) : 0.f;
  }
  int ya, yb;
  float wya, wyb;
  src_idx(Y, sh, h, ya, yb, wya, wyb);            // rows outside the image: no valid pixel uses them
  // the 4 pixels' weights on the run's columns x0 + c - 1 (tile column c) and x0 + c (c + 1);
  // lv = the label of a valid pixel, -1 otherwise
  const int xl = x0 + c - 1, xr = x0 + c;
  float cl[4], cr[4];
  int lv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int i0, i1;
    float l0, l1;
    src_idx(X0 + j, sw, w, i0, i1, l0, l1);
    cl[j] = (i0 == xl ? l0 : 0.f) + (i1 == xl ? l1 : 0.f);
    cr[j] = (i0 == xr ? l0 : 0.f) + (i1 == xr ? l1 : 0.f);
    lv[j] = (lab[j] >= 0 && lab[j] < K && lab[j] != ignore) ? (int)lab[j] : -1;
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = t + i * CT_NT;
    if (e < LP * K) lg[(e % K) * LP + e / K] = v[i];
  }
  // classes K .. KF - 1: a very negative logit (exp2 -> 0, maxima unchanged), so the class loops
  // below run KF iterations without a test on K (a runtime test became a branch per class)
  for (int e = t; e < (KF - K) * LP; e += CT_NT) lg[K * LP + e] = -1e30f;
  __syncthreads();
  // pass 1: the run's two row-interpolated columns per class (registers, log2 units), the bound
  const float* la = lg + (min(max(ya - y0 + 1, 0), LH - 1)) * LW + c;
  const float* lb = lg + (min(max(yb - y0 + 1, 0), LH - 1)) * LW + c;
  const float wa2 = wya * LOG2E, wb2 = wyb * LOG2E;
  float ml[KF], mr[KF];
  float M = -INFINITY;
#pragma unroll
  for (int k = 0; k < KF; ++k) {
    ml[k] = __builtin_fmaf(wa2, la[k * LP], wb2 * lb[k * LP]);
    mr[k] = __builtin_fmaf(wa2, la[k * LP + 1], wb2 * lb[k * LP + 1]);
    M = fmaxf(M, fmaxf(ml[k], mr[k]));
  }
  // pass 2: the softmax denominators (pixels outside the image: shift 0, unused)
  float shv[4], sv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    shv[j] = (cl[j] + cr[j]) * M;
    sv[j] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < KF; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      sv[j] += __builtin_amdgcn_exp2f(__builtin_fmaf(cl[j], ml[k], __builtin_fmaf(cr[j], mr[k], -shv[j])));
  // a pixel whose own maximum lies more than ~100 binary orders below the bound (logits far apart
  // between neighbouring low-res pixels) underflowed: redo it with its own maximum
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (lv[j] >= 0 && !(sv[j] >= 0x1p-100f)) {
      float m = -INFINITY;
#pragma unroll
      for (int k = 0; k < KF; ++k) m = fmaxf(m, __builtin_fmaf(cl[j], ml[k], cr[j] * mr[k]));
      shv[j] = m;
      sv[j] = 0.f;
#pragma unroll
      for (int k = 0; k < KF; ++k)
        sv[j] += __builtin_amdgcn_exp2f(__builtin_fmaf(cl[j], ml[k], __builtin_fmaf(cr[j], mr[k], -m)));
    }
  const float gs = FWD ? 1.f : dloss[0] * stats[1];
  float al[4], ar[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float inv = lv[j] >= 0 ? gs / sv[j] : 0.f;
    al[j] = cl[j] * inv;
    ar[j] = cr[j] * inv;
  }
  if constexpr (FWD) {
    // loss of the valid pixels this tile owns (full-res [4 y0, 4 y0 + 4 CT_Y) x [4 x0, 4 x0 + 4 CT_X))
    float ls = 0.f, lc = 0.f;
    const bool rown = Y >= 4 * y0 && Y < 4 * (y0 + CT_Y);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int X = X0 + j;
      if (lv[j] >= 0 && rown && X >= 4 * x0 && X < 4 * (x0 + CT_X)) {
        const int q = lv[j] * LP;
        const float zl = __builtin_fmaf(cl[j], __builtin_fmaf(wa2, la[q], wb2 * lb[q]),
                                        cr[j] * __builtin_fmaf(wa2, la[q + 1], wb2 * lb[q + 1]));
        ls += (shv[j] + __builtin_amdgcn_logf(sv[j]) - zl) * LN2;
        lc += 1.f;
      }
    }
    ls = wave_sum(ls);
    lc = wave_sum(lc);
    if ((t & 63) == 0) {
      red[0][t >> 6] = ls;
      red[1][t >> 6] = lc;
    }
  }
  // pass 3: the gradient's x-adjoint, the run's two column sums; the right column's go to LDS at
  // once (lanes with nothing to write write the spare row: no per-class branch), the left
  // column's wait in registers for the barrier; then the -onehot terms at the pixels' classes
  float* trow = t1 + (act ? ri : 0) * CT_X * KP;
  float* wrow = (act && c < CT_X) ? trow + c * KP : t1 + CT_R * CT_X * KP;
  float sl[KF];
#pragma unroll
  for (int k = 0; k < KF; ++k) {
    float gl = 0.f, gr = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(cl[j], ml[k], __builtin_fmaf(cr[j], mr[k], -shv[j])));
      gl = __builtin_fmaf(al[j], e, gl);
      gr = __builtin_fmaf(ar[j], e, gr);
    }
    wrow[k] = gr;                                 // classes >= K: 0, never read
    sl[k] = gl;
  }
  if (act && c < CT_X)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lv[j] >= 0) trow[c * KP + lv[j]] -= cr[j] * gs;
  __syncthreads();
  if (act && c >= 1) {
#pragma unroll
    for (int k = 0; k < KF; ++k) trow[(c - 1) * KP + k] += sl[k];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lv[j] >= 0) trow[(c - 1) * KP + lv[j]] -= cl[j] * gs;
  }
  __syncthreads();
  if constexpr (FWD) {
    if (t == 0) {
      float a = 0.f, n = 0.f;
#pragma unroll
      for (int i = 0; i < CT_NT / 64; ++i) {
        a += red[0][i];
        n += red[1][i];
      }
      part[blockIdx.x * 2] = a;
      part[blockIdx.x * 2 + 1] = n;
    }
  }
  // y-adjoint: low-res row y takes full-res rows [4y - 2, 4y + 6) = footprint rows [4 yl, 4 yl + 8)
  for (int e = t; e < CT_Y * CT_X * KF; e += CT_NT) {
    const int k = e % KF, xq = (e / KF) % CT_X, yl = e / (KF * CT_X);
    if (k >= K || xq >= nx || yl >= ny) continue;
    const float* tc = t1 + (4 * yl * CT_X + xq) * KP + k;
    float acc = 0.f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc = __builtin_fmaf(wtab[yl][jj], tc[jj * CT_X * KP], acc);
    const long o = ((long)b * h * w + (long)(y0 + yl) * w + x0 + xq) * K + k;
    if constexpr (FWD) reinterpret_cast<float*>(dst)[o] = acc;
    else reinterpret_cast<T*>(dst)[o] = from_f32<T>(acc);
  }
}

// dlogits = adj * dloss[0] * stats[1]
template <typename T>
__global__ void ce_scale_kernel(const float* __restrict__ adj, const float* __restrict__ dloss,
                                const float* __restrict__ stats, T* __restrict__ dl, long n) {
  const float gs = dloss[0] * stats[1];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dl[i] = from_f32<T>(adj[i] * gs);
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

int ce_cells_nblk(int B, int h, int w) { return B * ((h + CT_Y - 1) / CT_Y) * ((w + CT_X - 1) / CT_X); }

// loss partials (part: ce_cells_nblk x 2 floats) and adj (B, h, w, K) fp32 = bilinear adjoint of
// (softmax - onehot), unscaled; exact x4, K <= 40
int ce_cells_fwd_launch(const void* logits, const int64_t* label, float* adj, float* part, int B, int h, int w, int H,
                        int W, int K, int ignore, int dtype, hipStream_t s) {
  const int tx = (w + CT_X - 1) / CT_X, ty = (h + CT_Y - 1) / CT_Y;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((ce_cells<T, true>), dim3(B * tx * ty), dim3(CT_NT), 0, s, (const T*)logits, label, nullptr,
                       nullptr, (void*)adj, part, h, w, H, W, K, ignore, tx, ty);
  });
  return cmx_check_launch("ce_cells_fwd");
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
  const int tx = (w + CT_X - 1) / CT_X, ty = (h + CT_Y - 1) / CT_Y;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((ce_cells<T, false>), dim3(B * tx * ty), dim3(CT_NT), 0, s, (const T*)logits, label, dloss,
                       stats, dlogits, nullptr, h, w, H, W, K, ignore_index, tx, ty);
  });
  return cmx_check_launch("upsample_ce_bwd");
}

// the backward of cmx_upsample_ce_fwd_adj: dlogits = adj * dloss[0] * stats[1] (n elements)
int cmx_upsample_ce_bwd_scale(const float* adj, const float* dloss, const float* stats, void* dlogits, int64_t n,
                              int dtype, hipStream_t s) {
  CMX_REQUIRE(adj && dloss && stats && dlogits && n >= 0, CMX_ERR_ARG, "upsample_ce_bwd_scale: null operand");
  if (n == 0) return CMX_OK;
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(ce_scale_kernel<T>, dim3(grid), dim3(256), 0, s, adj, dloss, stats, (T*)dlogits, (long)n);
  });
  return cmx_check_launch("upsample_ce_bwd_scale");
}

}  // extern "C"

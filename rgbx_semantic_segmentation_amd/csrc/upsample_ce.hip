// Fused final upsample + per-pixel cross-entropy (training path).
//
// Replaces  F.interpolate(out, size=(H, W), bilinear, align_corners=False)  followed by
// nn.CrossEntropyLoss(reduction='mean', ignore_index=255)  (builder.py:233,249;
// train.py:72-73), without materialising the full-resolution logits: each full-res pixel
// interpolates its K logits from the 4 low-res neighbours (NHWC), computes log-softmax
// and NLL, and writes the un-normalised gradient (softmax - onehot, 0 at ignored pixels).
// A finalize kernel produces loss = sum / n_valid and 1 / n_valid on the device; the
// backward is the separable bilinear adjoint of that gradient scaled by
// grad_output / n_valid (bilinear.hip), so the scaled 1/N never needs a host sync.
#include "cmx_common.h"

namespace {

__device__ __forceinline__ void src_index(int dst, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  float s = (dst + 0.5f) * scale - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

constexpr int KMAX = 64;

template <typename T>
__global__ __launch_bounds__(256) void upsample_ce_kernel(const T* __restrict__ logits, const int64_t* __restrict__ label,
                                                          T* __restrict__ grad, float* __restrict__ part, int B, int h,
                                                          int w, int H, int W, int K, int ignore) {
  __shared__ float red[2][256];
  const float sh = (float)h / H, sw = (float)w / W;
  const long total = (long)B * H * W;
  float lsum = 0.f, lcnt = 0.f;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < (int)total; p += gridDim.x * blockDim.x) {
    const int x = p % W;
    const int y = (p / W) % H;
    const int b = p / (W * H);
    const long lab = label[p];
    T* gp = grad + p * K;
    if (lab == ignore || lab < 0 || lab >= K) {
      for (int k = 0; k < K; ++k) gp[k] = from_f32<T>(0.f);
      continue;
    }
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    src_index(y, sh, h, y0, y1, ly0, ly1);
    src_index(x, sw, w, x0, x1, lx0, lx1);
    const T* base = logits + (long)b * h * w * K;
    const T* pa = base + ((long)y0 * w + x0) * K;
    const T* pb = base + ((long)y0 * w + x1) * K;
    const T* pc = base + ((long)y1 * w + x0) * K;
    const T* pd = base + ((long)y1 * w + x1) * K;
    float z[KMAX];
    float m = -INFINITY;
    for (int k = 0; k < K; ++k) {
      const float v = ly0 * (lx0 * to_f32(pa[k]) + lx1 * to_f32(pb[k])) + ly1 * (lx0 * to_f32(pc[k]) + lx1 * to_f32(pd[k]));
      z[k] = v;
      m = fmaxf(m, v);
    }
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += __expf(z[k] - m);
    const float lse = m + __logf(se);
    lsum += lse - z[lab];
    lcnt += 1.f;
    const float inv = 1.f / se;
    for (int k = 0; k < K; ++k) gp[k] = from_f32<T>(__expf(z[k] - m) * inv - (k == lab ? 1.f : 0.f));
  }
  red[0][threadIdx.x] = lsum;
  red[1][threadIdx.x] = lcnt;
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

// out[0] = loss (sum / count), out[1] = 1 / count, out[2] = count
__global__ void ce_finalize_kernel(const float* __restrict__ part, int nblk, float* __restrict__ out) {
  __shared__ double red[2][256];
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 256) { s += part[2 * i]; c += part[2 * i + 1]; }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { red[0][threadIdx.x] += red[0][threadIdx.x + o]; red[1][threadIdx.x] += red[1][threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double cnt = red[1][0];
    out[0] = cnt > 0 ? (float)(red[0][0] / cnt) : NAN;   // PyTorch: mean over zero valid pixels is NaN
    out[1] = cnt > 0 ? (float)(1.0 / cnt) : 0.f;
    out[2] = (float)cnt;
  }
}

int ce_nblk(long total) {
  long nb = (total + 255) / 256;
  return (int)(nb < 2048 ? (nb ? nb : 1) : 2048);
}
}  // namespace

// ce_fused.hip: LDS-tiled loss-only forward (grad == NULL)
int ce_fwd_tiled_nblk(int B, int H, int W);
bool ce_tiled_ok(int h, int w, int H, int W, int K);
int ce_fwd_tiled_launch(const void* logits, const int64_t* label, float* part, int B, int h, int w, int H, int W,
                        int K, int ignore, int dtype, hipStream_t s);
int ce_cells_nblk(int B, int h, int w);
int ce_cells_fwd_launch(const void* logits, const int64_t* label, float* adj, float* part, int B, int h, int w, int H,
                        int W, int K, int ignore, int dtype, hipStream_t s);

extern "C" {

size_t cmx_upsample_ce_workspace(int B, int H, int W) {
  const long a = ce_nblk((long)B * H * W), b = ce_fwd_tiled_nblk(B, H, W);
  return (size_t)(a > b ? a : b) * 2 * sizeof(float);
}

// logits (B, h, w, K) dtype; label (B, H, W) int64; grad (B, H, W, K) dtype (softmax - onehot);
// out (3) fp32 = [loss, 1/n_valid, n_valid]
int cmx_upsample_ce_fwd(const void* logits, const int64_t* label, void* grad, float* out, float* workspace, int B,
                        int h, int w, int H, int W, int K, int ignore_index, int dtype, hipStream_t s) {
  CMX_REQUIRE(K > 0 && K <= KMAX, CMX_ERR_SHAPE, "upsample_ce: K=%d > %d", K, KMAX);
  if (!grad) {                 // loss only (the backward recomputes the gradient: cmx_upsample_ce_bwd)
    CMX_REQUIRE(ce_tiled_ok(h, w, H, W, K), CMX_ERR_SHAPE, "upsample_ce: loss-only mode needs H = 4h, W = 4w, K <= 40");
    const int nbt = ce_fwd_tiled_nblk(B, H, W);
    const int st = ce_fwd_tiled_launch(logits, label, workspace, B, h, w, H, W, K, ignore_index, dtype, s);
    if (st) return st;
    hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, s, workspace, nbt, out);
    return cmx_check_launch("upsample_ce_fwd");
  }
  const int nb = ce_nblk((long)B * H * W);
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(upsample_ce_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)logits, label, (T*)grad, workspace,
                       B, h, w, H, W, K, ignore_index);
  });
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, s, workspace, nb, out);
  return cmx_check_launch("upsample_ce_fwd");
}

// training form of the x4 path: loss (out, as above) and adj (B, h, w, K) fp32 = bilinear adjoint of
// (softmax - onehot) in one pass; the backward is cmx_upsample_ce_bwd_scale
int cmx_upsample_ce_fwd_adj(const void* logits, const int64_t* label, float* adj, float* out, float* workspace, int B,
                            int h, int w, int H, int W, int K, int ignore_index, int dtype, hipStream_t s) {
  CMX_REQUIRE(B > 0 && adj && ce_tiled_ok(h, w, H, W, K), CMX_ERR_SHAPE,
              "upsample_ce_fwd_adj: needs H = 4h, W = 4w, K <= 40 (K=%d, %dx%d -> %dx%d)", K, h, w, H, W);
  const int nb = ce_cells_nblk(B, h, w);
  const int st = ce_cells_fwd_launch(logits, label, adj, workspace, B, h, w, H, W, K, ignore_index, dtype, s);
  if (st) return st;
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, s, workspace, nb, out);
  return cmx_check_launch("upsample_ce_fwd_adj");
}

}  // extern "C"

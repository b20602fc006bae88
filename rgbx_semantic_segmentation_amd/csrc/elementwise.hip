// Vectorised elementwise + column-reduction kernels (HBM-bound; 16 B per lane per access).
//
//  * residual add with per-sample DropPath scale  (Block.forward, dual_segformer.py:176-180:
//    x + drop_path(f(x)), timm DropPath = per-sample keep/keep_prob scaling)
//  * activations (ReLU of CrossPath.channel_proj*, net_utils.py:273-274)
//  * column sums for bias gradients of every Linear / 1x1 conv on the path
//  * fp32 -> bf16 cast for weight shadows
#include "cmx_common.h"

template <typename T>
__global__ void residual_add_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                    const float* __restrict__ scale, T* out, long n_per_sample,
                                    long nvec) {
  constexpr int V = VecT<T>::N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    const int e = i * V;
    const float s = scale ? scale[e / n_per_sample] : 1.f;
    float a[V], b[V];
    load_vec<T>(x + e, a);
    load_vec<T>(y + e, b);
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] += s * b[j];
    store_vec<T>(out + e, a);
  }
}

template <typename T>
__global__ void scale_samples_kernel(const T* __restrict__ x, const float* __restrict__ scale, T* out,
                                     long n_per_sample, long nvec) {
  constexpr int V = VecT<T>::N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    const int e = i * V;
    const float s = scale[e / n_per_sample];
    float a[V];
    load_vec<T>(x + e, a);
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] *= s;
    store_vec<T>(out + e, a);
  }
}

template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long nvec, int act) {
  constexpr int V = VecT<T>::N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    float a[V];
    load_vec<T>(x + i * V, a);
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] = act_fwd(a[j], act);
    store_vec<T>(y + i * V, a);
  }
}

// dx = dy * act'(z); for ReLU, z may be the post-activation output (same sign pattern).
template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ z, T* __restrict__ dx,
                               long nvec, int act) {
  constexpr int V = VecT<T>::N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nvec; i += gridDim.x * blockDim.x) {
    float a[V], b[V];
    load_vec<T>(dy + i * V, a);
    load_vec<T>(z + i * V, b);
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] *= act_grad(b[j], act);
    store_vec<T>(dx + i * V, a);
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst, long n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)n; i += gridDim.x * blockDim.x)
    dst[i] = from_f32<bf16>(src[i]);
}

template <typename S>
__global__ void cast_f32_h16_kernel(const float* __restrict__ src, S* __restrict__ dst, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = from_f32<S>(src[i]);
}

// Column sums of x (G, M, N) -> ws partials (G, nblk, N).  TPR lanes span a column tile of
// TPR*V columns (blockIdx.z), 256/TPR row slots stride over rows.
template <typename T, int TPR>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x, float* __restrict__ ws,
                                                     long M, int N, long ld) {
  constexpr int V = VecT<T>::N;
  constexpr int RS = 256 / TPR;
  __shared__ float red[RS][TPR * V];
  const int g = blockIdx.y;
  const int lane = threadIdx.x % TPR, slot = threadIdx.x / TPR;
  const int col = (blockIdx.z * TPR + lane) * V;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  if (col < N) {
    const T* base = x + (long)g * M * ld + col;
    for (long m = (long)blockIdx.x * RS + slot; m < M; m += (long)gridDim.x * RS) {
      float v[V];
      load_vec<T>(base + m * ld, v);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[slot][lane * V + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < TPR * V; c += 256) {
    float s = 0.f;
    for (int r = 0; r < RS; ++r) s += red[r][c];
    const int gc = blockIdx.z * TPR * V + c;
    if (gc < N) ws[((long)g * gridDim.x + blockIdx.x) * N + gc] = s;
  }
}

// scalar fallback for widths that are not a multiple of the vector width
template <typename T>
__global__ void colsum_scalar_kernel(const T* __restrict__ x, float* __restrict__ ws, long M, int N, long ld) {
  const int g = blockIdx.y;
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    float acc = 0.f;
    const T* base = x + (long)g * M * ld + c;
    for (long m = blockIdx.x; m < M; m += gridDim.x) acc += to_f32(base[m * ld]);
    ws[((long)g * gridDim.x + blockIdx.x) * N + c] = acc;
  }
}

__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ src, float* __restrict__ dst, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8];
    load_vec<bf16>(src + i * 8, v);
    reinterpret_cast<float4*>(dst + i * 8)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(dst + i * 8)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

static unsigned ew_grid(long nvec) {
  long b = (nvec + 255) / 256;
  return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

static int colsum_nblk(long M) {
  long nb = (M + 63) / 64;
  return (int)(nb < 256 ? nb : 256);
}

// ---------------------------------------------------------------- per-step stochastic masks
// One launch draws every random mask of a training step (builder._stochastic):
//   DropPath (timm drop_path, dual_segformer.py:141-180): dp[i] = floor(keep[i] + u) / keep[i]
//   Dropout2d (MLPDecoder.py:63, per sample and channel): d2[i] = (u >= p) / (1 - p)
// and bumps the BN num_batches_tracked counter (BatchNorm2d.forward in train mode).  u is a
// counter-based uniform draw: splitmix64 of (seed, step, element), the step counter kept on
// the device, so a HIP-graph replay draws fresh masks with no host involvement.  One block:
// every thread reads the step before thread 0 advances it.
__device__ __forceinline__ float u01(unsigned long long seed, unsigned long long step, unsigned long long i) {
  unsigned long long z = seed ^ (step * 0x9E3779B97F4A7C15ull) ^ (i * 0xD1B54A32D192ED03ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.f / 16777216.f);   // 24 random bits -> [0, 1)
}

__global__ __launch_bounds__(256) void step_masks_kernel(const float* __restrict__ keep, int nkeep,
                                                         float* __restrict__ dp, int nd2, float p,
                                                         float* __restrict__ d2, unsigned long long seed,
                                                         unsigned long long* __restrict__ step,
                                                         long long* __restrict__ nbt, int nnbt) {
  const unsigned long long st = *step;
  for (int i = threadIdx.x; i < nkeep; i += blockDim.x) {
    const float k = keep[i];
    dp[i] = floorf(k + u01(seed, st, (unsigned long long)i)) / k;
  }
  for (int i = threadIdx.x; i < nd2; i += blockDim.x)
    d2[i] = u01(seed ^ 0x5851F42D4C957F2Dull, st, (unsigned long long)i) >= p ? 1.f / (1.f - p) : 0.f;
  for (int i = threadIdx.x; i < nnbt; i += blockDim.x) nbt[i] += 1;   // one counter per BatchNorm
  __syncthreads();
  if (threadIdx.x == 0) *step = st + 1;
}

extern "C" {

int cmx_residual_add(const void* x, const void* y, const float* scale, void* out, long n_per_sample,
                     long n, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(n % V == 0 && (!scale || n_per_sample % V == 0), CMX_ERR_SHAPE,
              "residual_add: sizes must be multiples of %d", V);
  if (n == 0) return CMX_OK;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(residual_add_kernel<T>, dim3(ew_grid(n / V)), dim3(256), 0, s, (const T*)x,
                       (const T*)y, scale, (T*)out, n_per_sample, n / V);
  });
  return cmx_check_launch("residual_add");
}

int cmx_scale_samples(const void* x, const float* scale, void* out, long n_per_sample, long n, int dtype,
                      hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(n % V == 0 && n_per_sample % V == 0, CMX_ERR_SHAPE, "scale_samples: sizes");
  if (n == 0) return CMX_OK;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(scale_samples_kernel<T>, dim3(ew_grid(n / V)), dim3(256), 0, s, (const T*)x,
                       scale, (T*)out, n_per_sample, n / V);
  });
  return cmx_check_launch("scale_samples");
}

int cmx_act_fwd(const void* x, void* y, long n, int act, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(n % V == 0, CMX_ERR_SHAPE, "act_fwd: n %% %d", V);
  if (n == 0) return CMX_OK;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(act_fwd_kernel<T>, dim3(ew_grid(n / V)), dim3(256), 0, s, (const T*)x, (T*)y,
                       n / V, act);
  });
  return cmx_check_launch("act_fwd");
}

int cmx_act_bwd(const void* dy, const void* z, void* dx, long n, int act, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(n % V == 0, CMX_ERR_SHAPE, "act_bwd: n %% %d", V);
  if (n == 0) return CMX_OK;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(ew_grid(n / V)), dim3(256), 0, s, (const T*)dy,
                       (const T*)z, (T*)dx, n / V, act);
  });
  return cmx_check_launch("act_bwd");
}

int cmx_cast_f32_bf16(const float* src, void* dst, long n, hipStream_t s) {
  if (n == 0) return CMX_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(ew_grid(n)), dim3(256), 0, s, src, (bf16*)dst, n);
  return cmx_check_launch("cast_f32_bf16");
}

// fp32 -> bf16 (dtype 1) / fp16 (dtype 2), round to nearest even: the weight shadow refresh
int cmx_cast_f32_h16(const float* src, void* dst, long n, int dtype, hipStream_t s) {
  CMX_REQUIRE(dtype == 1 || dtype == 2, CMX_ERR_DTYPE, "cast_f32_h16: dtype %d", dtype);
  if (n == 0) return CMX_OK;
  if (dtype == 2) hipLaunchKernelGGL(cast_f32_h16_kernel<f16>, dim3(ew_grid(n)), dim3(256), 0, s, src, (f16*)dst, n);
  else hipLaunchKernelGGL(cast_f32_h16_kernel<bf16>, dim3(ew_grid(n)), dim3(256), 0, s, src, (bf16*)dst, n);
  return cmx_check_launch("cast_f32_h16");
}

int cmx_cast_bf16_f32(const void* src, float* dst, long n, hipStream_t s) {
  CMX_REQUIRE(n % 8 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, CMX_ERR_SHAPE,
              "cast_bf16_f32: n=%ld (n %% 8, 16-B aligned)", n);
  if (n == 0) return CMX_OK;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(ew_grid(n / 8)), dim3(256), 0, s, (const bf16*)src, dst, n / 8);
  return cmx_check_launch("cast_bf16_f32");
}

size_t cmx_colsum_workspace(long M, int G, int N) {
  return (size_t)G * colsum_nblk(M) * N * sizeof(float);
}

// out[g, n] (+)= alpha * sum_m x[g, m, n]; x rows have leading dimension ld (elements).
int cmx_colsum(const void* x, float* out, float* ws, long M, int G, int N, long ld, int accumulate,
               float alpha, int dtype, hipStream_t s) {
  const int V = dtype == 0 ? 4 : 8;
  CMX_REQUIRE(M > 0 && ld >= N, CMX_ERR_SHAPE, "colsum: N=%d ld=%ld", N, ld);
  const int nb = colsum_nblk(M);
  const int chunks = N / V;
  const bool vec = (N % V == 0) && (ld % V == 0);
  CMX_DISPATCH(dtype, T, {
    if (!vec) {
      hipLaunchKernelGGL((colsum_scalar_kernel<T>), dim3(nb, G), dim3(N < 256 ? 64 * ((N + 63) / 64) : 256), 0, s,
                         (const T*)x, ws, M, N, ld);
    } else if (chunks <= 16) {
      hipLaunchKernelGGL((colsum_kernel<T, 16>), dim3(nb, G, 1), dim3(256), 0, s, (const T*)x, ws, M,
                         N, ld);
    } else {
      hipLaunchKernelGGL((colsum_kernel<T, 64>), dim3(nb, G, cdiv(chunks, 64)), dim3(256), 0, s,
                         (const T*)x, ws, M, N, ld);
    }
  });
  int st = cmx_check_launch("colsum");
  if (st) return st;
  return cmx_reduce_partials(ws, out, G, nb, N, accumulate, alpha, s);
}

int cmx_step_masks(const float* keep, int nkeep, float* dp, int nd2, float p, float* d2, uint64_t seed,
                   uint64_t* step, int64_t* nbt, int nnbt, hipStream_t s) {
  CMX_REQUIRE(nkeep >= 0 && nd2 >= 0 && step && (nkeep == 0 || (keep && dp)) && (nd2 == 0 || (d2 && p < 1.f)),
              CMX_ERR_ARG, "step_masks: nkeep=%d nd2=%d p=%f", nkeep, nd2, p);
  hipLaunchKernelGGL(step_masks_kernel, dim3(1), dim3(256), 0, s, keep, nkeep, dp, nd2, p, d2,
                     (unsigned long long)seed, (unsigned long long*)step, (long long*)nbt, nbt ? nnbt : 0);
  return cmx_check_launch("step_masks");
}

}  // extern "C"

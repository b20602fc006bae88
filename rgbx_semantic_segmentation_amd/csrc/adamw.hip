// Fused AdamW over the flat fp32 parameter buffer (one launch for all 66.6 M parameters).
//
// Replaces torch.optim.AdamW(params_list, lr, betas=(0.9, 0.999), weight_decay=0.01)
// with the two param groups of utils/init_func.py:group_weight (decay on Linear/Conv
// weights, none on biases and norm affine params) — train.py:111-115,128-129 — using the
// single-tensor update order of torch.optim.AdamW:
//   p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = b2*v + (1-b2)*g*g
//   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// with torch's scalar precision: the betas arrive as doubles, and 1 - b1, 1 - b2, 1 - lr*wd and
// the bias corrections are formed in double and rounded to fp32 once (as torch rounds its
// Python-float scalars), so 1 - 0.999 is 0.001f and not 1.f - 0.999f (1.3e-5 apart).
// lr and t are read from device memory so the step can be replayed from a HIP graph while
// WarmUpPolyLR changes lr.  The per-64-element flag follows the flat layout (every parameter
// starts on a 64-element boundary): 1 = decay, 0 = none, 2 = in neither of group_weight's groups
// (IFRM's lambdas, which the reference's optimizer never sees): left untouched.  Optionally emits the bf16 weight shadow for
// the next step's GEMMs and scales the gradient (1/world_size after a SUM all-reduce).
// HBM-bound: 16 B read (p,g,m,v) + 12 B written (p,m,v) [+2 B shadow] per parameter.
// The step count is read at every block's start as t_prev and used as t = t_prev + 1; the LAST
// block to finish (arrival ticket) stores t, after every block has read t_prev -- the increment
// needs no launch of its own.  The tickets live in caller-owned memory (cmx_adamw_tickets()
// zeroed uint32s per optimizer; the last block resets them), so launches of different optimizers may
// overlap; NULL takes the library's device-global set (one such launch in flight per device).
#include "cmx_common.h"

// step-count tickets: a block takes a ticket of its group of ADAMW_GRP consecutive blocks; the
// last of a group takes one of the top-level ticket; the last of those stores t.  One counter
// for 65 K blocks serialised 65 K atomics on one address (770 us per launch); spread over 1024
// group counters they overlap (no more than 64 arrivals per address).
constexpr int ADAMW_GRP = 64;
constexpr int ADAMW_NGRP = 4096;
__device__ unsigned int g_adamw_ticket = 0;
__device__ unsigned int g_adamw_grp_ticket[ADAMW_NGRP];

// NT = nontemporal (streaming) loads and stores: every byte is touched once per step
typedef float adamw_f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* a) {
  if constexpr (NT) {
    const adamw_f4 t = __builtin_nontemporal_load(reinterpret_cast<const adamw_f4*>(a));
    return make_float4(t.x, t.y, t.z, t.w);
  } else {
    return *reinterpret_cast<const float4*>(a);
  }
}
template <bool NT>
__device__ __forceinline__ void st4(float* a, float x, float y, float z, float w) {
  if constexpr (NT) __builtin_nontemporal_store((adamw_f4){x, y, z, w}, reinterpret_cast<adamw_f4*>(a));
  else *reinterpret_cast<float4*>(a) = make_float4(x, y, z, w);
}

// S = the weight shadow's 16-bit type (bf16 or f16, the compute dtype's GEMM operand)
// the step's scalars (bias corrections from the device step count, the decay factor, the unscale):
// the same fp64 expressions for every lane of the launch
struct AdamwScalars {
  float step_size, bc2s, decf, gscale;
  double t;
};
__device__ __forceinline__ AdamwScalars adamw_scalars(const float* lr_ptr, const float* step_ptr, double b1d,
                                                      double b2d, double wd, float gscale, const float* loss_scale) {
  AdamwScalars a;
  const double lr = *lr_ptr;
  a.t = (double)*step_ptr + 1.0;
  a.step_size = (float)(lr / (1.0 - pow(b1d, a.t)));
  a.bc2s = (float)sqrt(1.0 - pow(b2d, a.t));
  a.decf = (float)(1.0 - lr * wd);
  a.gscale = loss_scale ? gscale / *loss_scale : gscale;       // unscale
  return a;
}

// BS: the scalars computed once per workgroup by lane 0 and shared through LDS (two fp64 pow,
// a sqrt and divides per lane were each thread's prologue before its single float4 group)
template <typename S, bool NT = false, bool BS = true>
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, S* __restrict__ shadow, const uint8_t* __restrict__ decay64,
                             long n, const float* __restrict__ lr_ptr, float* __restrict__ step_ptr, double b1d,
                             double b2d, float eps, double wd, float gscale_in, const float* __restrict__ loss_scale,
                             const float* __restrict__ found_inf, int store_step, unsigned* __restrict__ tickets) {
  // GradScaler semantics (train.py:185-198): a step whose gradients held inf / nan is skipped
  if (found_inf && *found_inf != 0.f) return;
  AdamwScalars sc;
  if constexpr (BS) {
    __shared__ AdamwScalars ssc;
    if (threadIdx.x == 0) ssc = adamw_scalars(lr_ptr, step_ptr, b1d, b2d, wd, gscale_in, loss_scale);
    __syncthreads();
    sc = ssc;
  } else {
    sc = adamw_scalars(lr_ptr, step_ptr, b1d, b2d, wd, gscale_in, loss_scale);
  }
  const float step_size = sc.step_size, bc2s = sc.bc2s, decf = sc.decf, gscale = sc.gscale;
  const double t = sc.t;
  const float omb1 = (float)(1.0 - b1d), b2 = (float)b2d, omb2 = (float)(1.0 - b2d);
  const long nv = n / 4;
  auto update = [&](const long e, float4 pp, const float4 gg, float4 mm, float4 vv, const uint8_t flag) {
    if (flag == 2) return;                             // 0: no decay, 1: decay, 2: frozen
    const float dec = flag ? decf : 1.f;
    float pa[4] = {pp.x, pp.y, pp.z, pp.w}, ga[4] = {gg.x, gg.y, gg.z, gg.w};
    float ma[4] = {mm.x, mm.y, mm.z, mm.w}, va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * gscale;
      pa[j] *= dec;
      ma[j] = ma[j] + omb1 * (gj - ma[j]);
      va[j] = va[j] * b2 + omb2 * gj * gj;
      const float denom = sqrtf(va[j]) / bc2s + eps;
      pa[j] = pa[j] - step_size * (ma[j] / denom);
    }
    st4<NT>(p + e, pa[0], pa[1], pa[2], pa[3]);
    st4<NT>(m + e, ma[0], ma[1], ma[2], ma[3]);
    st4<NT>(v + e, va[0], va[1], va[2], va[3]);
    if (shadow) *reinterpret_cast<uint2*>(shadow + e) = make_uint2(pack2<S>(pa[0], pa[1]), pack2<S>(pa[2], pa[3]));
  };
  // two float4 groups per thread per iteration: eight 16-B loads in flight before any update
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < nv; i += 2 * stride) {
    const long e0 = i * 4, e1 = (i + stride) * 4;
    const float4 p0 = ld4<NT>(p + e0), p1 = ld4<NT>(p + e1);
    const float4 g0 = ld4<NT>(g + e0), g1 = ld4<NT>(g + e1);
    const float4 m0 = ld4<NT>(m + e0), m1 = ld4<NT>(m + e1);
    const float4 v0 = ld4<NT>(v + e0), v1 = ld4<NT>(v + e1);
    const uint8_t f0 = decay64[e0 >> 6], f1 = decay64[e1 >> 6];
    update(e0, p0, g0, m0, v0, f0);
    update(e1, p1, g1, m1, v1, f1);
  }
  if (i < nv) {
    const long e = i * 4;
    update(e, ld4<NT>(p + e), ld4<NT>(g + e), ld4<NT>(m + e), ld4<NT>(v + e), decay64[e >> 6]);
  }
  // the step count: the last block to arrive stores t (every block read t_prev at its start);
  // a segment launch that is not the step's last (store_step = 0) leaves it to that one
  if (!store_step) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    // relaxed: every thread of this block consumed t_prev before the barrier above (an
    // acquire / release here would write back and invalidate the L2 once per block)
    const unsigned grp = blockIdx.x / ADAMW_GRP, ngrp = (gridDim.x + ADAMW_GRP - 1) / ADAMW_GRP;
    const unsigned gsize = min((unsigned)ADAMW_GRP, gridDim.x - grp * ADAMW_GRP);
    unsigned* top = tickets ? tickets : &g_adamw_ticket;
    unsigned* gt = (tickets ? tickets + 1 : g_adamw_grp_ticket) + grp;
    const unsigned pg = __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (pg == gsize - 1) {
      __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned prev = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == ngrp - 1) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *step_ptr = (float)t;
      }
    }
  }
}

// found_inf[0] = 1 if any of g[0, n) is inf / nan (left untouched otherwise; reset by the
// loss-scale update).  Benign race: every writer stores the same 1.
// Blocks of 64 elements flagged 2 in flags64 (frozen slots) are skipped.
__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ g, long n,
                                                        const uint8_t* __restrict__ flags64, float* __restrict__ found) {
  int bad = 0;
  const long nv = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x) {
    if (flags64 && flags64[i >> 4] == 2) continue;
    const float4 x = reinterpret_cast<const float4*>(g)[i];
    bad |= (int)!isfinite(x.x) | (int)!isfinite(x.y) | (int)!isfinite(x.z) | (int)!isfinite(x.w);
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) *found = 1.f;
}

// torch.cuda.amp.GradScaler.update(): backoff on overflow, grow after `interval` clean steps
__global__ void loss_scale_update_kernel(float* scale, int* tracker, float* found, float growth, float backoff,
                                         int interval) {
  if (*found != 0.f) {
    *scale *= backoff;
    *tracker = 0;
  } else if (++*tracker >= interval) {
    *scale *= growth;
    *tracker = 0;
  }
  *found = 0.f;
}

static int adamw_launch(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype,
                        const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1,
                        double beta2, float eps, double weight_decay, float grad_scale, const float* loss_scale,
                        const float* found_inf, int store_step, int max_blocks, unsigned* tickets, hipStream_t s);

extern "C" {

// n must be a multiple of 64; the step count at step_ptr is incremented by this call and the
// incremented value used (torch order); a step skipped for found_inf leaves it unchanged
size_t cmx_adamw_tickets(void) { return 1 + ADAMW_NGRP; }

int cmx_adamw_step(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype, const uint8_t* decay64,
                   int64_t n, const float* lr_ptr, float* step_ptr, double beta1, double beta2, float eps,
                   double weight_decay, float grad_scale, unsigned* tickets, hipStream_t s) {
  return cmx_adamw_step_scaled(p, g, m, v, shadow, shadow_dtype, decay64, n, lr_ptr, step_ptr, beta1, beta2, eps,
                               weight_decay, grad_scale, nullptr, nullptr, tickets, s);
}

int cmx_adamw_step_scaled(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype,
                          const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1,
                          double beta2, float eps, double weight_decay, float grad_scale, const float* loss_scale,
                          const float* found_inf, unsigned* tickets, hipStream_t s) {
  return adamw_launch(p, g, m, v, shadow, shadow_dtype, decay64, n, lr_ptr, step_ptr, beta1, beta2, eps, weight_decay,
                      grad_scale, loss_scale, found_inf, 1, 0, tickets, s);
}

int cmx_adamw_step_segment(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype,
                           const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1,
                           double beta2, float eps, double weight_decay, float grad_scale, int store_step,
                           int max_blocks, unsigned* tickets, hipStream_t s) {
  return adamw_launch(p, g, m, v, shadow, shadow_dtype, decay64, n, lr_ptr, step_ptr, beta1, beta2, eps, weight_decay,
                      grad_scale, nullptr, nullptr, store_step, max_blocks, tickets, s);
}

}  // extern "C"

static int adamw_launch(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype,
                        const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1,
                        double beta2, float eps, double weight_decay, float grad_scale, const float* loss_scale,
                        const float* found_inf, int store_step, int max_blocks, unsigned* tickets, hipStream_t s) {
  CMX_REQUIRE(n % 64 == 0, CMX_ERR_SHAPE, "adamw: n must be a multiple of 64");
  CMX_REQUIRE(!shadow || shadow_dtype == 1 || shadow_dtype == 2, CMX_ERR_DTYPE, "adamw: shadow dtype %d", shadow_dtype);
  // CMX_ADAMW_BLOCKS caps the grid (A/B knob; each block takes one relaxed ticket, so the
  // cap is a scheduling choice, not a correctness one); max_blocks > 0 caps one launch (a
  // segment update beside the backward on a side stream keeps to a share of the chip)
  static int& cap = cmx_knob("ADAMW_BLOCKS", 0);
  long blocks = (n / 4 + 255) / 256;
  if (cap > 0 && blocks > cap) blocks = cap;
  if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
  CMX_REQUIRE(blocks <= (long)ADAMW_GRP * ADAMW_NGRP, CMX_ERR_SHAPE, "adamw: %ld blocks exceed the ticket groups", blocks);
  // nontemporal p / g / m / v traffic (CMX_ADAMW_NT=0: cached): 375 -> 348 us standalone
  static int& nt = cmx_knob("ADAMW_NT", 1);
  // CMX_ADAMW_BS=0: every lane computes the step's scalars itself (A/B)
  static int& bs = cmx_knob("ADAMW_BS", 1);
#define CMX_ADAMW_(S_, NT_, BS_)                                                                                    \
  hipLaunchKernelGGL((adamw_kernel<S_, NT_, BS_>), dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v,            \
                     (S_*)shadow, decay64, (long)n, lr_ptr, step_ptr, beta1, beta2, eps, weight_decay, grad_scale,   \
                     loss_scale, found_inf, store_step, tickets)
#define CMX_ADAMW(S_, NT_)                     \
  do {                                          \
    if (bs) CMX_ADAMW_(S_, NT_, true);          \
    else CMX_ADAMW_(S_, NT_, false);            \
  } while (0)
  if (shadow_dtype == 2) {
    if (nt) CMX_ADAMW(f16, true);
    else CMX_ADAMW(f16, false);
  } else {
    if (nt) CMX_ADAMW(bf16, true);
    else CMX_ADAMW(bf16, false);
  }
#undef CMX_ADAMW
#undef CMX_ADAMW_
  return cmx_check_launch("adamw_step");
}

extern "C" {

int cmx_grad_nonfinite(const float* g, int64_t n, const uint8_t* flags64, float* found_inf, hipStream_t s) {
  CMX_REQUIRE(n % 4 == 0 && found_inf && (!flags64 || n % 64 == 0), CMX_ERR_SHAPE,
              "grad_nonfinite: n %% 4 (n %% 64 with flags)");
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, (long)n, flags64, found_inf);
  return cmx_check_launch("grad_nonfinite");
}

int cmx_loss_scale_update(float* scale, int* growth_tracker, float* found_inf, float growth_factor,
                          float backoff_factor, int growth_interval, hipStream_t s) {
  hipLaunchKernelGGL(loss_scale_update_kernel, dim3(1), dim3(1), 0, s, scale, growth_tracker, found_inf, growth_factor,
                     backoff_factor, growth_interval);
  return cmx_check_launch("loss_scale_update");
}

}  // extern "C"

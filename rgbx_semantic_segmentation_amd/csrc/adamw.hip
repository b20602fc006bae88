// Fused AdamW over the flat fp32 parameter buffer (one launch for all 66.6 M parameters).
//
// Replaces torch.optim.AdamW(params_list, lr, betas=(0.9, 0.999), weight_decay=0.01)
// with the two param groups of utils/init_func.py:group_weight (decay on Linear/Conv
// weights, none on biases and norm affine params) — train.py:111-115,128-129 — using the
// single-tensor update order of torch.optim.AdamW:
//   p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = b2*v + (1-b2)*g*g
//   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// lr and t are read from device memory so the step can be replayed from a HIP graph while
// WarmUpPolyLR changes lr.  The per-64-element decay flag follows the flat layout (every
// parameter starts on a 64-element boundary).  Optionally emits the bf16 weight shadow for
// the next step's GEMMs and scales the gradient (1/world_size after a SUM all-reduce).
// HBM-bound: 16 B read (p,g,m,v) + 12 B written (p,m,v) [+2 B shadow] per parameter.
#include "cmx_common.h"

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, bf16* __restrict__ shadow, const uint8_t* __restrict__ decay64,
                             long n, const float* __restrict__ lr_ptr, const float* __restrict__ step_ptr, float b1,
                             float b2, float eps, float wd, float gscale) {
  const float lr = *lr_ptr;
  const float t = *step_ptr;
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float step_size = lr / bc1;
  const long nv = n / 4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)nv; i += gridDim.x * blockDim.x) {
    const long e = i * 4;
    float4 pp = *reinterpret_cast<float4*>(p + e);
    float4 gg = *reinterpret_cast<const float4*>(g + e);
    float4 mm = *reinterpret_cast<float4*>(m + e);
    float4 vv = *reinterpret_cast<float4*>(v + e);
    const float dec = decay64[e >> 6] ? 1.f - lr * wd : 1.f;
    float pa[4] = {pp.x, pp.y, pp.z, pp.w}, ga[4] = {gg.x, gg.y, gg.z, gg.w};
    float ma[4] = {mm.x, mm.y, mm.z, mm.w}, va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * gscale;
      pa[j] *= dec;
      ma[j] = ma[j] + (1.f - b1) * (gj - ma[j]);
      va[j] = va[j] * b2 + (1.f - b2) * gj * gj;
      const float denom = sqrtf(va[j]) / bc2s + eps;
      pa[j] = pa[j] - step_size * (ma[j] / denom);
    }
    *reinterpret_cast<float4*>(p + e) = make_float4(pa[0], pa[1], pa[2], pa[3]);
    *reinterpret_cast<float4*>(m + e) = make_float4(ma[0], ma[1], ma[2], ma[3]);
    *reinterpret_cast<float4*>(v + e) = make_float4(va[0], va[1], va[2], va[3]);
    if (shadow) {
      uint32_t a = pack2_bf16(pa[0], pa[1]);
      uint32_t b = pack2_bf16(pa[2], pa[3]);
      *reinterpret_cast<uint2*>(shadow + e) = make_uint2(a, b);
    }
  }
}

__global__ void step_incr_kernel(float* step) { *step += 1.f; }

extern "C" {

// n must be a multiple of 64; step_ptr is incremented by this call before use (torch order)
int cmx_adamw_step(float* p, const float* g, float* m, float* v, void* shadow_bf16, const uint8_t* decay64, int64_t n,
                   const float* lr_ptr, float* step_ptr, float beta1, float beta2, float eps, float weight_decay,
                   float grad_scale, hipStream_t s) {
  CMX_REQUIRE(n % 64 == 0, CMX_ERR_SHAPE, "adamw: n must be a multiple of 64");
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, s, step_ptr);
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, (bf16*)shadow_bf16, decay64,
                     (long)n, lr_ptr, step_ptr, beta1, beta2, eps, weight_decay, grad_scale);
  return cmx_check_launch("adamw_step");
}

}  // extern "C"

// DecoderHead (MLPDecoder.py:8-81) with linear_c{1..4} folded into the linear_fuse 1x1 conv.
// Branch i of the reference is  Wf_i up_i(x_i Wc_i^T + bc_i)  (Wf_i = the conv's column slot of
// that branch, up_1 = identity).  Bilinear upsampling is linear with weights summing to 1, so
//   Z = sum_i up_i(x_i M_i^T) + b,    M_i = Wf_i Wc_i  (E x C_i),    b = bf + sum_i Wf_i bc_i
// and the (B, N_i, E) projections of the reference are never formed.  Backward, with
// dY_i = up_i^T dZ and dM_i = dY_i^T x_i (queued weight-gradient GEMMs) and gb = sum_rows dZ:
//   dWf_i = dM_i Wc_i^T + gb bc_i^T     dWc_i = Wf_i^T dM_i     dbc_i = Wf_i^T gb     dbf = gb
// The GEMMs (composition, branch products, dM_i, the chain rule) run on cmx_gemm /
// cmx_gemm_multi / the grouped launch (functions.DecoderFoldF); the pieces here are the
// non-GEMM terms around them.
#include "cmx_common.h"

namespace {

struct FoldBias {
  const float* bc[4];     // slot order of Wf's columns: c4, c3, c2, c1
  float* dbc[4];
};

// b[k] = bf[k] + sum_j Wf[k, j] bcat[j], one wave per row k; each lane reads 16-byte runs of
// the row (8 x 16-bit or 4 x fp32 elements, inside one slot since E % 8 == 0)
template <typename T>
__global__ void fold_bias_kernel(const T* __restrict__ Wf, long ldw, const float* __restrict__ bf, FoldBias p,
                                 float* __restrict__ b, int E) {
  constexpr int V = VecT<T>::N;
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (k >= E) return;                                   // whole wave
  const T* row = Wf + (long)k * ldw;
  float acc = 0.f;
  for (int j = lane * V; j < 4 * E; j += 64 * V) {
    const int s = j / E, e = j - s * E;
    float w[V];
    load_vec<T>(row + j, w);
    const float* bc = p.bc[s] + e;
#pragma unroll
    for (int i = 0; i < V; ++i) acc += w[i] * bc[i];
  }
  acc = wave_sum(acc);
  if (lane == 0) b[k] = bf[k] + acc;
}

// Three block roles in one grid (256 threads):
//   [0, ncast)             dMh = T(dM), 8 elements per thread and step (skipped when dMh is null)
//   next (4E/64)*(E/64)    one 64 x 64 tile of Wf: WfT = Wf^T through LDS (the A operand of the
//                          dWc GEMMs), dWf = gb bcat^T (overwritten; the dM_i Wc_i^T GEMMs then
//                          accumulate onto it), dbf = gb
//   next 4E/64             dbc[j] = sum_k Wf[k, j] gb[k] for 64 columns j, 4 waves splitting k
template <typename T>
__global__ void fold_prep_kernel(const float* __restrict__ dM, T* __restrict__ dMh, long n8, int ncast,
                                 const float* __restrict__ gb, const T* __restrict__ Wf, long ldw, T* __restrict__ WfT,
                                 float* __restrict__ dWf, long ldg, FoldBias p, float* __restrict__ dbf, int E) {
  __shared__ float tile[64][65];
  __shared__ float red[4][64];
  const int t = threadIdx.x;
  int bid = blockIdx.x;
  if (bid < ncast) {
    if constexpr (is_h16<T>)
    for (long i = (long)bid * 256 + t; i < n8; i += (long)ncast * 256) {
      const float4 a = reinterpret_cast<const float4*>(dM)[2 * i];
      const float4 c = reinterpret_cast<const float4*>(dM)[2 * i + 1];
      const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      store_vec<T>(dMh + 8 * i, v);
    }
    return;
  }
  bid -= ncast;
  const int nj = 4 * E / 64, nk = E / 64;
  const int c = t & 63, w = t >> 6;
  if (bid < nj * nk) {
    const int j0 = (bid % nj) * 64, k0 = (bid / nj) * 64;
    const int slot = j0 / E;
    const float bcv = p.bc[slot][j0 - slot * E + c];
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int r = w + 4 * i;
      tile[r][c] = to_f32(Wf[(long)(k0 + r) * ldw + j0 + c]);
      dWf[(long)(k0 + r) * ldg + j0 + c] = gb[k0 + r] * bcv;
    }
    if (j0 == 0 && t < 64) dbf[k0 + t] = gb[k0 + t];
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int r = w + 4 * i;
      WfT[(long)(j0 + r) * E + k0 + c] = from_f32<T>(tile[c][r]);
    }
    return;
  }
  bid -= nj * nk;
  const int j0 = bid * 64, slot = j0 / E, q = E / 4;
  float acc = 0.f;
#pragma unroll 8
  for (int k = w * q; k < (w + 1) * q; ++k) acc += to_f32(Wf[(long)k * ldw + j0 + c]) * gb[k];
  red[w][c] = acc;
  __syncthreads();
  if (t < 64) p.dbc[slot][j0 - slot * E + t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

}  // namespace

extern "C" {

int cmx_decoder_fold_bias(const void* Wf, int64_t ldw, const float* bf, const float* bc4, const float* bc3,
                          const float* bc2, const float* bc1, float* b, int E, int dtype, hipStream_t s) {
  CMX_REQUIRE(Wf && bf && bc4 && bc3 && bc2 && bc1 && b && E > 0 && E % 8 == 0 && ldw >= 4 * E && ldw % 8 == 0 &&
              (uintptr_t)Wf % 16 == 0, CMX_ERR_ARG, "decoder_fold_bias: E=%d ldw=%ld (multiples of 8, 16-B aligned)",
              E, (long)ldw);
  FoldBias p{{bc4, bc3, bc2, bc1}, {nullptr, nullptr, nullptr, nullptr}};
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(fold_bias_kernel<T>, dim3(cdiv(E, 4)), dim3(256), 0, s, (const T*)Wf, (long)ldw, bf, p, b, E);
  });
  return cmx_check_launch("decoder_fold_bias");
}

int cmx_decoder_fold_bwd_prep(const float* dM, void* dMh, int64_t n, const float* gb, const void* Wf, int64_t ldw,
                              void* WfT, float* dWf, int64_t ldg, const float* bc4, const float* bc3, const float* bc2,
                              const float* bc1, float* dbc4, float* dbc3, float* dbc2, float* dbc1, float* dbf, int E,
                              int dtype, hipStream_t s) {
  CMX_REQUIRE(E > 0 && E % 64 == 0 && ldw >= 4 * E && ldg >= 4 * E && gb && Wf && WfT && dWf && dbf, CMX_ERR_SHAPE,
              "decoder_fold_bwd_prep: E=%d (a multiple of 64) ldw=%ld ldg=%ld", E, (long)ldw, (long)ldg);
  CMX_REQUIRE(bc4 && bc3 && bc2 && bc1 && dbc4 && dbc3 && dbc2 && dbc1, CMX_ERR_ARG, "decoder_fold_bwd_prep: biases");
  CMX_REQUIRE(!dMh || (dM && n % 8 == 0 && (uintptr_t)dM % 16 == 0 && (uintptr_t)dMh % 16 == 0), CMX_ERR_SHAPE,
              "decoder_fold_bwd_prep: cast of n=%ld (n %% 8, 16-B aligned)", (long)n);
  FoldBias p{{bc4, bc3, bc2, bc1}, {dbc4, dbc3, dbc2, dbc1}};
  const long n8 = dMh ? n / 8 : 0;
  const int ncast = n8 ? (int)(cdiv(n8, 256) < 512 ? cdiv(n8, 256) : 512) : 0;
  const int grid = ncast + (4 * E / 64) * (E / 64) + 4 * E / 64;
  CMX_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(fold_prep_kernel<T>, dim3(grid), dim3(256), 0, s, dM, (T*)dMh, n8, ncast, gb, (const T*)Wf,
                       (long)ldw, (T*)WfT, dWf, (long)ldg, p, dbf, E);
  });
  return cmx_check_launch("decoder_fold_bwd_prep");
}

}  // extern "C"

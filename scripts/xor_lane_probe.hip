// Checks cmx_common.h's xor_lane<O> (DPP / v_permlane*_swap lane exchange) against __shfl_xor
// for every offset, and group_sum against the __shfl_xor butterfly bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/xor_lane_probe.hip -o build/xor_lane_probe
//   ./build/xor_lane_probe        (prints "xor_lane ok" and exits 0, or the first mismatch and 1)
#include "../rgbx_semantic_segmentation_amd/csrc/cmx_common.h"
#include <stdio.h>
#include <string.h>

__global__ void probe(const float* in, float* got, float* want) {
  const int t = threadIdx.x, w = blockIdx.x;
  const float v = in[w * 64 + t];
  float* g = got + (long)w * 64 * 12;
  float* r = want + (long)w * 64 * 12;
  g[0 * 64 + t] = xor_lane<1>(v);   r[0 * 64 + t] = __shfl_xor(v, 1, 64);
  g[1 * 64 + t] = xor_lane<2>(v);   r[1 * 64 + t] = __shfl_xor(v, 2, 64);
  g[2 * 64 + t] = xor_lane<4>(v);   r[2 * 64 + t] = __shfl_xor(v, 4, 64);
  g[3 * 64 + t] = xor_lane<8>(v);   r[3 * 64 + t] = __shfl_xor(v, 8, 64);
  g[4 * 64 + t] = xor_lane<16>(v);  r[4 * 64 + t] = __shfl_xor(v, 16, 64);
  g[5 * 64 + t] = xor_lane<32>(v);  r[5 * 64 + t] = __shfl_xor(v, 32, 64);
  for (int q = 0; q < 6; ++q) {
    const int width = 2 << q;
    float s = v;
    for (int o = width >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    g[(6 + q) * 64 + t] = group_sum(v, width);
    r[(6 + q) * 64 + t] = s;
  }
}

int main() {
  const int W = 64, n = W * 64, m = n * 12;
  float* h = (float*)malloc(n * sizeof(float));
  unsigned s = 12345u;
  for (int i = 0; i < n; ++i) {                  // values of mixed magnitude: the add order shows
    s = s * 1664525u + 1013904223u;
    h[i] = ((int)(s >> 8) - (1 << 23)) * (1.f / (1 << 23)) * (float)(1 << ((s >> 3) & 15));
  }
  float *din, *dg, *dr;
  if (hipMalloc(&din, n * 4) || hipMalloc(&dg, m * 4) || hipMalloc(&dr, m * 4)) return 2;
  hipMemcpy(din, h, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(W), dim3(64), 0, 0, din, dg, dr);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  float* g = (float*)malloc(m * 4);
  float* r = (float*)malloc(m * 4);
  hipMemcpy(g, dg, m * 4, hipMemcpyDeviceToHost);
  hipMemcpy(r, dr, m * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < m; ++i)
    if (memcmp(&g[i], &r[i], 4)) {
      const int k = (i / 64) % 12;
      printf("mismatch: %s %d, lane %d: %a vs %a\n", k < 6 ? "xor_lane" : "group_sum", k < 6 ? 1 << k : 2 << (k - 6),
             i % 64, g[i], r[i]);
      return 1;
    }
  printf("xor_lane ok (%d values, offsets 1..32, group_sum widths 2..64)\n", m);
  return 0;
}

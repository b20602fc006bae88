// Probe: does the dirty-L2 writeback at a kernel boundary cost time, and do write-through
// (sc1) stores remove it?  Kernels writing `bytes` with plain or sc1 16-B global stores, a
// reader kernel, and a trivial kernel; timed by the probe script with HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/wt_probe.hip -o scripts/libwt_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void write_plain(uint4* __restrict__ p, long n, uint32_t v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = make_uint4(v, v + 1, v + 2, v + 3);
}

__global__ __launch_bounds__(256) void write_sc1(uint4* __restrict__ p, long n, uint32_t v) {
  // buffer store with cache policy sc1 (CPol::SC1 = 16 on gfx942 / gfx950): write-through
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7ffffff0, 0x00020000);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){v, v + 1, v + 2, v + 3}, r, (int)(i * 16), 0, 16);
}

__global__ __launch_bounds__(256) void write_nt(uint4* __restrict__ p, long n, uint32_t v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
  {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((u32x4){v, v + 1, v + 2, v + 3}, reinterpret_cast<u32x4*>(p + i));
  }
}

__global__ __launch_bounds__(256) void read_sum(const uint4* __restrict__ p, long n, uint32_t* out) {
  uint32_t s = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint4 x = p[i];
    s += x.x ^ x.y ^ x.z ^ x.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

__global__ void tiny(uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] += 1;
}

extern "C" {
int wt_write(int mode, void* p, long bytes, int grid, hipStream_t s) {
  const long n = bytes / 16;
  if (mode == 0) hipLaunchKernelGGL(write_plain, dim3(grid), dim3(256), 0, s, (uint4*)p, n, 7u);
  else if (mode == 1) hipLaunchKernelGGL(write_sc1, dim3(grid), dim3(256), 0, s, (uint4*)p, n, 7u);
  else hipLaunchKernelGGL(write_nt, dim3(grid), dim3(256), 0, s, (uint4*)p, n, 7u);
  return (int)hipGetLastError();
}
int wt_read(const void* p, long bytes, int grid, void* out, hipStream_t s) {
  hipLaunchKernelGGL(read_sum, dim3(grid), dim3(256), 0, s, (const uint4*)p, bytes / 16, (uint32_t*)out);
  return (int)hipGetLastError();
}
int wt_tiny(void* out, hipStream_t s) {
  hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, (uint32_t*)out);
  return (int)hipGetLastError();
}
}

// LDS-DMA helpers shared by the gfx950 kernels that stage tiles HBM -> LDS with
// buffer_load ... lds (no register staging): buffer resource, wave-wide 16-B DMA, counted waits.
#pragma once
#include "cmx_common.h"

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// One LDS-DMA wave-instruction: 64 lanes x 16 B from rsrc + voffset[lane] to LDS bytes
// [lds, lds + 1024) in lane order.  Inline asm on purpose: through the compiler intrinsic,
// hipcc cannot tell the DMA's LDS range from the buffer being read and waits vmcnt(0)
// before every ds_read, which serialises the prefetch with the MFMAs.  The kernel orders
// the DMA itself: `s_waitcnt vmcnt(0)` + barrier before a staged buffer is read.
// The resource is wave-uniform at every call site; readfirstlane pins it to SGPRs even when the
// compiler cannot prove that (e.g. a record loaded through a searched index).
__device__ __forceinline__ void dma16(const i32x4 rsrc, uint32_t lds, int voffset) {
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane(rsrc.x);
  r.y = __builtin_amdgcn_readfirstlane(rsrc.y);
  r.z = __builtin_amdgcn_readfirstlane(rsrc.z);
  r.w = __builtin_amdgcn_readfirstlane(rsrc.w);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voffset), "s"(r) : "memory");   // m0 is reserved: hipcc uses it for nothing else in these kernels
}

constexpr int OOB = (int)0x80000000;            // voffset past num_records -> the load returns 0

__device__ __forceinline__ i32x4 make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);               // stride 0 (raw buffer)
  r.z = 0x7ffffff0;                             // num_records: every in-range offset is < 2^31 - 16
  r.w = 0x00020000;                             // gfx9 data format dword
  return r;
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt[3:0] | [15:14])
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}


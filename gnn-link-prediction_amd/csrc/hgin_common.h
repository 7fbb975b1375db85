// Shared helpers for libhgin.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/hgin.h"

namespace hgin {

constexpr int kWave = 64;  // CDNA wavefront

void set_error(const char* fmt, ...);

// Launch trace (hgin_trace_enable / hgin_trace_read): when on, every dispatch site records which kernel variant
// it launched, so tests can prove which instantiations a call exercised.  Off by default; one relaxed atomic load
// per launch when off.
bool trace_on();
void trace_launch(const char* fmt, ...);
#define HGIN_TRACE(...)                                       \
  do {                                                        \
    if (::hgin::trace_on()) ::hgin::trace_launch(__VA_ARGS__); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Launch bookkeeping: returns 0 or the hipError_t of the launch (after recording a message).
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return HGIN_OK;
}

// Async memset whose status is folded into the call's return value.
inline int memset_async(void* p, int v, size_t bytes, hipStream_t s, const char* what) {
  hipError_t e = hipMemsetAsync(p, v, bytes, s);
  if (e != hipSuccess) {
    set_error("%s: hipMemsetAsync failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return HGIN_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// XCD-aware workgroup order.  gfx950 hands workgroup L of a launch to XCD L % 8, and each XCD has its own
// L2, so workgroups that read the same rows should sit on one XCD.  Over a grid padded to a multiple of 8,
// logical index q = (L % 8) * (total / 8) + L / 8 gives every XCD a contiguous run of logical work items
// (e.g. all output tiles of one row range).  Callers launch round_up8(n) workgroups and return when q >= n.
constexpr int kXcds = 8;
inline int64_t round_up8(int64_t n) { return (n + kXcds - 1) / kXcds * kXcds; }
__device__ __forceinline__ int64_t xcd_logical(int64_t L, int64_t padded_total) {
  return (L % kXcds) * (padded_total / kXcds) + L / kXcds;
}
bool xcd_remap_enabled();   // always on (the round-5 A/B switch is gone)

// bf16 storage (cfg5): raw uint16_t bit patterns; arithmetic is always fp32.
// Widening is exact; narrowing is round-to-nearest-even with NaN -> 0x7FC0, bit-identical to
// torch's float -> bfloat16 conversion (c10::BFloat16), so the CPU oracle can pin every rounding.
__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
// The rounding is gfx950's v_cvt_pk_bf16_f32 (RNE: equal to the integer form (u + 0x7fff + lsb) >> 16 on every
// non-NaN input, tools/bf16_cvt_check.hip over 1M bit patterns incl. denormals, ties and overflow), with NaN lanes
// replaced by 0x7FC0 (the instruction keeps the sign and payload; torch canonicalises).
using f32x2_cvt_t = __attribute__((ext_vector_type(2))) float;
using bf16x2_cvt_t = __attribute__((ext_vector_type(2))) __bf16;
// The NaN fix-up is a real branch taken only by lanes holding a NaN: one v_cmp_u_f32 per pair on the common path
// instead of two compares, two selects and the bit merges (the volatile asm keeps the compiler from flattening it
// into selects) — the bf16 GEMM epilogues and the PReLU-fused dW pack every output element.
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  uint32_t p = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_cvt_t{lo, hi}, bf16x2_cvt_t));
  if (__builtin_expect(__builtin_isunordered(lo, hi), 0)) {
    asm volatile("");
    if (lo != lo) p = (p & 0xffff0000u) | 0x7fc0u;
    if (hi != hi) p = (p & 0x0000ffffu) | 0x7fc00000u;
  }
  return p;
}
__device__ __forceinline__ uint32_t f2bf(float f) { return pack_bf2(f, 0.0f) & 0xffffu; }

// fp32 GEMMs on the bf16 matrix cores ("split" mode of hgin_gemm_nt / hgin_gemm_tn): each fp32 operand
// a = a1 + a2 + a3 with a1 = bf16(a), a2 = bf16(a - a1), a3 = bf16(a - a1 - a2) (RNE; every residual is
// exact in fp32, so a1 + a2 + a3 carries a's full 24-bit significand), and a product ab is formed from the
// six bf16 MFMA terms a1b1, a1b2, a2b1, a1b3, a2b2, a3b1 with fp32 accumulation; the dropped terms are
// below 2^-25 |ab|.  Measured error against fp64 is at or below the exact f32-MFMA kernel's
// (tools/gemm_diag.hip: max 6.0e-7 vs 7.3e-7 of sum |ab| at K = 256) at 16x the matrix rate per term.
// Out-of-range edge: |a| above the largest bf16 (3.39e38) rounds a1 to inf.
// split4: 4 fp32 -> 3 planes of 4 packed bf16.
// Pairs go through one v_cvt_pk_bf16_f32 per plane (the packed pair IS the plane's dword) and are widened
// back with a shift / mask: 5.5 VALU ops per element.
using f32x2_t = __attribute__((ext_vector_type(2))) float;
using bf16x2_t = __attribute__((ext_vector_type(2))) __bf16;
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& p1, uint32_t& p2, uint32_t& p3) {
  p1 = cvt_pk_bf16(x0, x1);
  const float r0 = x0 - bf_lo(p1), r1 = x1 - bf_hi(p1);
  p2 = cvt_pk_bf16(r0, r1);
  const float s0 = r0 - bf_lo(p2), s1 = r1 - bf_hi(p2);
  p3 = cvt_pk_bf16(s0, s1);
}
__device__ __forceinline__ void split4(const float4 v, uint2 (&o)[3]) {
  split2(v.x, v.y, o[0].x, o[1].x, o[2].x);
  split2(v.z, v.w, o[0].y, o[1].y, o[2].y);
}
// LDS row of a split operand: 3 planes x 32 bf16 (one 32-deep K-tile) + 16 B pad = 208 B = 13 x 16 B, so the
// 16 rows of a ds_read_b128 lane group fall on 16 distinct 16-B bank slots (13 is odd).
constexpr int kSplitRowWords = 52;
bool gemm_split_enabled();   // HGIN_F32_GEMM=mfma32 selects the exact f32-MFMA kernels; default split

// LDS-DMA (global_load_lds_dwordx4: 64 lanes x 16 B into 1 KiB at a wave-uniform LDS address) issued from
// inline asm: the compiler does not see it, so it does not guard the kernel's later LDS reads with a vmcnt(0)
// of its own (which would drain a DMA ring); kernels that use it count their vector-memory ops and wait with
// wait_vm<N>() (loads, stores and LDS-DMA retire in issue order for vmcnt).  Used by the weight-stationary
// GEMMs (hgin_gemm_nt.hip k_ws_bf16, hgin_gemm_tn.hip k_wsd_bf16).
template <bool kNt = false>
__device__ __forceinline__ void glds16_asm(const void* g, void* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(lds_wave_base));
  if constexpr (kNt)
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g), "s"(m0) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Element-type traits shared by the fp32 and bf16 instantiations of the memory-bound kernels.
template <typename T>
struct Elem;
template <>
struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <>
struct Elem<uint16_t> {
  static __device__ __forceinline__ float ld(const uint16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(uint16_t* p, float v) { *p = (uint16_t)f2bf(v); }
};

}  // namespace hgin

#define HGIN_ARG_CHECK(cond, ...)     \
  do {                                \
    if (!(cond)) {                    \
      ::hgin::set_error(__VA_ARGS__); \
      return HGIN_E_ARG;              \
    }                                 \
  } while (0)

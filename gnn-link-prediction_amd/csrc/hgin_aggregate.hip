// A3 + A4 — GINConv message + sum aggregate + (1 + eps) self term, fused.
//
// Reference: PyG MessagePassing.propagate at models.py:208 = index_select gather (x_j = x_src[ei[0]],
// an [E, F] tensor written and re-read) + torch_scatter.scatter(..., reduce='sum') (zeros +
// scatter_add_, atomics on the GPU), then models.py:212-215 (cat or +=) as separate kernels.
//
// Here: one pass over a stable CSR (hgin_csr.hip).  A lane group of G lanes owns one destination row;
// each lane holds VEC consecutive features (float4 when the layout allows: 16 B per lane, the row read
// as one contiguous G*16-byte segment), walks the row's neighbours in edge order and accumulates
// sequentially — acc = ((0 + x_1) + x_2) + ...  — exactly CPU scatter_add_'s order, with no FMA
// contraction (explicit __fadd_rn / __fmul_rn), so results are bit-identical to the reference's CPU path.
// U neighbour rows are loaded before any of them is added, keeping U * G * 16 B in flight per group
// while the add order stays sequential.  The self term is applied in the epilogue of the same pass,
// writing straight into the concat layout: no [E, F] messages, no atomics, no cat.
//
// HBM bytes per launch (the roofline model):
//   E * (4 + 4 * F_src) + (N + 1) * 4 + N * 4 * F_out  [+ N * 4 * F_dst when a self term is read]
#include "hgin_common.h"

namespace hgin {
namespace {

// Batched tail: GIN rows are short (uniform random graphs: mean degree 5-10), so with full-batch-then-one-at-a-time
// walking most neighbours of most rows were fetched one dependent round trip at a time.  Batched: every batch of up to
// U = 8 neighbour rows is in flight together (lanes past the row's end issue nothing); the adds stay sequential in edge
// order (bit-identical).  (Round 6: the one-at-a-time tail and U = 16 variants and their switches are gone: measured
// slower or equal, profiles/r01_agg_tail.txt.)
constexpr int kAggU = 8;

// Non-temporal self-term loads / output stores (the streamed-once data) so they do not evict the gathered source
// table from L2 / the Infinity Cache.  Measured: 3-9 % faster for the concat layer at every size
// (profiles/r01_agg_nt.txt); for the other modes 1-2 % slower at cfg2, whose tables fit in the 256 MiB Infinity
// Cache, and 4-5 % faster at cfg3, whose tables do not (aggregate 5.48-5.57 -> 5.77 TB/s, step 212-214 -> 209.6
// ms: profiles/r02/agg_variants_cfg3.txt).  So: concat always, the other modes once the output stream alone
// exceeds 512 MiB (cfg2's largest is 307 MB).
bool agg_nt(int combine, int64_t n_rows, int64_t out_row_bytes) {
  return combine == HGIN_COMBINE_CONCAT || n_rows * out_row_bytes > (int64_t(512) << 20);
}

template <int VEC>
struct Vec;
// NT = true: streamed-once data (the self-term rows and the output) use non-temporal loads / stores so they
// do not evict the gathered source table from L2 / the Infinity Cache.
using f4v = __attribute__((ext_vector_type(4))) float;

template <>
struct Vec<1> {
  using T = float;
  static __device__ __forceinline__ T load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, T v) { *p = v; }
  template <bool NT>
  static __device__ __forceinline__ T load_s(const float* p) { return NT ? __builtin_nontemporal_load(p) : *p; }
  template <bool NT>
  static __device__ __forceinline__ void store_s(float* p, T v) {
    if (NT) __builtin_nontemporal_store(v, p); else *p = v;
  }
  static __device__ __forceinline__ float get(const T& v, int) { return v; }
  static __device__ __forceinline__ void set(T& v, int, float x) { v = x; }
};
template <>
struct Vec<4> {
  using T = float4;
  static __device__ __forceinline__ T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void store(float* p, T v) { *reinterpret_cast<float4*>(p) = v; }
  template <bool NT>
  static __device__ __forceinline__ T load_s(const float* p) {
    if (!NT) return load(p);
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  template <bool NT>
  static __device__ __forceinline__ void store_s(float* p, T v) {
    if (!NT) return store(p, v);
    const f4v t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(p));
  }
  static __device__ __forceinline__ float get(const T& v, int c) {
    return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
  }
  static __device__ __forceinline__ void set(T& v, int c, float x) {
    if (c == 0) v.x = x; else if (c == 1) v.y = x; else if (c == 2) v.z = x; else v.w = x;
  }
};

// The neighbour walk issues every batch's loads together, the last partial batch included (kAggU above).
template <int VEC, int G, int U, bool NT>
__global__ __launch_bounds__(256) void k_aggregate(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                   int64_t n_rows, const float* __restrict__ x_src, int64_t ld_src,
                                                   int f_src, const float* __restrict__ x_dst, int64_t ld_dst,
                                                   int f_dst, const float* __restrict__ eps, int combine,
                                                   float* __restrict__ out, int64_t ld_out) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int kRowsPerWave = kWave / G;
  const int lane = threadIdx.x & (kWave - 1);
  const int grp = lane / G;
  const int gl = lane % G;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  const int64_t r = wave_id * kRowsPerWave + grp;
  if (r >= n_rows) return;
  const int beg = rowptr[r];
  const int end = rowptr[r + 1];
  const float s = combine != HGIN_COMBINE_NONE ? __fadd_rn(1.0f, eps[0]) : 1.0f;
  float* __restrict__ orow = out + r * ld_out;

  for (int f0 = gl * VEC; f0 < f_src; f0 += G * VEC) {
    float acc[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) acc[c] = 0.0f;
    // every batch, including a row's last partial one, issues its (up to U) neighbour loads together;
    // lanes past the row's end load nothing and add nothing (rows are mostly shorter than U)
    for (int k = beg; k < end; k += U) {
      const int n = end - k;
      T v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = T{};
        if (u < n) v[u] = V::load(x_src + (int64_t)col[k + u] * ld_src + f0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < n) {
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[c] = __fadd_rn(acc[c], V::get(v[u], c));
        }
      }
    }
    T o;
    if (combine == HGIN_COMBINE_ADD) {
      const T xd = V::template load_s<NT>(x_dst + r * ld_dst + f0);
#pragma unroll
      for (int c = 0; c < VEC; ++c) V::set(o, c, __fadd_rn(acc[c], __fmul_rn(s, V::get(xd, c))));
    } else {
#pragma unroll
      for (int c = 0; c < VEC; ++c) V::set(o, c, acc[c]);
    }
    V::template store_s<NT>(orow + f0, o);
  }
  if (combine == HGIN_COMBINE_CONCAT) {
    for (int f0 = gl * VEC; f0 < f_dst; f0 += G * VEC) {
      const T xd = V::template load_s<NT>(x_dst + r * ld_dst + f0);
      T o;
#pragma unroll
      for (int c = 0; c < VEC; ++c) V::set(o, c, __fmul_rn(s, V::get(xd, c)));
      V::template store_s<NT>(orow + f_src + f0, o);
    }
  }
}

template <int VEC, int G>
int launch_aggregate(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* x_src, int64_t ld_src,
                     int f_src, const float* x_dst, int64_t ld_dst, int f_dst, const float* eps, int combine,
                     float* out, int64_t ld_out, hipStream_t s) {
  constexpr int kRowsPerWave = kWave / G;
  const int64_t waves = ceil_div(n_rows, kRowsPerWave);
  const int64_t blocks = ceil_div(waves, 256 / kWave);
  const bool nt = agg_nt(combine, n_rows, (int64_t)(f_src + (combine == HGIN_COMBINE_CONCAT ? f_dst : 0)) * 4);
  HGIN_TRACE("k_aggregate<f32,G%d,mode%d>", G, combine);
#define HGIN_AGG_L(NTV)                                                                                    \
  k_aggregate<VEC, G, kAggU, NTV><<<dim3((unsigned)blocks), 256, 0, s>>>(rowptr, col, n_rows, x_src, ld_src, \
                                                                        f_src, x_dst, ld_dst, f_dst, eps,     \
                                                                        combine, out, ld_out)
  if (nt) HGIN_AGG_L(true); else HGIN_AGG_L(false);
#undef HGIN_AGG_L
  return check_launch("hgin_aggregate_f32");
}

template <int VEC>
int dispatch_g(int lanes_needed, const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* x_src,
               int64_t ld_src, int f_src, const float* x_dst, int64_t ld_dst, int f_dst, const float* eps,
               int combine, float* out, int64_t ld_out, hipStream_t s) {
#define HGIN_AGG_CASE(GV)                                                                                     \
  if (lanes_needed <= GV)                                                                                    \
    return launch_aggregate<VEC, GV>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps, \
                                     combine, out, ld_out, s);
  HGIN_AGG_CASE(4)
  HGIN_AGG_CASE(8)
  HGIN_AGG_CASE(16)
  HGIN_AGG_CASE(32)
#undef HGIN_AGG_CASE
  return launch_aggregate<VEC, 64>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps, combine,
                                   out, ld_out, s);
}

// ---------------------------------------------------------------------------------------------------
// bf16 storage (cfg5): the same row-per-lane-group walk, each lane owning 8 features (one 16-B load per
// neighbour row), fp32 sequential accumulation in edge order, one RNE rounding per output element.
// Bytes per launch: E * (4 + 2 * F_src) + (N + 1) * 4 + N * 2 * F_out [+ N * 2 * F_dst].
template <int VEC>
struct BVec;
template <>
struct BVec<1> {
  using T = uint16_t;
  static __device__ __forceinline__ T load(const uint16_t* p) { return *p; }
  template <bool NT>
  static __device__ __forceinline__ T load_s(const uint16_t* p) { return *p; }
  static __device__ __forceinline__ void unpack(const T& v, float (&f)[1]) { f[0] = bf2f(v); }
  template <bool NT>
  static __device__ __forceinline__ void store(uint16_t* p, const float (&f)[1]) { *p = (uint16_t)f2bf(f[0]); }
};
using u4v = __attribute__((ext_vector_type(4))) unsigned int;
template <>
struct BVec<8> {
  using T = uint4;
  static __device__ __forceinline__ T load(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }
  template <bool NT>
  static __device__ __forceinline__ T load_s(const uint16_t* p) {
    if (!NT) return load(p);
    const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  static __device__ __forceinline__ void unpack(const T& v, float (&f)[8]) {
    f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
    f[4] = bf_lo(v.z); f[5] = bf_hi(v.z); f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
  }
  template <bool NT>
  static __device__ __forceinline__ void store(uint16_t* p, const float (&f)[8]) {
    const u4v t = {pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7])};
    if (NT) __builtin_nontemporal_store(t, reinterpret_cast<u4v*>(p));
    else *reinterpret_cast<u4v*>(p) = t;
  }
};

template <int VEC, int G, int U, bool NT>
__global__ __launch_bounds__(256) void k_aggregate_bf16(const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ col, int64_t n_rows,
                                                        const uint16_t* __restrict__ x_src, int64_t ld_src, int f_src,
                                                        const uint16_t* __restrict__ x_dst, int64_t ld_dst, int f_dst,
                                                        const float* __restrict__ eps, int combine,
                                                        uint16_t* __restrict__ out, int64_t ld_out) {
  using V = BVec<VEC>;
  using T = typename V::T;
  constexpr int kRowsPerWave = kWave / G;
  const int lane = threadIdx.x & (kWave - 1);
  const int grp = lane / G;
  const int gl = lane % G;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  const int64_t r = wave_id * kRowsPerWave + grp;
  if (r >= n_rows) return;
  const int beg = rowptr[r];
  const int end = rowptr[r + 1];
  const float s = combine != HGIN_COMBINE_NONE ? __fadd_rn(1.0f, eps[0]) : 1.0f;
  uint16_t* __restrict__ orow = out + r * ld_out;

  for (int f0 = gl * VEC; f0 < f_src; f0 += G * VEC) {
    float acc[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) acc[c] = 0.0f;
    for (int k = beg; k < end; k += U) {   // batched tail, as k_aggregate
      const int n = end - k;
      T v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = T{};
        if (u < n) v[u] = V::load(x_src + (int64_t)col[k + u] * ld_src + f0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < n) {
          float f[VEC];
          V::unpack(v[u], f);
#pragma unroll
          for (int c = 0; c < VEC; ++c) acc[c] = __fadd_rn(acc[c], f[c]);
        }
      }
    }
    if (combine == HGIN_COMBINE_ADD) {
      float xd[VEC];
      V::unpack(V::template load_s<NT>(x_dst + r * ld_dst + f0), xd);
#pragma unroll
      for (int c = 0; c < VEC; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(s, xd[c]));
    }
    V::template store<NT>(orow + f0, acc);
  }
  if (combine == HGIN_COMBINE_CONCAT) {
    for (int f0 = gl * VEC; f0 < f_dst; f0 += G * VEC) {
      float xd[VEC];
      V::unpack(V::template load_s<NT>(x_dst + r * ld_dst + f0), xd);
#pragma unroll
      for (int c = 0; c < VEC; ++c) xd[c] = __fmul_rn(s, xd[c]);
      V::template store<NT>(orow + f_src + f0, xd);
    }
  }
}

template <int VEC, int G>
int launch_aggregate_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const uint16_t* x_src,
                          int64_t ld_src, int f_src, const uint16_t* x_dst, int64_t ld_dst, int f_dst, const float* eps,
                          int combine, uint16_t* out, int64_t ld_out, hipStream_t s) {
  constexpr int kRowsPerWave = kWave / G;
  const int64_t blocks = ceil_div(ceil_div(n_rows, kRowsPerWave), 256 / kWave);
  HGIN_TRACE("k_aggregate<bf16,G%d,mode%d>", G, combine);
#define HGIN_AGGB_L(NTV)                                                                       \
  k_aggregate_bf16<VEC, G, kAggU, NTV><<<dim3((unsigned)blocks), 256, 0, s>>>(                            \
      rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps, combine, out, ld_out)
  const bool nt = agg_nt(combine, n_rows, (int64_t)(f_src + (combine == HGIN_COMBINE_CONCAT ? f_dst : 0)) * 2);
  if (nt) HGIN_AGGB_L(true); else HGIN_AGGB_L(false);
#undef HGIN_AGGB_L
  return check_launch("hgin_aggregate_bf16");
}

template <int VEC>
int dispatch_g_bf16(int lanes_needed, const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                    const uint16_t* x_src, int64_t ld_src, int f_src, const uint16_t* x_dst, int64_t ld_dst, int f_dst,
                    const float* eps, int combine, uint16_t* out, int64_t ld_out, hipStream_t s) {
#define HGIN_AGG_CASE(GV)                                                                                    \
  if (lanes_needed <= GV)                                                                                   \
    return launch_aggregate_bf16<VEC, GV>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, \
                                          eps, combine, out, ld_out, s);
  HGIN_AGG_CASE(4)
  HGIN_AGG_CASE(8)
  HGIN_AGG_CASE(16)
  HGIN_AGG_CASE(32)
#undef HGIN_AGG_CASE
  return launch_aggregate_bf16<VEC, 64>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps,
                                        combine, out, ld_out, s);
}

// ---------------------------------------------------------------------------------------------------
// 16-B quads of a feature row (fp32: 4, bf16: 8 elements) for the pipelined walk below.  (A wide-lane variant
// with 2-4 quads per lane, k_agg_q, and an LDS-DMA gather, k_agg_lds, were measured and removed: DESIGN.md §3.)
template <typename T>
struct Quad;
template <>
struct Quad<float> {
  static constexpr int E = 4;
  static __device__ __forceinline__ void unpack(const uint4& v, float* f) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <>
struct Quad<uint16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ void unpack(const uint4& v, float* f) {
    f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
    f[4] = bf_lo(v.z); f[5] = bf_hi(v.z); f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
  }
};

template <bool NT>
__device__ __forceinline__ uint4 ld_quad(const void* p) {
  if (!NT) return *reinterpret_cast<const uint4*>(p);
  const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ void st_quad(void* p, const uint4& v) {
  const u4v t = {v.x, v.y, v.z, v.w};
  if (NT) __builtin_nontemporal_store(t, reinterpret_cast<u4v*>(p));
  else *reinterpret_cast<u4v*>(p) = t;
}

// ---------------------------------------------------------------------------------------------------
// Software-pipelined persistent walk (the bf16 kernel; fp32 keeps the kernels above).
// The kernels above pay up to four dependent memory round trips per destination row — rowptr, then the
// row's col entries, then the neighbour rows, then the self-term row — and a wave exits after one row per
// lane group.  Here every wave loops over rows r, r + S, r + 2S, ... (S = resident lane groups of the
// grid) and, in the iteration that gathers row r, also issues rowptr of row r + 2S, the first col chunk of
// row r + S (one coalesced G-lane load; lane j holds col[beg + j], broadcast to the group by ds_bpermute)
// and row r's self-term quad: one round trip per row.  Per-feature sums stay sequential in edge order
// (bit-identical to the kernels above and to CPU scatter_add_).  One 16-B quad per lane: f_src, f_dst <=
// G * E elements (E = 4 fp32 / 8 bf16).  The walk's trip count is the wave's largest row (wave-uniform,
// so every lane reaches the broadcasts); lanes past their row's end load nothing.
// Measured (tools/agg_bench.py, profiles/r01_agg_pipe.txt): bf16 1.7-1.9 % faster over the cfg2 / cfg3 relation
// shapes (cfg3 backward +7.8 %), fp32 6-9 % slower (fewer resident waves: 5-6 per SIMD against the one-row
// kernels' short-lived 8), so the default is the pipelined walk for bf16 and the batched-tail kernel for fp32.
template <typename T>
constexpr bool agg_pipe_enabled() {
  return sizeof(T) == 2;
}

template <int G>
__device__ __forceinline__ int wave_max_over_groups(int v) {
#pragma unroll
  for (int off = G; off < kWave; off <<= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

template <typename T, int G, int U, bool NT>
__global__ __launch_bounds__(256) void k_agg_pipe(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                  int64_t n_rows, const T* __restrict__ x_src, int64_t ld_src,
                                                  int f_src, const T* __restrict__ x_dst, int64_t ld_dst, int f_dst,
                                                  const float* __restrict__ eps, int combine, T* __restrict__ out,
                                                  int64_t ld_out) {
  static_assert(G % U == 0, "a col chunk must hold whole batches");
  constexpr int E = Quad<T>::E;
  constexpr int kRowsPerWave = kWave / G;
  const int lane = threadIdx.x & (kWave - 1);
  const int grp = lane / G;
  const int gl = lane % G;
  const int64_t S = (int64_t)gridDim.x * (blockDim.x / kWave) * kRowsPerWave;
  int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) * kRowsPerWave;
  int64_t r = r0 + grp;
  const int f0 = gl * E;
  const bool src_lane = f0 < f_src;
  const bool self_lane = combine != HGIN_COMBINE_NONE && f0 < f_dst;
  const float s = combine != HGIN_COMBINE_NONE ? __fadd_rn(1.0f, eps[0]) : 1.0f;

  int beg = 0, end = 0, begn = 0, endn = 0;
  if (r < n_rows) { beg = rowptr[r]; end = rowptr[r + 1]; }
  if (r + S < n_rows) { begn = rowptr[r + S]; endn = rowptr[r + S + 1]; }
  int cur = gl < end - beg ? col[beg + gl] : 0;
  for (; r0 < n_rows; r0 += S, r += S) {
    // prefetches for the next two rows of this lane group, issued with this row's loads
    int begnn = 0, endnn = 0;
    if (r + 2 * S < n_rows) { begnn = rowptr[r + 2 * S]; endnn = rowptr[r + 2 * S + 1]; }
    const int curn = gl < endn - begn ? col[begn + gl] : 0;
    const bool valid = r < n_rows;
    uint4 xd = make_uint4(0u, 0u, 0u, 0u);
    if (valid && self_lane) xd = ld_quad<NT>(x_dst + r * ld_dst + f0);

    const int n = end - beg;     // 0 past the last row
    const int n_wave = wave_max_over_groups<G>(n);
    float acc[E];
#pragma unroll
    for (int c = 0; c < E; ++c) acc[c] = 0.0f;
    for (int k = 0; k < n_wave; k += U) {
      if (k != 0 && (k & (G - 1)) == 0) cur = k + gl < n ? col[beg + k + gl] : 0;   // rows longer than G
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = __shfl(cur, grp * G + ((k + u) & (G - 1)));
        v[u] = make_uint4(0u, 0u, 0u, 0u);
        if (k + u < n && src_lane) v[u] = ld_quad<false>(x_src + (int64_t)idx * ld_src + f0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u < n) {
          float f[E];
          Quad<T>::unpack(v[u], f);
#pragma unroll
          for (int c = 0; c < E; ++c) acc[c] = __fadd_rn(acc[c], f[c]);
        }
      }
    }
    if (valid) {
      T* __restrict__ orow = out + r * ld_out;
      float xs[E];
      Quad<T>::unpack(xd, xs);
      if (combine == HGIN_COMBINE_ADD) {
#pragma unroll
        for (int c = 0; c < E; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(s, xs[c]));
      }
      if (src_lane) st_quad<NT>(orow + f0, Quad<T>::pack(acc));
      if (combine == HGIN_COMBINE_CONCAT && self_lane) {
#pragma unroll
        for (int c = 0; c < E; ++c) xs[c] = __fmul_rn(s, xs[c]);
        st_quad<NT>(orow + f_src + f0, Quad<T>::pack(xs));
      }
    }
    beg = begn; end = endn; begn = begnn; endn = endnn; cur = curn;
  }
}

template <typename F>
int64_t agg_resident_blocks(F kernel) {
  int per_cu = 0, dev = 0, cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
    cus = prop.multiProcessorCount;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
  return (int64_t)per_cu * cus;
}

template <typename T, int G, int U, bool NT>
int launch_agg_pipe_g(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const T* x_src, int64_t ld_src,
                      int f_src, const T* x_dst, int64_t ld_dst, int f_dst, const float* eps, int combine, T* out,
                      int64_t ld_out, hipStream_t s) {
  static const int64_t slots = agg_resident_blocks(k_agg_pipe<T, G, U, NT>);
  const int64_t need = ceil_div(n_rows, (int64_t)(256 / G));
  const int64_t blocks = need < slots ? need : slots;
  HGIN_TRACE("k_agg_pipe<%s,G%d,mode%d>", sizeof(T) == 4 ? "f32" : "bf16", G, combine);
  k_agg_pipe<T, G, U, NT><<<dim3((unsigned)blocks), 256, 0, s>>>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst,
                                                                  ld_dst, f_dst, eps, combine, out, ld_out);
  return HGIN_OK;
}

// Returns -1000 when the shapes do not fit the pipelined kernel (one aligned quad per lane, <= 64 lanes).
template <typename T>
int try_agg_pipe(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const T* x_src, int64_t ld_src, int f_src,
                 const T* x_dst, int64_t ld_dst, int f_dst, const float* eps, int combine, T* out, int64_t ld_out,
                 hipStream_t s, const char* what) {
  constexpr int E = Quad<T>::E;
  const int fd = combine == HGIN_COMBINE_NONE ? 0 : f_dst;
  if (!agg_pipe_enabled<T>() || f_src % E || fd % E || !aligned16(x_src) || ld_src % E || !aligned16(out) ||
      ld_out % E)
    return -1000;
  if (fd && (!aligned16(x_dst) || ld_dst % E)) return -1000;
  const int widest = f_src > fd ? f_src : fd;
  const int lanes = (widest + E - 1) / E;
  if (lanes < 1 || lanes > kWave) return -1000;
  const bool nt = agg_nt(combine, n_rows, (int64_t)(f_src + (combine == HGIN_COMBINE_CONCAT ? f_dst : 0)) * (int64_t)sizeof(T));
  int rc;
#define HGIN_PIPE_G(GV, UV)                                                                                      \
  rc = nt ? launch_agg_pipe_g<T, GV, UV, true>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps, \
                                               combine, out, ld_out, s)                                         \
          : launch_agg_pipe_g<T, GV, UV, false>(rowptr, col, n_rows, x_src, ld_src, f_src, x_dst, ld_dst, f_dst, eps, \
                                                combine, out, ld_out, s);
  if (lanes <= 4) { HGIN_PIPE_G(4, 4) }
  else if (lanes <= 8) { HGIN_PIPE_G(8, 8) }
  else if (lanes <= 16) { HGIN_PIPE_G(16, 8) }
  else if (lanes <= 32) { HGIN_PIPE_G(32, 8) }
  else { HGIN_PIPE_G(64, 8) }
#undef HGIN_PIPE_G
  if (rc) return rc;
  return check_launch(what);
}

int check_aggregate_args(const char* what, const int32_t* rowptr, int64_t n_rows, int64_t ld_src, int64_t f_src,
                         const void* x_dst, int64_t ld_dst, int64_t f_dst, const float* eps, int combine,
                         const void* out, int64_t ld_out) {
  HGIN_ARG_CHECK(combine == HGIN_COMBINE_NONE || combine == HGIN_COMBINE_ADD || combine == HGIN_COMBINE_CONCAT,
                 "%s: bad combine mode %d", what, combine);
  HGIN_ARG_CHECK(n_rows >= 0 && f_src >= 0 && f_src < (1 << 24), "%s: bad sizes", what);
  if (n_rows == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr != nullptr && out != nullptr, "%s: rowptr/out NULL", what);
  int64_t out_w = f_src;
  if (combine != HGIN_COMBINE_NONE) {
    HGIN_ARG_CHECK(x_dst != nullptr && eps != nullptr, "%s: combine needs x_dst and eps", what);
    HGIN_ARG_CHECK(f_dst >= 0 && f_dst < (1 << 24), "%s: bad f_dst", what);
    if (combine == HGIN_COMBINE_ADD)
      HGIN_ARG_CHECK(f_dst == f_src, "%s: ADD needs f_dst == f_src (%lld vs %lld)", what, (long long)f_dst,
                     (long long)f_src);
    if (combine == HGIN_COMBINE_CONCAT) out_w = f_src + f_dst;
    HGIN_ARG_CHECK(ld_dst >= f_dst, "%s: ld_dst < f_dst", what);
  }
  HGIN_ARG_CHECK(ld_src >= f_src && ld_out >= out_w, "%s: leading dimension too small", what);
  return HGIN_OK;
}

// ---------------------------------------------------------------------------------------------------
// Long rows (degree skew; SURVEY.md §7 "Hard parts", §8.D skew variant).  The row-per-lane-group walk above
// is serial in a row's edges, so one destination with millions of in-edges (Zipf(1.1) destinations: the top
// link of cfg3 gets ~9 % of a relation's 30M edges) stalls the whole launch.  The host splits such rows out
// of the CSR (ops.py: rows with more than HGIN_LONG_ROW edges are emptied in a compacted copy the main
// kernel runs on — so it writes their self term, and zeros for the neighbour sum) and hands them here as
// chunks of consecutive edges (items: [row-local chunk start, end) pairs, in edge order):
//   k_long_partial: one wave per chunk, lanes across the features, the chunk's edges summed in edge order
//                   (fp32) -> partial[chunk][F];
//   k_long_combine: one wave per long row, its chunk partials added in chunk order, then the self term
//                   ((1 + eps) x_dst for ADD, one rounding as the main kernel), stored over columns [0, F).
// Fixed chunking and fixed combine order: bitwise reproducible run to run, but re-associated against the
// CPU's sequential edge-order sum (a tolerance, not bit-exact; tests/test_gpu_kernels.py).
template <typename T>
struct LongElem;
template <>
struct LongElem<float> {
  static __device__ __forceinline__ void load4(const float* p, float (&f)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  static __device__ __forceinline__ void store4(float* p, const float (&f)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};
template <>
struct LongElem<uint16_t> {
  static __device__ __forceinline__ void load4(const uint16_t* p, float (&f)[4]) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
  }
  static __device__ __forceinline__ void store4(uint16_t* p, const float (&f)[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]));
  }
};

template <typename T, int U>
__global__ __launch_bounds__(256) void k_long_partial(const int32_t* __restrict__ col, const int32_t* __restrict__ items,
                                                      int64_t n_items, const T* __restrict__ x_src, int64_t ld_src,
                                                      int f_src, float* __restrict__ partial) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t item = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (item >= n_items) return;
  const int beg = items[2 * item];
  const int end = items[2 * item + 1];
  float* prow = partial + item * f_src;
  for (int f0 = lane * 4; f0 < f_src; f0 += kWave * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = beg; k < end; k += U) {
      const int n = end - k;
      float v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u][0] = v[u][1] = v[u][2] = v[u][3] = 0.f;
        if (u < n) LongElem<T>::load4(x_src + (int64_t)col[k + u] * ld_src + f0, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < n)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = __fadd_rn(acc[c], v[u][c]);
    }
    *reinterpret_cast<float4*>(prow + f0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_long_combine(const int32_t* __restrict__ long_rows,
                                                      const int32_t* __restrict__ item_ptr, int64_t n_long,
                                                      const float* __restrict__ partial, int f_src,
                                                      const T* __restrict__ x_dst, int64_t ld_dst,
                                                      const float* __restrict__ eps, int combine, T* __restrict__ out,
                                                      int64_t ld_out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (j >= n_long) return;
  const int64_t r = long_rows[j];
  const int i0 = item_ptr[j], i1 = item_ptr[j + 1];
  const float s = combine != HGIN_COMBINE_NONE ? __fadd_rn(1.0f, eps[0]) : 1.0f;
  for (int f0 = lane * 4; f0 < f_src; f0 += kWave * 4) {
    float acc[4];
    {
      const float4 p = *reinterpret_cast<const float4*>(partial + (int64_t)i0 * f_src + f0);
      acc[0] = p.x; acc[1] = p.y; acc[2] = p.z; acc[3] = p.w;
    }
    for (int i = i0 + 1; i < i1; ++i) {
      const float4 p = *reinterpret_cast<const float4*>(partial + (int64_t)i * f_src + f0);
      acc[0] = __fadd_rn(acc[0], p.x); acc[1] = __fadd_rn(acc[1], p.y);
      acc[2] = __fadd_rn(acc[2], p.z); acc[3] = __fadd_rn(acc[3], p.w);
    }
    if (combine == HGIN_COMBINE_ADD) {
      float xd[4];
      LongElem<T>::load4(x_dst + r * ld_dst + f0, xd);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(s, xd[c]));
    }
    LongElem<T>::store4(out + r * ld_out + f0, acc);
  }
}

template <typename T>
int aggregate_long(const char* what, const int32_t* col, const int32_t* items, int64_t n_items,
                   const int32_t* long_rows, const int32_t* item_ptr, int64_t n_long, const T* x_src, int64_t ld_src,
                   int64_t f_src, const T* x_dst, int64_t ld_dst, int64_t f_dst, const float* eps, int combine, T* out,
                   int64_t ld_out, float* partial, size_t partial_bytes, void* stream) {
  HGIN_ARG_CHECK(combine == HGIN_COMBINE_NONE || combine == HGIN_COMBINE_ADD || combine == HGIN_COMBINE_CONCAT,
                 "%s: bad combine", what);
  HGIN_ARG_CHECK(n_items >= 0 && n_long >= 0 && f_src >= 0, "%s: bad sizes", what);
  if (n_long == 0 || f_src == 0) return HGIN_OK;
  constexpr int E4 = 4;
  HGIN_ARG_CHECK(col && items && long_rows && item_ptr && x_src && out && partial, "%s: NULL argument", what);
  HGIN_ARG_CHECK(f_src % E4 == 0 && ld_src % E4 == 0 && ld_out % E4 == 0, "%s: f_src / ld must be multiples of 4", what);
  HGIN_ARG_CHECK(combine != HGIN_COMBINE_ADD || (x_dst && eps && f_dst == f_src && ld_dst % E4 == 0),
                 "%s: ADD needs x_dst / eps with f_dst == f_src", what);
  HGIN_ARG_CHECK(combine == HGIN_COMBINE_NONE || eps, "%s: combine needs eps", what);
  HGIN_ARG_CHECK(partial_bytes >= (size_t)n_items * (size_t)f_src * sizeof(float), "%s: partial workspace too small",
                 what);
  hipStream_t s = as_stream(stream);
  const unsigned pb = (unsigned)ceil_div(n_items, 4);
  HGIN_TRACE("k_long_partial+k_long_combine<%s,mode%d>", sizeof(T) == 4 ? "f32" : "bf16", combine);
  k_long_partial<T, 8><<<pb, 256, 0, s>>>(col, items, n_items, x_src, ld_src, (int)f_src, partial);
  const unsigned cb = (unsigned)ceil_div(n_long, 4);
  k_long_combine<T><<<cb, 256, 0, s>>>(long_rows, item_ptr, n_long, partial, (int)f_src, x_dst, ld_dst, eps, combine,
                                       out, ld_out);
  return check_launch(what);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_aggregate_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const uint16_t* x_src,
                                   int64_t ld_src, int64_t f_src, const uint16_t* x_dst, int64_t ld_dst, int64_t f_dst,
                                   const float* eps, int combine, uint16_t* out, int64_t ld_out, void* stream) {
  if (int rc = check_aggregate_args("hgin_aggregate_bf16", rowptr, n_rows, ld_src, f_src, x_dst, ld_dst, f_dst, eps,
                                    combine, out, ld_out))
    return rc;
  if (n_rows == 0) return HGIN_OK;
  hipStream_t s = as_stream(stream);
  const bool dst_ok = combine == HGIN_COMBINE_NONE || (aligned16(x_dst) && ld_dst % 8 == 0 && f_dst % 8 == 0);
  const bool vec8 = f_src % 8 == 0 && aligned16(x_src) && ld_src % 8 == 0 && aligned16(out) && ld_out % 8 == 0 &&
                    dst_ok && (f_src > 0 || f_dst > 0);
  const int fd = combine == HGIN_COMBINE_CONCAT ? (int)f_dst : 0;
  const int64_t widest = f_src > fd ? f_src : fd;
  {
    const int rc = try_agg_pipe<uint16_t>(rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst, (int)f_dst,
                                          eps, combine, out, ld_out, s, "hgin_aggregate_bf16");
    if (rc != -1000) return rc;
  }
  if (vec8)
    return dispatch_g_bf16<8>((int)ceil_div(widest, 8), rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst,
                              (int)f_dst, eps, combine, out, ld_out, s);
  return dispatch_g_bf16<1>((int)widest, rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst, (int)f_dst,
                            eps, combine, out, ld_out, s);
}

extern "C" int hgin_aggregate_f32(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* x_src,
                                  int64_t ld_src, int64_t f_src, const float* x_dst, int64_t ld_dst, int64_t f_dst,
                                  const float* eps, int combine, float* out, int64_t ld_out, void* stream) {
  if (int rc = check_aggregate_args("hgin_aggregate_f32", rowptr, n_rows, ld_src, f_src, x_dst, ld_dst, f_dst, eps,
                                    combine, out, ld_out))
    return rc;
  if (n_rows == 0) return HGIN_OK;
  hipStream_t s = as_stream(stream);
  const bool dst_ok = combine == HGIN_COMBINE_NONE || (aligned16(x_dst) && ld_dst % 4 == 0 && f_dst % 4 == 0);
  const bool vec4 = f_src % 4 == 0 && aligned16(x_src) && ld_src % 4 == 0 && aligned16(out) && ld_out % 4 == 0 &&
                    dst_ok && (f_src > 0 || f_dst > 0);
  const int fd = combine == HGIN_COMBINE_CONCAT ? (int)f_dst : 0;
  {
    const int rc = try_agg_pipe<float>(rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst, (int)f_dst, eps,
                                       combine, out, ld_out, s, "hgin_aggregate_f32");
    if (rc != -1000) return rc;
  }
  if (vec4) {
    const int64_t widest = f_src > fd ? f_src : fd;
    return dispatch_g<4>((int)ceil_div(widest, 4), rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst,
                         (int)f_dst, eps, combine, out, ld_out, s);
  }
  const int64_t widest = f_src > fd ? f_src : fd;
  return dispatch_g<1>((int)widest, rowptr, col, n_rows, x_src, ld_src, (int)f_src, x_dst, ld_dst, (int)f_dst, eps,
                       combine, out, ld_out, s);
}


extern "C" int hgin_aggregate_long_f32(const int32_t* col, const int32_t* items, int64_t n_items,
                                       const int32_t* long_rows, const int32_t* item_ptr, int64_t n_long,
                                       const float* x_src, int64_t ld_src, int64_t f_src, const float* x_dst,
                                       int64_t ld_dst, int64_t f_dst, const float* eps, int combine, float* out,
                                       int64_t ld_out, float* partial, size_t partial_bytes, void* stream) {
  return aggregate_long<float>("hgin_aggregate_long_f32", col, items, n_items, long_rows, item_ptr, n_long, x_src,
                               ld_src, f_src, x_dst, ld_dst, f_dst, eps, combine, out, ld_out, partial, partial_bytes,
                               stream);
}

extern "C" int hgin_aggregate_long_bf16(const int32_t* col, const int32_t* items, int64_t n_items,
                                        const int32_t* long_rows, const int32_t* item_ptr, int64_t n_long,
                                        const uint16_t* x_src, int64_t ld_src, int64_t f_src, const uint16_t* x_dst,
                                        int64_t ld_dst, int64_t f_dst, const float* eps, int combine, uint16_t* out,
                                        int64_t ld_out, float* partial, size_t partial_bytes, void* stream) {
  return aggregate_long<uint16_t>("hgin_aggregate_long_bf16", col, items, n_items, long_rows, item_ptr, n_long, x_src,
                                  ld_src, f_src, x_dst, ld_dst, f_dst, eps, combine, out, ld_out, partial,
                                  partial_bytes, stream);
}

// A5 — GIN MLP update on MFMA, the readout Linear(+PReLU) layers, and the plain NT
// GEMM of the input-gradient backward.
//
// Reference: GINLayer.mlp = Sequential(Linear(K, N), PReLU()) (models.py:236-239) applied at
// models.py:217 (addmm + prelu as two kernels), HeteroConv's torch.stack(outs).sum(0) for the second
// relation into a node type (models.py:286-298), and the readout Sequential(Linear, PReLU) layers applied
// to cat(x_path, raw path features) (models.py:300-330, :362-374).  One kernel computes
//     z = [A1 | A2] W^T + b ;  y = prelu(z) [+ accum]          (EPI 1; EPI 2: y = z; EPI 0: no bias)
// with fp32 operands on the bf16 matrix cores by default: each operand is split into three bf16 planes at
// staging time and every product is formed from six v_mfma_f32_32x32x16_bf16 terms (hgin_common.h, "split"
// mode); HGIN_F32_GEMM=mfma32 selects the exact f32 matrix-core path (v_mfma_f32_32x32x2_f32, 157 TF/s peak).
// The two A sources remove the readout's torch.cat: columns [0, K1) come from A1, [K1, K) from A2.
//
// Tiling: 256 threads = 4 waves.  Each wave owns 2 x TN MFMA tiles of 32 x 32 (64 rows x 32*TN columns);
// the waves form a WM x WN grid: TN = 2 -> 2 x 2 waves, a 128 x 128 workgroup tile (H = 128/256 layers);
// TN = 1 -> 4 x 1 waves, a 256 x 32 tile for narrow outputs (the readout's Linear(128, 32) and its head),
// so no MFMA work is spent on columns that do not exist.
// A and W are both K-contiguous (torch Linear.weight is [N, K]), so inside a K-chunk of 8 the MFMA k-step
// t (0..3) of lane half h (0/1) uses k = 8c + 4h + t: every lane reads its operands for four k-steps with
// ONE ds_read_b128 from a [row][BK + 4] LDS image (row stride 36 floats puts the 16 rows of a ds_read_b128
// lane group on 16 distinct 4-bank slots).  The next K-tile's global loads (float4) are issued into
// registers before the current tile's MFMAs and written to LDS after them (3 waves/SIMD).
// Epilogue through LDS: the 32x32 C/D layout gives each lane one column (4-B stores, store-issue bound), so
// each wave parks 32 rows of its tile in LDS and writes them back as row-contiguous float4s.
// C/D map of the 32x32 f32 MFMA (gfx950): col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
// Measured choices (tools/gemm_bench.py; profiles/r01_gemm_variants.txt, r01_gemm_persistent_variants.txt):
// register prefetch at 3 waves/SIMD beats 2 waves by 7-14 % and the unpipelined loop by 3-6 %; a
// persistent grid with cross-tile prefetch was 5 % slower (it needs 2 waves/SIMD).
#include "hgin_common.h"

#include <type_traits>

namespace hgin {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kBK = 32;
constexpr int kLds = kBK + 4;

struct Src2 {
  const float* p1;
  int64_t ld1;
  const float* p2;
  int64_t ld2;
  int64_t k1;
  // optional: columns from p2 are (1 + eps2[0]) * p2 (the GIN self term of a concat GINConv, models.py:212-213,
  // applied as the tile is loaded instead of materialised by the aggregate; same fp32 product, one rounding)
  const float* eps2 = nullptr;
};

// ROWS x 32 floats of [p1 | p2] starting at (row0, k0) -> ROWS/32 float4 per thread:
// thread t owns column chunk q = t & 7 of rows (t >> 3) + 32 i.
// kClean (K and k1 multiples of kBK, 16-B aligned rows): a K-tile lies wholly in p1 or p2 (a scalar choice)
// and rows past the end are clamped to the last row instead of branched around — their products land in
// output rows / columns that are never stored — so the loads are branch-free and the compiler keeps the
// prefetch in flight under the MFMAs (a per-load branch made it wait at each join).  Otherwise every
// element is bounds-checked.
__device__ __forceinline__ float self_scale(const float* eps2) { return eps2 ? __fadd_rn(1.0f, eps2[0]) : 1.0f; }

template <bool kClean, int ROWS, int NT = 256>
__device__ __forceinline__ void load_tile(float4 (&r)[ROWS / (NT / 8)], const Src2& s, int64_t row0, int64_t rows,
                                          int64_t k0, int64_t K, int tid, float sc2 = 1.0f) {
  constexpr int RP = NT / 8;   // rows per pass of the workgroup's threads
  if constexpr (kClean) {
    // select between the loaded VALUES: a select between the two struct fields' addresses would make
    // the compiler copy the by-value kernel argument into scratch
    const bool first = k0 < s.k1;
    const uintptr_t u1 = reinterpret_cast<uintptr_t>(s.p1), u2 = reinterpret_cast<uintptr_t>(s.p2);
    const int64_t l1 = s.ld1, l2 = s.ld2;
    const float* base = reinterpret_cast<const float*>(first ? u1 : u2);
    const int64_t ld = first ? l1 : l2;
    const int64_t kk = (first ? k0 : k0 - s.k1) + (tid & 7) * 4;
#pragma unroll
    for (int i = 0; i < ROWS / RP; ++i) {
      int64_t gr = row0 + (tid >> 3) + RP * i;
      gr = gr < rows ? gr : rows - 1;
      const float4 v = *reinterpret_cast<const float4*>(base + gr * ld + kk);
      r[i] = v;
    }
    // (eps2 scaling of a clean p2 tile is applied when the tile is staged: scale_tile)
  } else {
    const int64_t kk = k0 + (tid & 7) * 4;
#pragma unroll
    for (int i = 0; i < ROWS / RP; ++i) {
      const int64_t gr = row0 + (tid >> 3) + RP * i;
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      if (gr < rows) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int64_t k = kk + c;
          t[c] = k < K ? (k < s.k1 ? s.p1[gr * s.ld1 + k] : __fmul_rn(sc2, s.p2[gr * s.ld2 + (k - s.k1)])) : 0.0f;
        }
      }
      r[i] = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
}

// The eps2 scale of a clean p2 tile, applied at staging time (after the MFMAs the prefetch hides under):
// scaling inside load_tile would consume the loaded values at once and make the loads wait there.
template <int ROWS, int NT = 256>
__device__ __forceinline__ void scale_tile(float4 (&r)[ROWS / (NT / 8)], float sc) {
#pragma unroll
  for (int i = 0; i < ROWS / (NT / 8); ++i)
    r[i] = make_float4(__fmul_rn(sc, r[i].x), __fmul_rn(sc, r[i].y), __fmul_rn(sc, r[i].z), __fmul_rn(sc, r[i].w));
}

template <int ROWS, int NT = 256>
__device__ __forceinline__ void store_tile(float* __restrict__ dst, const float4 (&r)[ROWS / (NT / 8)], int tid) {
#pragma unroll
  for (int i = 0; i < ROWS / (NT / 8); ++i)
    *reinterpret_cast<float4*>(dst + ((tid >> 3) + (NT / 8) * i) * kLds + (tid & 7) * 4) = r[i];
}

// Split mode (hgin_common.h): the same tile written as three bf16 planes per row.  NT image: 48-word rows
// (3 planes x 16 words, no pad) with the 4-word chunks of a plane XOR-swizzled by (row >> 2) & 3.  Row bases
// 48 r mod 64 = 16 (3 r mod 4), so the split stores (8 lanes x 2 words per row, 4 rows per 32 lanes) cover
// 4 disjoint 16-word bank blocks and a ds_read_b128 lane group (16 rows, one logical chunk) hits 4 bases x 4
// swizzled chunks = 16 distinct slots: both conflict-free.  (The 52-word rows of hgin_common.h kept the reads
// conflict-free but made the stores 2-way: SQ_LDS_BANK_CONFLICT ~0.9 of the LDS-active cycles, PMC at
// M = 3M, K = 512, N = 256, profiles/r02/gemm_pmc_cfg3.txt.)
constexpr int kSplitRowWordsNT = 48;
__device__ __forceinline__ int nt_chunk(int row, int c) { return (c ^ ((row >> 2) & 3)) << 2; }

template <int ROWS, int NT = 256>
__device__ __forceinline__ void store_tile_split(uint32_t* __restrict__ dst, const float4 (&r)[ROWS / (NT / 8)],
                                                 int tid) {
#pragma unroll
  for (int i = 0; i < ROWS / (NT / 8); ++i) {
    uint2 o[3];
    split4(r[i], o);
    const int rr = (tid >> 3) + (NT / 8) * i;
    const int q = tid & 7;                        // float4 quad q = chunk q >> 1, half q & 1
    uint32_t* row = dst + rr * kSplitRowWordsNT + nt_chunk(rr, q >> 1) + (q & 1) * 2;
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(row + p * 16) = o[p];
  }
}

// 4 consecutive output columns of one row: fp32 (16-B) or bf16 (8-B) accesses, scalar at the ragged edge.
template <typename OutT>
struct Out4;
template <>
struct Out4<float> {
  using raw = float4;   // a prefetched group in its storage form (4 VGPRs)
  static __device__ __forceinline__ float rt(float v) { return v; }   // the value a store keeps
  static __device__ __forceinline__ raw ld_raw(const float* p, bool full, int nv) {
    if (full) return *reinterpret_cast<const float4*>(p);
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nv; ++i) t[i] = p[i];
    return make_float4(t[0], t[1], t[2], t[3]);
  }
  static __device__ __forceinline__ void unpack(const raw& v, float (&o)[4]) {
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&o)[4], bool full, int nv) {
    if (full) *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    else for (int t = 0; t < nv; ++t) p[t] = o[t];
  }
  // non-temporal forms (streamed-once outputs / epilogue inputs)
  static __device__ __forceinline__ void st_nt(float* p, const float (&o)[4], bool full, int nv) {
    using f4v = __attribute__((ext_vector_type(4))) float;
    if (full) __builtin_nontemporal_store(f4v{o[0], o[1], o[2], o[3]}, reinterpret_cast<f4v*>(p));
    else for (int t = 0; t < nv; ++t) __builtin_nontemporal_store(o[t], p + t);
  }
  static __device__ __forceinline__ raw ld_raw_nt(const float* p, bool full, int nv) {
    using f4v = __attribute__((ext_vector_type(4))) float;
    if (!full) return ld_raw(p, full, nv);
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  static __device__ __forceinline__ void ld(const float* p, float (&o)[4], bool full, int nv) {
    if (full) {
      const float4 v = *reinterpret_cast<const float4*>(p);
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else {
      for (int t = 0; t < nv; ++t) o[t] = p[t];
    }
  }
};
template <>
struct Out4<uint16_t> {
  using raw = uint2;    // 4 packed bf16 (2 VGPRs)
  static __device__ __forceinline__ float rt(float v) { return bf2f(f2bf(v)); }
  static __device__ __forceinline__ raw ld_raw(const uint16_t* p, bool full, int nv) {
    if (full) return *reinterpret_cast<const uint2*>(p);
    uint32_t t[4] = {0u, 0u, 0u, 0u};
    for (int i = 0; i < nv; ++i) t[i] = p[i];
    return make_uint2(t[0] | (t[1] << 16), t[2] | (t[3] << 16));
  }
  static __device__ __forceinline__ void unpack(const raw& v, float (&o)[4]) {
    o[0] = bf_lo(v.x); o[1] = bf_hi(v.x); o[2] = bf_lo(v.y); o[3] = bf_hi(v.y);
  }
  static __device__ __forceinline__ void st(uint16_t* p, const float (&o)[4], bool full, int nv) {
    if (full) *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
    else for (int t = 0; t < nv; ++t) p[t] = (uint16_t)f2bf(o[t]);
  }
  static __device__ __forceinline__ void st_nt(uint16_t* p, const float (&o)[4], bool full, int nv) {
    using u2v = __attribute__((ext_vector_type(2))) unsigned int;
    if (full) __builtin_nontemporal_store(u2v{pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3])}, reinterpret_cast<u2v*>(p));
    else st(p, o, full, nv);
  }
  static __device__ __forceinline__ raw ld_raw_nt(const uint16_t* p, bool full, int nv) {
    using u2v = __attribute__((ext_vector_type(2))) unsigned int;
    if (!full) return ld_raw(p, full, nv);
    const u2v v = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p));
    return make_uint2(v.x, v.y);
  }
  static __device__ __forceinline__ void ld(const uint16_t* p, float (&o)[4], bool full, int nv) {
    if (full) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      o[0] = bf_lo(v.x); o[1] = bf_hi(v.x); o[2] = bf_lo(v.y); o[3] = bf_hi(v.y);
    } else {
      for (int t = 0; t < nv; ++t) o[t] = bf2f(p[t]);
    }
  }
};

// EPI 4 — the dX GEMM of a GINConv backward with the self term's backward fused (models.py:210-215 reached
// from train.py:43; replaces hgin_combine_bwd_* after the GEMM): C = g_comb = g_z W is stored as usual and,
// for the self columns [cs, N) (cs = F_src for concat, 0 for add), g_x_dst[:, c - cs] = (1 + eps) C[:, c]
// (optional) and a per-workgroup partial of sum(C[:, c] * x_dst[:, c - cs]) (the eps gradient; fixed order,
// summed over workgroups by k_final_scalar).  C is used as stored (bf16: after its rounding), as the separate
// combine backward would read it.
struct CombEpi {
  const void* xd;     // x_dst [M, N - cs], row stride ldxd (C's element type)
  int64_t ldxd;
  void* gd;           // g_x_dst [M, N - cs] or NULL, row stride ldgd
  int64_t ldgd;
  int64_t cs;         // first self column of C (a multiple of 4)
  const float* eps;   // device float[1]
  float* part;        // [workgroup tiles] eps-gradient partials
  const void* gp = nullptr;   // optional: a gradient g_x_dst accumulates onto (may alias gd), row stride ldgp
  int64_t ldgp = 0;
  bool nt_io = false;         // non-temporal epilogue streams (outputs, accum / x_dst / g_prev rows)
  bool zy = false;            // bf16 EPI 1 without accum: z may be left unwritten when the slope is > 0 (k_ws_bf16)
};

// Epilogue shared by the fp32 and bf16 kernels.  Per 32-row half (tm) each wave parks its 32 x WCOLS
// results in LDS, then writes row-contiguous 4-column groups (bias, PReLU, accum applied on the way out).
// A lane always owns the same 4 columns, so its bias values are loaded once, and the accum rows it will
// need are loaded before the LDS round trip: no dependent global load inside the store loop.
using f32x4v = __attribute__((ext_vector_type(4))) float;

// C/D layouts: f32x16 acc[2][TN] — 32 x 32 MFMA tiles (row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5), col = lane & 31);
// f32x4v acc[4][2 TN] — 16 x 16 tiles of v_mfma_f32_16x16x32_bf16 (row = 4 (lane >> 4) + reg, col = lane & 15).
template <int TN>
__device__ __forceinline__ void park_acc(const f32x16 (&acc)[2][TN], float* Cw, int kLc, int tm, int lane) {
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int e = 0; e < 16; ++e) Cw[((e & 3) + 8 * (e >> 2) + 4 * lh) * kLc + tn * 32 + li] = acc[tm][tn][e];
}
template <int TN2>
__device__ __forceinline__ void park_acc(const f32x4v (&acc)[4][TN2], float* Cw, int kLc, int tm, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int bn = 0; bn < TN2; ++bn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        Cw[(j * 16 + 4 * (lane >> 4) + i) * kLc + bn * 16 + (lane & 15)] = acc[2 * tm + j][bn][i];
}

template <int EPI, int TN, typename OutT, typename AccT = f32x16[2][TN]>
__device__ __forceinline__ void epilogue(const AccT& acc, float* smem, int wave, int wm, int wn, int lane,
                                         int li, int lh, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                         const float* __restrict__ bias, const float* __restrict__ prelu,
                                         const OutT* __restrict__ accum, OutT* __restrict__ Z, OutT* __restrict__ Y,
                                         int64_t ldc, bool vec_out, const CombEpi& ce = CombEpi{},
                                         float* ep_out = nullptr) {
  constexpr int WCOLS = TN * 32;
  constexpr int kLc = WCOLS + 4;
  constexpr int kQ = WCOLS / 4;     // 4-column groups per row
  constexpr int kRS = 64 / kQ;      // rows between a lane's consecutive rows
  constexpr int kJ = 32 / kRS;      // rows per lane per 32-row half
  const float a_slope = EPI == 1 ? prelu[0] : 0.0f;
  float* Cw = smem + wave * 32 * kLc;
  const int c = (lane % kQ) * 4;
  const int r0 = lane / kQ;
  const int64_t col = n0 + wn * WCOLS + c;
  const int nv = col < N ? (N - col < 4 ? (int)(N - col) : 4) : 0;
  const bool full = vec_out && nv == 4;
  float bcol[4] = {0.f, 0.f, 0.f, 0.f};
  float ep = 0.0f;                                   // EPI 4: this lane's eps-gradient partial
  const float sc_self = EPI == 4 ? __fadd_rn(1.0f, ce.eps[0]) : 0.0f;
  const bool self_cols = EPI == 4 && col >= ce.cs && nv > 0;   // col, cs multiples of 4: whole group
  const OutT* xd = static_cast<const OutT*>(ce.xd);
  OutT* gd = static_cast<OutT*>(ce.gd);
  const OutT* gp = static_cast<const OutT*>(ce.gp);
  if (EPI == 1 || EPI == 2) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < nv) bcol[t] = bias[col + t];
  }
  __syncthreads();   // every wave is done with the A/B tiles
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
    typename Out4<OutT>::raw acc_raw[kJ];
    typename Out4<OutT>::raw prev_raw[EPI == 4 ? kJ : 1];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {   // accum (EPI 1) / x_dst, g_prev (EPI 4) rows: loaded before the LDS round trip
      acc_raw[j] = {};
      const int64_t row = m0 + wm * 64 + tm * 32 + r0 + kRS * j;
      if (EPI == 1 && accum && row < M && nv)
        acc_raw[j] = ce.nt_io ? Out4<OutT>::ld_raw_nt(accum + row * ldc + col, full, nv)
                              : Out4<OutT>::ld_raw(accum + row * ldc + col, full, nv);
      if (EPI == 4 && self_cols && row < M)
        acc_raw[j] = ce.nt_io ? Out4<OutT>::ld_raw_nt(xd + row * ce.ldxd + (col - ce.cs), full, nv)
                              : Out4<OutT>::ld_raw(xd + row * ce.ldxd + (col - ce.cs), full, nv);
      if constexpr (EPI == 4) {
        prev_raw[j] = {};
        if (gp && gd && self_cols && row < M)
          prev_raw[j] = ce.nt_io ? Out4<OutT>::ld_raw_nt(gp + row * ce.ldgp + (col - ce.cs), full, nv)
                                 : Out4<OutT>::ld_raw(gp + row * ce.ldgp + (col - ce.cs), full, nv);
      }
    }
    park_acc(acc, Cw, kLc, tm, lane);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int r = r0 + kRS * j;
      const int64_t row = m0 + wm * 64 + tm * 32 + r;
      if (row >= M || nv == 0) continue;
      const float4 v4 = *reinterpret_cast<const float4*>(Cw + r * kLc + c);
      float o[4] = {v4.x, v4.y, v4.z, v4.w};
      float zz[4] = {0.f, 0.f, 0.f, 0.f};
      float acc_in[4];
      Out4<OutT>::unpack(acc_raw[j], acc_in);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (EPI == 2) {
          o[t] = __fadd_rn(o[t], bcol[t]);
        } else if (EPI == 1) {
          zz[t] = __fadd_rn(o[t], bcol[t]);
          const float y = zz[t] > 0.0f ? zz[t] : __fmul_rn(a_slope, zz[t]);
          o[t] = accum ? __fadd_rn(acc_in[t], y) : y;
        }
      }
      if (ce.nt_io) {
        Out4<OutT>::st_nt(Y + row * ldc + col, o, full, nv);
        if (EPI == 1 && Z) Out4<OutT>::st_nt(Z + row * ldc + col, zz, full, nv);
      } else {
        Out4<OutT>::st(Y + row * ldc + col, o, full, nv);
        if (EPI == 1 && Z) Out4<OutT>::st(Z + row * ldc + col, zz, full, nv);
      }
      if (EPI == 4 && self_cols) {
        float c4[4], x4[4], g4[4], p4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t) c4[t] = Out4<OutT>::rt(o[t]);   // C as stored
        const int64_t sc = col - ce.cs;
        Out4<OutT>::unpack(acc_raw[j], x4);
        if constexpr (EPI == 4) {
          if (gp) Out4<OutT>::unpack(prev_raw[j], p4);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < nv) ep = __fadd_rn(ep, __fmul_rn(c4[t], x4[t]));
          g4[t] = __fmul_rn(sc_self, c4[t]);
          if (gp) g4[t] = __fadd_rn(p4[t], g4[t]);   // accumulate onto another relation's g_x_dst
        }
        if (gd) {
          if (ce.nt_io) Out4<OutT>::st_nt(gd + row * ce.ldgd + sc, g4, full, nv);
          else Out4<OutT>::st(gd + row * ce.ldgd + sc, g4, full, nv);
        }
      }
    }
    if (tm == 0) __syncthreads();
  }
  if (EPI == 4) *ep_out = ep;
}

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

// EPI 4: the workgroup's eps-gradient partial, a fixed tree over its 256 lanes -> part[tile]
__device__ __forceinline__ void tile_partial(float* smem, float ep, float* part, int64_t q) {
  __syncthreads();   // the epilogue's LDS staging is done
  const int t = threadIdx.x;
  smem[t] = ep;
  __syncthreads();
  for (int off = (int)blockDim.x / 2; off > 0; off >>= 1) {
    if (t < off) smem[t] = __fadd_rn(smem[t], smem[t + off]);
    __syncthreads();
  }
  if (t == 0) part[q] = smem[0];
}

// kBdma (split mode, clean tiles, N a multiple of BN): the B operand comes pre-split — hgin_nt_planes_f32's three
// bf16 planes, whose per-stage rows are already the LDS image's rows (same chunk swizzle) — and each K-tile's B
// image is copied HBM/L2 -> LDS by global_load_lds_dwordx4 (inline asm, per-lane source addresses), issued after
// the first barrier of a K-tile step and awaited (vmcnt 0) before the second: the A split pass between them hides its
// latency.  No B split VALU (a quarter of the loop's VALU at K = 512, N = 256), no B prefetch registers.
template <int EPI, bool kClean, int TN, int WNv, bool kSplit, int NW = 4, int kBdma = 0>
__global__ __launch_bounds__(NW * 64, (NW == 8 || TN == 4) ? 2 : 3) void k_gemm_nt(Src2 A, Src2 B, int64_t M, int64_t N, int64_t K,
                                                    const float* __restrict__ bias, const float* __restrict__ prelu,
                                                    const float* __restrict__ accum, float* __restrict__ Z,
                                                    float* __restrict__ Y, int64_t ldc, bool vec_out,
                                                    int64_t n_tiles, bool xcd, CombEpi ce,
                                                    const uint16_t* __restrict__ Bp = nullptr) {
  constexpr int NT = NW * 64;             // threads
  constexpr int WN = WNv;                 // waves along N
  constexpr int WM = NW / WN;             // waves along M
  constexpr int BM = WM * 64;             // rows per workgroup tile
  constexpr int BN = WN * TN * 32;        // columns per workgroup tile
  constexpr int WCOLS = TN * 32;          // columns per wave
  constexpr int kRowW = kSplit ? kSplitRowWordsNT : kLds;   // 4-B words per LDS row
  __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * kRowW];
  float* As = smem;
  float* Bs = smem + BM * kRowW;
  uint32_t* Ash = reinterpret_cast<uint32_t*>(As);
  uint32_t* Bsh = reinterpret_cast<uint32_t*>(Bs);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int li = lane & 31;
  const int lh = lane >> 5;
  // N-tiles vary fastest in the logical order and the logical order is XCD-contiguous: the workgroups
  // reading the same A rows run on one XCD, so the second N-tile finds those rows in that XCD's L2 instead
  // of streaming A from HBM again (N = 256 layers).
  const int64_t n_tiles_n = (N + BN - 1) / BN;
  const int64_t q = xcd ? xcd_logical(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  if (q >= n_tiles) return;
  const int64_t m0 = (q / n_tiles_n) * BM;
  const int64_t n0 = (q % n_tiles_n) * BN;

  f32x16 acc[2][TN];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  float4 ra[BM / (NT / 8)], rb[(BN >= NT / 8 && !kBdma) ? BN / (NT / 8) : 1];
  const float sc2 = self_scale(A.eps2);
  bool scale_a = false;   // ra holds a clean p2 tile still to be scaled by sc2
  auto load_a = [&](int64_t k0) {
    load_tile<kClean, BM, NT>(ra, A, m0, M, k0, K, tid, sc2);
    scale_a = kClean && A.eps2 != nullptr && k0 >= A.k1;
  };
  constexpr int kBChunks = BN * kSplitRowWordsNT / 4;       // 16-B chunks of the B image
  constexpr int kBInst = kBdma ? kBChunks / 64 / NW : 1;    // LDS-DMA instructions per wave per K-tile
  static_assert(!kBdma || (kSplit && kClean && kBChunks % (64 * NW) == 0), "kBdma shape");
  uint32_t boff[kBInst];   // byte offset of this lane's chunk inside one stage of the planes
  if constexpr (kBdma) {
#pragma unroll
    for (int i = 0; i < kBInst; ++i) {
      const int j = (wave * kBInst + i) * 64 + lane;        // image chunk: row j / 12, word group j % 12
      const int rr = j / 12, w = j % 12;
      boff[i] = (uint32_t)((((w >> 2) * N + n0 + rr) * 64) + (w & 3) * 16);
    }
  }
  auto dma_b = [&](int64_t k0) {
    if constexpr (kBdma) {
      const char* base = reinterpret_cast<const char*>(Bp) + (k0 / kBK) * 3 * N * 64;
      char* dst = reinterpret_cast<char*>(Bsh);
#pragma unroll
      for (int i = 0; i < kBInst; ++i) glds16_asm(base + boff[i], dst + (wave * kBInst + i) * 1024);
    }
  };
  auto stage = [&]() {
    if (scale_a) scale_tile<BM, NT>(ra, sc2);
    if constexpr (kSplit) {
      store_tile_split<BM, NT>(Ash, ra, tid);
      if constexpr (!kBdma) store_tile_split<BN, NT>(Bsh, rb, tid);
    } else {
      store_tile<BM, NT>(As, ra, tid);
      store_tile<BN, NT>(Bs, rb, tid);
    }
  };
  load_a(0);
  if constexpr (kBdma) dma_b(0);
  else load_tile<kClean, BN, NT>(rb, B, n0, N, 0, K, tid);
  stage();
  if constexpr (kBdma) wait_vm<0>();
  __syncthreads();
  for (int64_t k0 = 0; k0 < K; k0 += kBK) {
    const bool more = k0 + kBK < K;
    if (more) {   // next K-tile's global loads stay in flight under this K-tile's MFMAs
      load_a(k0 + kBK);
      if constexpr (!kBdma) load_tile<kClean, BN, NT>(rb, B, n0, N, k0 + kBK, K, tid);
    }
    const uint32_t* Bcur = Bsh;
    __builtin_amdgcn_s_setprio(1);   // keep the MFMA cluster together (T5)
    if constexpr (kSplit) {
      // two 16-deep k-blocks; lane (i, h) reads k = 16 kb + 8 h .. +7 of each plane (one ds_read_b128)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        bf16x8 fa[2][3];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fa[t][p] = *reinterpret_cast<const bf16x8*>(Ash + (wm * 64 + t * 32 + li) * kSplitRowWordsNT + p * 16 +
                                                        nt_chunk(li, kb * 2 + lh));
        // B fragments one 32-column block at a time (TN = 4: 12 instead of 48 fragment VGPRs live); per accumulator
        // the same six products in the same order
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          bf16x8 fb[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[p] = *reinterpret_cast<const bf16x8*>(Bcur + (wn * WCOLS + tn * 32 + li) * kSplitRowWordsNT + p * 16 +
                                                     nt_chunk(li, kb * 2 + lh));
#pragma unroll
          for (int tm = 0; tm < 2; ++tm) {   // smallest terms first
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][2], fb[0], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[1], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[2], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[0], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[1], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[0], acc[tm][tn], 0, 0, 0);
          }
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < kBK / 8; ++c) {
        float4 fa[2], fb[TN];
#pragma unroll
        for (int t = 0; t < 2; ++t)
          fa[t] = *reinterpret_cast<const float4*>(As + (wm * 64 + t * 32 + li) * kLds + c * 8 + lh * 4);
#pragma unroll
        for (int t = 0; t < TN; ++t)
          fb[t] = *reinterpret_cast<const float4*>(Bs + (wn * WCOLS + t * 32 + li) * kLds + c * 8 + lh * 4);
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) {
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].x, fb[tn].x, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].y, fb[tn].y, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].z, fb[tn].z, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].w, fb[tn].w, acc[tm][tn], 0, 0, 0);
          }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      __syncthreads();
      if constexpr (kBdma) dma_b(k0 + kBK);
      stage();
      if constexpr (kBdma) wait_vm<0>();
      __syncthreads();
    }
  }

  float ep = 0.0f;
  epilogue<EPI, TN, float>(acc, smem, wave, wm, wn, lane, li, lh, m0, n0, M, N, bias, prelu, accum, Z, Y, ldc,
                           vec_out, ce, &ep);
  if constexpr (EPI == 4) tile_partial(smem, ep, ce.part, q);
}

// HGIN_NT_BDMA=0: the 128 x 128 split-mode tile splits B itself even where pre-split planes are passed
bool nt_bdma_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_NT_BDMA");
    return !(v && v[0] == '0');
  }();
  return on;
}

// The split-mode tile at N a multiple of 256 as 128 x 256 (4 waves of 64 x 128, 128 accumulator VGPRs each) at two
// workgroups per CU (A split once per 256 columns: half the split VALU per MFMA of the 128 x 128 tile): the first
// layer's K = 512 forward at M = 6M 9.61 -> 9.38 ms, with accum 10.18 -> 10.03 ms (profiles/r04/gpu_a/gemm_ab_*.json);
// bit-identical (tests/test_gpu_gemm_switch.py).  HGIN_NT_T256=0 keeps the 128 x 128 tile.
constexpr bool nt_t256_enabled() { return true; }

template <int EPI, int TN, int WN, int NW = 4>
int64_t launch_nt_tn(bool vec, const Src2& a, const Src2& b, int64_t M, int64_t N, int64_t K, const float* bias,
                     const float* prelu, const float* accum, float* z, float* y, int64_t ldc, bool vec_out,
                     hipStream_t s, const CombEpi& ce, const void* planes = nullptr) {
  constexpr int BM = (NW / WN) * 64;
  constexpr int BN = WN * TN * 32;
  const int64_t tiles = ceil_div(N, BN) * ceil_div(M, BM);
  const bool xcd = xcd_remap_enabled();
  dim3 grid((unsigned)(xcd ? round_up8(tiles) : tiles));
  if constexpr (TN == 2 && WN == 2 && NW == 4) {
    if (planes && vec && gemm_split_enabled() && N % 256 == 0 && nt_bdma_enabled() && nt_t256_enabled() &&
        (int64_t)N * K * 6 < (int64_t(1) << 32)) {
      const int64_t t2 = (N / 256) * ceil_div(M, 128);
      dim3 g2((unsigned)(xcd ? round_up8(t2) : t2));
      HGIN_TRACE("k_gemm_nt<EPI%d,128x256,split_bdma,N%lld,K%lld>", EPI, (long long)N, (long long)K);
      k_gemm_nt<EPI, true, 4, 2, true, 4, 1><<<g2, 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z, y, ldc,
                                                                  vec_out, t2, xcd, ce,
                                                                  static_cast<const uint16_t*>(planes));
      return t2;
    }
    if (planes && vec && gemm_split_enabled() && N % BN == 0 && nt_bdma_enabled() &&
        (int64_t)N * K * 6 < (int64_t(1) << 32)) {
      HGIN_TRACE("k_gemm_nt<EPI%d,%dx%d,split_bdma,N%lld,K%lld>", EPI, BM, BN, (long long)N, (long long)K);
      k_gemm_nt<EPI, true, 2, 2, true, 4, 1><<<grid, 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z, y, ldc,
                                                                  vec_out, tiles, xcd, ce,
                                                                  static_cast<const uint16_t*>(planes));
      return tiles;
    }
  }
  HGIN_TRACE("k_gemm_nt<EPI%d,%dx%d,%s,N%lld,K%lld>", EPI, (NW / WN) * 64, WN * TN * 32,
             gemm_split_enabled() ? "split" : "mfma32", (long long)N, (long long)K);
#define HGIN_NT_F32(CLEAN, SPLIT)                                                                           \
  k_gemm_nt<EPI, CLEAN, TN, WN, SPLIT, NW><<<grid, NW * 64, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z, y, ldc, \
                                                                    vec_out, tiles, xcd, ce, nullptr)
  if (gemm_split_enabled()) {
    if (vec) HGIN_NT_F32(true, true); else HGIN_NT_F32(false, true);
  } else {
    if (vec) HGIN_NT_F32(true, false); else HGIN_NT_F32(false, false);
  }
#undef HGIN_NT_F32
  return tiles;
}

// Resident workgroups of a kernel across the device (occupancy x CUs), queried once per kernel.
template <typename F>
int64_t resident_slots(F kernel) {
  int per_cu = 0, dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0)
    return 768;
  return (int64_t)per_cu * prop.multiProcessorCount;
}

// Row-tile height for N > 32.  A launch runs in "rounds" of resident
// workgroups and its last round is usually partly empty (cfg2: 782 tiles of 128 rows on 768 slots = two
// rounds for 1.02 rounds of work); 64-row tiles halve the granularity.  Pick the height with the smaller
// estimated time = rounds x relative tile time.  Measured (profiles/r01_gemm_bm64.txt): a 64-row tile costs
// ~0.73 of a 128-row one (4 vs 3 resident per CU, half the rows, but 1.5x the B-tile and LDS traffic per
// MFMA); kRel64 = 0.8 keeps 128 unless the round count drops clearly (M = 100k: 100.6 -> 90.3 us, -10 %).
template <int EPI>
bool use_bm64(int64_t M, int64_t N) {
  static const int64_t slots128 = gemm_split_enabled() ? resident_slots(k_gemm_nt<EPI, true, 2, 2, true>)
                                                       : resident_slots(k_gemm_nt<EPI, true, 2, 2, false>);
  static const int64_t slots64 = gemm_split_enabled() ? resident_slots(k_gemm_nt<EPI, true, 1, 4, true>)
                                                      : resident_slots(k_gemm_nt<EPI, true, 1, 4, false>);
  constexpr double kRel64 = 0.8;
  const int64_t nt = ceil_div(N, 128);
  const double t128 = (double)ceil_div(nt * ceil_div(M, 128), slots128);
  const double t64 = (double)ceil_div(nt * ceil_div(M, 64), slots64) * kRel64;
  return t64 < t128;
}

// Non-temporal epilogue streams (HGIN_GEMM_NT_IO = 0 / 1 forces; default: once the output stream exceeds
// 512 MiB, as the aggregate's streams — outputs read back only by later kernels, far beyond the caches).
bool gemm_nt_io(int64_t M, int64_t N, int64_t elem) {
  return M * N * elem > (int64_t(512) << 20);
}

template <int EPI>
int launch_nt(const Src2& a, const Src2& b, int64_t M, int64_t N, int64_t K, const float* bias, const float* prelu,
              const float* accum, float* z, float* y, int64_t ldc, hipStream_t s, const char* what,
              const CombEpi& ce_in = CombEpi{}, int64_t* tiles_out = nullptr, const void* planes = nullptr) {
  CombEpi ce = ce_in;
  ce.nt_io = gemm_nt_io(M, N, 4);
  const bool vec = K % kBK == 0 && a.k1 % kBK == 0 && aligned16(a.p1) && a.ld1 % 4 == 0 &&
                   (a.k1 == K || (aligned16(a.p2) && a.ld2 % 4 == 0)) && aligned16(b.p1) && b.ld1 % 4 == 0;
  const bool vec_out = ldc % 4 == 0 && aligned16(y) && (z == nullptr || aligned16(z)) &&
                       (accum == nullptr || aligned16(accum)) &&
                       (EPI != 4 || (aligned16(ce.xd) && ce.ldxd % 4 == 0 &&
                                     (ce.gd == nullptr || (aligned16(ce.gd) && ce.ldgd % 4 == 0))));
  int64_t tiles;
  // (an 8-wave 128 x 128 tile, 64 x 32 per wave at 4 waves / SIMD — launch_nt_tn<EPI, 1, 4, 8> — measured 5 %
  // slower than this 4-wave tile at the cfg3 shapes: profiles/r02/gemm_pmc_cfg3.txt)
  if (N <= 32)
    tiles = launch_nt_tn<EPI, 1, 1>(vec, a, b, M, N, K, bias, prelu, accum, z, y, ldc, vec_out, s, ce);
  else if (use_bm64<EPI == 4 ? 0 : EPI>(M, N))
    tiles = launch_nt_tn<EPI, 1, 4>(vec, a, b, M, N, K, bias, prelu, accum, z, y, ldc, vec_out, s, ce);
  else
    tiles = launch_nt_tn<EPI, 2, 2>(vec, a, b, M, N, K, bias, prelu, accum, z, y, ldc, vec_out, s, ce, planes);
  if (tiles_out) *tiles_out = tiles;
  return check_launch(what);
}

int check_a(const char* what, const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2, int64_t K) {
  HGIN_ARG_CHECK(k1 >= 0 && k1 <= K, "%s: k1 out of [0, K]", what);
  HGIN_ARG_CHECK(k1 == 0 || (a1 && lda1 >= k1), "%s: bad A1", what);
  HGIN_ARG_CHECK(k1 == K || (a2 && lda2 >= K - k1), "%s: bad A2", what);
  return HGIN_OK;
}

// ---------------------------------------------------------------------------------------------------
// bf16 operands (cfg5): v_mfma_f32_32x32x16_bf16, fp32 accumulate.  Same workgroup tiles, wave grid,
// register prefetch and LDS-staged epilogue as the fp32 kernel; a K-tile is 64 bf16 (128 B per row, so
// the [row][72] LDS image has the fp32 kernel's 144-B row stride and its conflict-free ds_read_b128).
// Operand maps (gfx950): lane (r = l & 31, h = l >> 5) holds A[row r][k = 8h + j] and B[k = 8h + j][col r],
// j = 0..7, per 16-wide k-step: one ds_read_b128 per fragment.  C/D map as the f32 MFMA.
// At the GIN shapes (K = 128..512, N = 128..256) these GEMMs are HBM-bound (A read once, Y/Z written
// once: ~43 flop/B at K = 256, N = 128, far below the bf16 MFMA ridge), so the tile keeps the whole of N
// per workgroup where it can and the epilogue writes 8-B bf16 quads.
// LDS-DMA (global_load_lds_dwordx4: 64 lanes x 16 B into 1 KiB at a wave-uniform LDS address) and counted
// vector-memory waits, used by k_ws_bf16.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}


constexpr int kBKh = 64;

struct Src2h {
  const uint16_t* p1;
  int64_t ld1;
  const uint16_t* p2;
  int64_t ld2;
  int64_t k1;
  const float* eps2 = nullptr;   // as Src2::eps2 (fp32 product of the bf16 value, rounded once to bf16)
};

// bf16 twin of load_tile (8 elements = 16 B per thread and row; kClean as there, at kBKh granularity).
__device__ __forceinline__ uint32_t scale_bf2(uint32_t w, float sc) {
  return pack_bf2(__fmul_rn(sc, bf_lo(w)), __fmul_rn(sc, bf_hi(w)));
}

// A K-tile of BKH bf16 per row: BKH / 8 threads per row (16 B each), 256 / (BKH / 8) rows per pass.
template <int BKH>
struct TileH {
  static constexpr int kTpr = BKH / 8;        // threads per row
  static constexpr int kRp = 256 / kTpr;      // rows per pass
  static constexpr int kLd = BKH + 8;         // LDS row stride (bf16): 80 B / 144 B / 272 B, all conflict-free
};

template <bool kClean, int ROWS, int BKH = kBKh>
__device__ __forceinline__ void load_tile_h(uint4 (&r)[ROWS / TileH<BKH>::kRp], const Src2h& s, int64_t row0,
                                            int64_t rows, int64_t k0, int64_t K, int tid, float sc2 = 1.0f) {
  constexpr int TPR = TileH<BKH>::kTpr, RP = TileH<BKH>::kRp;
  if constexpr (kClean) {
    // select between the loaded VALUES: a select between the two struct fields' addresses would make
    // the compiler copy the by-value kernel argument into scratch
    const bool first = k0 < s.k1;
    const uintptr_t u1 = reinterpret_cast<uintptr_t>(s.p1), u2 = reinterpret_cast<uintptr_t>(s.p2);
    const int64_t l1 = s.ld1, l2 = s.ld2;
    const uint16_t* base = reinterpret_cast<const uint16_t*>(first ? u1 : u2);
    const int64_t ld = first ? l1 : l2;
    const int64_t kk = (first ? k0 : k0 - s.k1) + (tid % TPR) * 8;
#pragma unroll
    for (int i = 0; i < ROWS / RP; ++i) {
      int64_t gr = row0 + (tid / TPR) + RP * i;
      gr = gr < rows ? gr : rows - 1;
      const uint4 v = *reinterpret_cast<const uint4*>(base + gr * ld + kk);
      r[i] = v;
    }
    // (eps2 scaling of a clean p2 tile is applied when the tile is staged: scale_tile_h)
  } else {
    const int64_t kk = k0 + (tid % TPR) * 8;
#pragma unroll
    for (int i = 0; i < ROWS / RP; ++i) {
      const int64_t gr = row0 + (tid / TPR) + RP * i;
      uint32_t t[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      if (gr < rows) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int64_t k = kk + c;
          t[c] = k < K ? (k < s.k1 ? s.p1[gr * s.ld1 + k]
                                   : (s.eps2 ? f2bf(__fmul_rn(sc2, bf2f(s.p2[gr * s.ld2 + (k - s.k1)])))
                                             : (uint32_t)s.p2[gr * s.ld2 + (k - s.k1)]))
                       : 0u;
        }
      }
      r[i] = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
    }
  }
}

template <int ROWS, int BKH = kBKh>
__device__ __forceinline__ void store_tile_h(uint16_t* __restrict__ dst, const uint4 (&r)[ROWS / TileH<BKH>::kRp],
                                             int tid) {
  constexpr int TPR = TileH<BKH>::kTpr, RP = TileH<BKH>::kRp, LD = TileH<BKH>::kLd;
#pragma unroll
  for (int i = 0; i < ROWS / RP; ++i)
    *reinterpret_cast<uint4*>(dst + ((tid / TPR) + RP * i) * LD + (tid % TPR) * 8) = r[i];
}

template <int EPI, bool kClean, int TN, int WNv, typename OutT, int BKH = kBKh>
__global__ __launch_bounds__(256, BKH <= 64 ? 3 : 2) void k_gemm_nt_bf16(Src2h A, Src2h B, int64_t M, int64_t N, int64_t K,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ prelu,
                                                         const OutT* __restrict__ accum, OutT* __restrict__ Z,
                                                         OutT* __restrict__ Y, int64_t ldc, bool vec_out,
                                                         int64_t n_tiles, bool xcd, CombEpi ce) {
  constexpr int WN = WNv;
  constexpr int WM = 4 / WN;
  constexpr int BM = WM * 64;
  constexpr int BN = WN * TN * 32;
  constexpr int WCOLS = TN * 32;
  constexpr int LDH = TileH<BKH>::kLd;
  constexpr int RPH = TileH<BKH>::kRp;
  constexpr int kTileBytes = (BM + BN) * LDH * 2;
  constexpr int kEpiBytes = 4 * 32 * (WCOLS + 4) * 4;
  __shared__ __attribute__((aligned(16))) float smem[(kTileBytes > kEpiBytes ? kTileBytes : kEpiBytes) / 4];
  uint16_t* As = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Bs = As + BM * LDH;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int64_t n_tiles_n = (N + BN - 1) / BN;
  const int64_t q = xcd ? xcd_logical(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  if (q >= n_tiles) return;
  const int64_t m0 = (q / n_tiles_n) * BM;
  const int64_t n0 = (q % n_tiles_n) * BN;

  f32x16 acc[2][TN];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  uint4 ra[BM / RPH], rb[BN >= RPH ? BN / RPH : 1];
  const float sc2 = self_scale(A.eps2);
  bool scale_a = false;   // ra holds a clean p2 tile still to be scaled (at staging time, as the fp32 kernel)
  auto load_a = [&](int64_t k0) {
    load_tile_h<kClean, BM, BKH>(ra, A, m0, M, k0, K, tid, sc2);
    scale_a = kClean && A.eps2 != nullptr && k0 >= A.k1;
  };
  auto scale_a_tile = [&]() {
    if (scale_a) {
#pragma unroll
      for (int i = 0; i < BM / RPH; ++i)
        ra[i] = make_uint4(scale_bf2(ra[i].x, sc2), scale_bf2(ra[i].y, sc2), scale_bf2(ra[i].z, sc2),
                           scale_bf2(ra[i].w, sc2));
    }
  };
  load_a(0);
  load_tile_h<kClean, BN, BKH>(rb, B, n0, N, 0, K, tid);
  scale_a_tile();
  store_tile_h<BM, BKH>(As, ra, tid);
  store_tile_h<BN, BKH>(Bs, rb, tid);
  __syncthreads();
  for (int64_t k0 = 0; k0 < K; k0 += BKH) {
    const bool more = k0 + BKH < K;
    if (more) {
      load_a(k0 + BKH);
      load_tile_h<kClean, BN, BKH>(rb, B, n0, N, k0 + BKH, K, tid);
    }
    __builtin_amdgcn_s_setprio(1);   // keep the MFMA cluster together (T5)
#pragma unroll
    for (int c = 0; c < BKH / 16; ++c) {
      bf16x8 fa[2], fb[TN];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        fa[t] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + t * 32 + li) * LDH + c * 16 + lh * 8);
#pragma unroll
      for (int t = 0; t < TN; ++t)
        fb[t] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WCOLS + t * 32 + li) * LDH + c * 16 + lh * 8);
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      __syncthreads();
      scale_a_tile();
      store_tile_h<BM, BKH>(As, ra, tid);
      store_tile_h<BN, BKH>(Bs, rb, tid);
      __syncthreads();
    }
  }

  float ep = 0.0f;
  epilogue<EPI, TN, OutT>(acc, smem, wave, wm, wn, lane, li, lh, m0, n0, M, N, bias, prelu, accum, Z, Y, ldc,
                          vec_out, ce, &ep);
  if constexpr (EPI == 4) tile_partial(smem, ep, ce.part, q);
}

template <int EPI, typename OutT>
bool use_bm64_bf16(int64_t M, int64_t N) {
  static const int64_t slots128 = resident_slots(k_gemm_nt_bf16<EPI, true, 2, 2, OutT>);
  static const int64_t slots64 = resident_slots(k_gemm_nt_bf16<EPI, true, 1, 4, OutT>);
  constexpr double kRel64 = 0.8;
  const int64_t nt = ceil_div(N, 128);
  const double t128 = (double)ceil_div(nt * ceil_div(M, 128), slots128);
  const double t64 = (double)ceil_div(nt * ceil_div(M, 64), slots64) * kRel64;
  return t64 < t128;
}

// ---------------------------------------------------------------------------------------------------
// k_ws_bf16 — weight-stationary streaming form of the bf16 NT GEMM for the GIN MLP shapes (K = 128 / 256 /
// 512, N = 128 / 256: the layer GEMMs of cfg5).  These GEMMs are HBM-bound (A read once, z / y written,
// accum read: ~200 flop/B at K = 512), and the tiled kernel above streams A twice per row block (two 128-col
// tiles, the second from L2) with one register-staged K-tile in flight per workgroup: ~4 TB/s.  Here:
//   * one persistent workgroup per CU (two where ws_wpc says so), N / 32 waves; wave w keeps
//     W[32 w .. 32 w + 31][0 .. K) in registers as its MFMA B fragments for the whole launch (K / 16 x 16 B
//     per lane: 128 VGPRs at K = 512), so W is read once per CU and A exactly once from HBM;
//   * the A rows of a 32-row block (64 at K = 128) and the block's accum rows stream HBM -> LDS with
//     global_load_lds_dwordx4 into an NST-deep ring (NST - 1 blocks in flight while one is computed), with
//     counted vmcnt waits and raw s_barriers: the loop has no VGPR-destination global load, so nothing in it
//     makes the compiler drain the ring (cdna_hip_programming.md §5, "Pipelining across barriers");
//   * every wave multiplies the whole block by its W slice (v_mfma_f32_32x32x16_bf16, the per-accumulator
//     k order of k_gemm_nt_bf16: bit-identical results), then the fp32 results are staged 16 rows at a time
//     through the block's dead A image and written as row-contiguous 8-B bf16 quads (bias, PReLU, accum from
//     the LDS copy), the same epilogue arithmetic as epilogue<1 / 2>;
//   * an eps-scaled second source (the first layer's concat self term, Src2h::eps2) is scaled in the block's
//     LDS image once, before the MFMAs (bf16(s * v), the tiled kernel's staging arithmetic).
// LDS images (16-B chunks): A row r of the block at r * 2K bytes, logical chunk c stored at slot c ^ (r & 15)
// (the DMA lanes fetch pre-swizzled sources; a ds_read_b128 group of 16 rows hits 16 distinct bank slots);
// accum rows linear; fp32 staging [16][N] with column bit 5 flipped on rows with bit 2 set (the two lane halves
// of an accumulator store hit opposite bank halves).
template <int K, int N, int CPW = 32>
struct WsCfg {
  static constexpr int NW = N / CPW;                    // waves (one CPW-column W slice each)
  static constexpr int NT = NW * 64;
  static constexpr int TN = CPW / 32;                   // 32-column MFMA tiles per wave
  static constexpr int RPP = NT / (N / 4);              // epilogue rows per pass (a thread per 4-column group)
  static constexpr int KS = K / 16;                     // MFMA k-steps
  static constexpr int BM = K >= 256 ? 32 : 64;         // rows per block (A image >= 16 KB: the staging area)
  static constexpr int TM = BM / 32;
  static constexpr int ROWB = K * 2;
  static constexpr int A_BYTES = BM * ROWB;
  static constexpr int C_BYTES = BM * N * 2;
  static constexpr int SLOT_A = A_BYTES;                // accum image follows the A image in a slot
  static constexpr int PA = A_BYTES / 1024 / NW;        // DMA pieces per wave per block
  static constexpr int PC = C_BYTES / 1024 / NW;
  static_assert(A_BYTES % (1024 * NW) == 0 && C_BYTES % (1024 * NW) == 0, "DMA pieces");
  static_assert(16 * N * 4 <= A_BYTES, "staging fits the A image");
  static_assert((A_BYTES / 16) % NT == 0, "eps-scaling pass");
};

// Workgroups per CU: two at 64 columns per wave (below) and for the readout's K = 512, N = 128 forward (4-wave
// workgroups: one per CU left each SIMD a single wave)
template <int K, int N, int CPW>
constexpr int ws_wpc() {
  return (CPW == 64 || (K == 512 && N == 128)) ? 2 : 1;
}

template <int K, int N, int NIMG, int CPW = 32>
struct WsRing {
  static constexpr int SLOT = WsCfg<K, N, CPW>::A_BYTES + NIMG * WsCfg<K, N, CPW>::C_BYTES;
  // ring depth: as deep as 144 KB of LDS allows (80 KB with two workgroups per CU), up to 4 (0: does not fit,
  // the tiled kernel is used)
  static constexpr int CAP = ws_wpc<K, N, CPW>() == 2 ? 81920 : 147456;
  static constexpr int NST = SLOT * 4 <= CAP ? 4 : SLOT * 3 <= CAP ? 3 : SLOT * 2 <= CAP ? 2 : 0;
  static constexpr int BYTES = SLOT * (NST > 0 ? NST : 1);
};

// Operands of one weight-stationary launch.  Row images (bf16 [M, N] rows streamed beside A, read by the
// epilogue from LDS): r1 = accum (EPI 1) / x_dst (EPI 4); r2 = g_prev (EPI 4).  Outputs: Y = y (EPI 1) / C (EPI 0,
// 4); Z = z (EPI 1) / g_x_dst (EPI 4).
struct WsArgs {
  const uint16_t* a1;
  int64_t lda1;
  const uint16_t* a2;
  int64_t lda2;
  int64_t k1;
  const float* eps2;
  const uint16_t* w;
  const float* bias;
  const float* prelu;
  const uint16_t* r1;
  int64_t ldr1;
  const uint16_t* r2;
  int64_t ldr2;
  uint16_t* y;
  int64_t ldy;
  uint16_t* z;
  int64_t ldz;
  const float* eps;   // EPI 4: the GIN eps (self term scale 1 + eps)
  float* part;        // EPI 4: one eps-gradient partial per workgroup
  int64_t M;
  bool nt_io;
  bool nt_in;
  bool zy = false;    // EPI 1, z kept, no accum: skip the z stores when prelu[0] > 0 (z is then recoverable from y)
};

// Operands of one fp32 weight-stationary forward launch (k_ws_f32, below).
struct WsArgs32 {
  const float* a;
  int64_t lda;
  const float* w;
  const float* bias;
  const float* prelu;
  const float* r1;     // EPI 1: accum (row stride N); EPI 4: x_dst
  int64_t ldr1;
  const float* r2;     // EPI 4: g_prev (DMA'd into the block's dead A slot)
  int64_t ldr2;
  float* z;            // EPI 1: z; EPI 4: g_x_dst
  int64_t ldz;
  float* y;            // EPI 1: y; EPI 4: C = g_comb
  int64_t ldy;
  const float* eps;    // EPI 4: the GIN eps
  float* part;         // EPI 4: one eps-gradient partial per workgroup
  int64_t M;
  bool nt_io;
  bool nt_in;
  int64_t ldw = 0;             // W row stride (0: K) — k_wss_f32's K = 512 halves read W[:, 0:256] / W[:, 256:512]
  const float* eps2 = nullptr; // k_wss_f32 kScale: A is scaled by 1 + eps2[0] before the split (the concat self term)
};

template <int K, int N, int EPI, bool kR1, bool kZ, bool kR2, int CPW = 32>
__global__ __launch_bounds__((WsCfg<K, N, CPW>::NT), (ws_wpc<K, N, CPW>())) void k_ws_bf16(WsArgs g) {
  using C = WsCfg<K, N, CPW>;
  constexpr int NIMG = (kR1 ? 1 : 0) + (kR2 ? 1 : 0);
  using R = WsRing<K, N, NIMG, CPW>;
  constexpr int NST = R::NST;
  constexpr int P = C::PA + NIMG * C::PC;                        // DMA instructions per wave per block
  constexpr int NPASS = 16 / C::RPP;                             // epilogue passes per 16-row half
  constexpr int S = C::TM * 2 * NPASS * (kZ ? 2 : 1);            // stores per lane per block
  constexpr int S0 = C::TM * 2 * NPASS;                          // ... when the z stores are skipped (zy)
  constexpr int QPR = N / 4;                                     // 4-column groups per row
  constexpr int kWaitSteady = (NST - 2) * P + (NST - 1) * S < 63 ? (NST - 2) * P + (NST - 1) * S : 63;
  constexpr int kWaitSteady0 = (NST - 2) * P + (NST - 1) * S0 < 63 ? (NST - 2) * P + (NST - 1) * S0 : 63;
  constexpr int kWaitEarly = (NST - 2) * P < 63 ? (NST - 2) * P : 63;
  extern __shared__ __attribute__((aligned(16))) char ws_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int64_t M = g.M;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;             // blocks blockIdx.x + i G, i < my

  // this wave's W slice as B fragments: lane (li, lh) holds W[CPW wave + 32 tn + li][16 t + 8 lh .. + 7]
  uint4 wf[C::TN][C::KS];
#pragma unroll
  for (int tn = 0; tn < C::TN; ++tn) {
    const uint16_t* wr = g.w + (int64_t)(wave * CPW + tn * 32 + li) * K + lh * 8;
#pragma unroll
    for (int t = 0; t < C::KS; ++t) wf[tn][t] = *reinterpret_cast<const uint4*>(wr + t * 16);
  }
  // row-pass columns of this thread (fixed), bias, PReLU slope, eps scales
  const int cq = (tid % QPR) * 4;
  const int rq = tid / QPR;                                      // row within an 8-row pass
  float bcol[4] = {0.f, 0.f, 0.f, 0.f};
  if (EPI == 1 || EPI == 2) {
#pragma unroll
    for (int t = 0; t < 4; ++t) bcol[t] = g.bias[cq + t];
  }
  const float a_slope = EPI == 1 ? g.prelu[0] : 0.0f;
  const float sc_self = EPI == 4 ? __fadd_rn(1.0f, g.eps[0]) : 0.0f;
  // zy (bf16 forward without accum, y = prelu(z) exactly): with a positive slope, z > 0 <=> y > 0 and z = y / a, so
  // the backward reads y instead (k_wsd_bf16 PRO's yalt) and the z stores — a third of this launch's HBM bytes — are
  // skipped; a wave-uniform branch, and the vmcnt bound of the ring counts the stores actually issued
  const bool skip_z = (EPI == 1 && kZ && !kR1) ? (g.zy && a_slope > 0.0f) : false;
  // eps-scaled second source (the first layer's concat self term): the A image's chunks with k >= k1 are
  // scaled in LDS once per block (bf16(s * v), the tiled kernel's staging arithmetic)
  const int64_t k1 = g.k1;
  const bool scale_any = g.eps2 != nullptr && k1 < K;
  const float sc2 = g.eps2 ? __fadd_rn(1.0f, g.eps2[0]) : 1.0f;
  // consume the prologue loads here, so that the compiler's own wait for them sits before the ring starts and
  // not inside the loop (where it would count the ring's DMAs)
#pragma unroll
  for (int tn = 0; tn < C::TN; ++tn)
#pragma unroll
    for (int t = 0; t < C::KS; ++t)
      asm volatile("" ::"v"(wf[tn][t].x), "v"(wf[tn][t].y), "v"(wf[tn][t].z), "v"(wf[tn][t].w));
#pragma unroll
  for (int t = 0; t < 4; ++t) asm volatile("" ::"v"(bcol[t]));

  auto dma = [&](const void* src, void* dst) {
    if (g.nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  // addresses: a block-uniform 64-bit base (row r0) plus a 32-bit per-lane offset (rows past M clamp to M - 1:
  // their products land in rows that are never stored)
  const int ki = (int)k1;
  // the thread index as an opaque value, re-read where used inside the loop: the per-lane DMA / scaling offsets
  // derived from it are then recomputed per block instead of being hoisted out of the loop into registers
  // (which spills the K = 512 kernels, whose W slice alone holds 128 VGPRs)
  auto tid_o = [&]() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto issue_rows = [&](const uint16_t* p, int64_t ld, char* img, int64_t r0, int rmax) {
    const uint16_t* pb = p + r0 * ld;
    const int lane = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < C::PC; ++q) {
      const int piece = wave * C::PC + q;
      const int off = piece * 1024 + lane * 16;
      const int r = off / (N * 2);
      dma(pb + ((r < rmax ? r : rmax) * (int)ld + (off % (N * 2)) / 2), img + piece * 1024);
    }
  };
  auto issue = [&](int64_t i) {
    char* base = ws_smem + (int)(i % NST) * R::SLOT;
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const uint16_t* b1 = g.a1 + r0 * g.lda1;
    const uint16_t* b2 = g.a2 + r0 * g.lda2;
    const int lane = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + lane * 16;
      int r = off / C::ROWB;
      const int c = ((off % C::ROWB) >> 4) ^ (r & 15);           // logical chunk stored at this slot
      r = r < rmax ? r : rmax;
      const int k = c * 8;
      dma(k < ki ? b1 + (r * (int)g.lda1 + k) : b2 + (r * (int)g.lda2 + (k - ki)), base + piece * 1024);
    }
    if constexpr (kR1) issue_rows(g.r1, g.ldr1, base + C::A_BYTES, r0, rmax);
    if constexpr (kR2) issue_rows(g.r2, g.ldr2, base + C::A_BYTES + (kR1 ? C::C_BYTES : 0), r0, rmax);
  };

#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < my) issue(i);

  float ep = 0.0f;                                               // EPI 4: this thread's eps-gradient partial
  for (int64_t i = 0; i < my; ++i) {
    // this wave's pieces of block i have landed: every younger vector-memory op may stay in flight.  Issue
    // order: DMA(i) at the top of iteration i - NST + 1, then that iteration's stores, then NST - 2 more
    // iterations of DMA + stores.  The counts are exact for full blocks; early iterations and a workgroup's
    // last blocks (the only partial block is the last) wait for more, never less.
    if (i + NST - 2 < my) {
      if (i >= NST - 1) {
        if (skip_z) wait_vm<kWaitSteady0>(); else wait_vm<kWaitSteady>();
      } else {
        wait_vm<kWaitEarly>();
      }
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();                 // every wave's pieces landed; the slot of block i-1 is free
    asm volatile("" ::: "memory");
    if (i + NST - 1 < my) issue(i + NST - 1);
    char* abase = ws_smem + (int)(i % NST) * R::SLOT;
    if (scale_any) {
      constexpr int CH = C::A_BYTES / 16;                        // 16-B chunks of the A image
      constexpr int RC = C::ROWB / 16;                           // chunks per image row
      const int tq = tid_o();
      constexpr bool kHalf = K >= 256 && (CH / 2) % C::NT == 0;
      if (kHalf && k1 == K / 2) {
        // equal halves (the concat of a 256-wide aggregate and a 256-wide x_dst): the row swizzle c ^ (r & 15) keeps
        // bit log2(RC / 2) >= 4, so the self half is exactly slots [RC / 2, RC) of every row — visit only those
#pragma unroll
        for (int q = 0; q < CH / 2 / C::NT; ++q) {
          const int j = q * C::NT + tq;
          uint4* pu = reinterpret_cast<uint4*>(abase + ((j / (RC / 2)) * RC + RC / 2 + j % (RC / 2)) * 16);
          const uint4 u = *pu;
          *pu = make_uint4(scale_bf2(u.x, sc2), scale_bf2(u.y, sc2), scale_bf2(u.z, sc2), scale_bf2(u.w, sc2));
        }
      } else {
#pragma unroll
        for (int q = 0; q < CH / C::NT; ++q) {
          const int ch = q * C::NT + tq;
          const int r = ch / RC;
          const int c = (ch % RC) ^ (r & 15);                    // logical chunk at this slot
          if (c * 8 >= k1) {
            uint4* pu = reinterpret_cast<uint4*>(abase + ch * 16);
            const uint4 u = *pu;
            *pu = make_uint4(scale_bf2(u.x, sc2), scale_bf2(u.y, sc2), scale_bf2(u.z, sc2), scale_bf2(u.w, sc2));
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int64_t ldy = EPI == 1 ? N : g.ldy, ldz = EPI == 1 ? N : g.ldz;
    uint16_t* yb = g.y + r0 * ldy;                                // block-uniform output bases
    uint16_t* zb = kZ ? g.z + r0 * ldz : nullptr;

    f32x16 acc[C::TM][C::TN];
#pragma unroll
    for (int tm = 0; tm < C::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < C::TN; ++tn)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.0f;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
#pragma unroll
      for (int tm = 0; tm < C::TM; ++tm) {
        const int r = tm * 32 + li;
        const uint4 u = *reinterpret_cast<const uint4*>(abase + r * C::ROWB + (((2 * t + lh) ^ (r & 15)) << 4));
#pragma unroll
        for (int tn = 0; tn < C::TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, u),
                                                                __builtin_bit_cast(bf16x8, wf[tn][t]), acc[tm][tn], 0,
                                                                0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    float* stg = reinterpret_cast<float*>(abase);                // the dead A image
    const uint16_t* img1 = reinterpret_cast<const uint16_t*>(abase + C::A_BYTES);
    const uint16_t* img2 = reinterpret_cast<const uint16_t*>(abase + C::A_BYTES + (kR1 ? C::C_BYTES : 0));
#pragma unroll
    for (int tm = 0; tm < C::TM; ++tm) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        __builtin_amdgcn_s_barrier();             // A image reads / the previous half's staging reads are done
        asm volatile("" ::: "memory");
#pragma unroll
        for (int tn = 0; tn < C::TN; ++tn)
#pragma unroll
          for (int e8 = 0; e8 < 8; ++e8) {
            const int e = 8 * h + e8;
            const int row = (e & 3) + 8 * ((e >> 2) & 1) + 4 * lh;        // row within the 16-row half
            stg[row * N + ((wave * CPW + tn * 32 + li) ^ (((row >> 2) & 1) << 5))] = acc[tm][tn][e];
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int pass = 0; pass < NPASS; ++pass) {
          const int row = pass * C::RPP + rq;
          const int brow = tm * 32 + h * 16 + row;                        // row within the block
          const int64_t grow = r0 + brow;
          const float4 v4 = *reinterpret_cast<const float4*>(stg + row * N + (cq ^ (((row >> 2) & 1) << 5)));
          float o[4] = {v4.x, v4.y, v4.z, v4.w};
          float zz[4] = {0.f, 0.f, 0.f, 0.f};
          float in1[4] = {0.f, 0.f, 0.f, 0.f}, in2[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (kR1) Out4<uint16_t>::unpack(*reinterpret_cast<const uint2*>(img1 + brow * N + cq), in1);
          if constexpr (kR2) Out4<uint16_t>::unpack(*reinterpret_cast<const uint2*>(img2 + brow * N + cq), in2);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (EPI == 2) {
              o[t] = __fadd_rn(o[t], bcol[t]);
            } else if (EPI == 1) {
              zz[t] = __fadd_rn(o[t], bcol[t]);
              const float y = zz[t] > 0.0f ? zz[t] : __fmul_rn(a_slope, zz[t]);
              o[t] = kR1 ? __fadd_rn(in1[t], y) : y;
            }
          }
          if (grow < M) {
            if constexpr (EPI == 4) {   // epilogue<4>'s self-term backward on C as stored (bf16-rounded)
#pragma unroll
              for (int t = 0; t < 4; ++t) {
                const float c4 = Out4<uint16_t>::rt(o[t]);
                ep = __fadd_rn(ep, __fmul_rn(c4, in1[t]));
                zz[t] = __fmul_rn(sc_self, c4);
                if (kR2) zz[t] = __fadd_rn(in2[t], zz[t]);
              }
            }
            const int oy = brow * (int)ldy + cq, oz = brow * (int)ldz + cq;
            if (g.nt_io) {
              Out4<uint16_t>::st_nt(yb + oy, o, true, 4);
              if constexpr (kZ)
                if (!skip_z) Out4<uint16_t>::st_nt(zb + oz, zz, true, 4);
            } else {
              Out4<uint16_t>::st(yb + oy, o, true, 4);
              if constexpr (kZ)
                if (!skip_z) Out4<uint16_t>::st(zb + oz, zz, true, 4);
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS reads of the slot are done
  }
  if constexpr (EPI == 4) tile_partial(reinterpret_cast<float*>(ws_smem), ep, g.part, blockIdx.x);
}

// Weight-stationary launch (HGIN_NT_WS = 0 / 1; default on) when the shape and operands allow it: N 128 / 256,
// K 128 / 256 / 512, k1 a multiple of 8, 16-B aligned rows everywhere (leading dimensions multiples of 8), W
// packed [N, K]; EPI 1 (forward MLP), EPI 0 (plain dX) and EPI 4 with the self term on every column (cs = 0).
bool ws_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_NT_WS");
    return !(v && v[0] == '0');
  }();
  return on;
}

// Non-temporal DMA of the streamed A / row-image rows (1-3 % faster at the cfg5 shapes, profiles/r02/gemm_ws_bf16.txt).
constexpr bool ws_nt_in() { return true; }

int ws_grid() {
  static const int g = [] {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    return prop.multiProcessorCount;
  }();
  return g;
}

// N = 256, K <= 256 without row images (the forward without accum, the plain dX): two 4-wave workgroups per CU, each
// wave holding 64 W columns (128 VGPRs at K = 256) — while one workgroup runs its epilogue's barriers the other's
// MFMAs run.  M = 3M, K = N = 256, bf16: 1.13 -> 1.04-1.07 ms (profiles/r06/gemm_ab_bf16.txt).  With a row image
// (accum, x_dst) the 80 KB per workgroup leave a 2-deep ring and it measured slower (1.17 -> 1.19-1.23 ms), so those
// keep 32 columns per wave and one workgroup per CU.
template <int K, int N, int EPI, bool kR1, bool kZ, bool kR2, int CPW = (N == 256 && K <= 256 && !kR1 && !kR2) ? 64 : 32>
int launch_ws_kn(const WsArgs& a, hipStream_t s, const char* what, int64_t* grid_out) {
  using Ring = WsRing<K, N, (kR1 ? 1 : 0) + (kR2 ? 1 : 0), CPW>;
  if constexpr (Ring::NST < 2) {
    return -1;
  } else {
    constexpr int lds = Ring::BYTES;
    auto kern = k_ws_bf16<K, N, EPI, kR1, kZ, kR2, CPW>;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (attr != hipSuccess) {
      set_error("%s: hipFuncSetAttribute failed: %s", what, hipGetErrorString(attr));
      return (int)attr;
    }
    const int64_t nblk = ceil_div(a.M, (int64_t)WsCfg<K, N, CPW>::BM);
    const int64_t g_max = (int64_t)ws_grid() * ws_wpc<K, N, CPW>();
    const int64_t grid = nblk < g_max ? nblk : g_max;
    HGIN_TRACE("k_ws_bf16<%d,%d,EPI%d%s>", K, N, EPI,
               CPW == 64 ? ",cpw64" : ws_wpc<K, N, CPW>() == 2 ? ",wpc2" : "");
    kern<<<(unsigned)grid, WsCfg<K, N, CPW>::NT, lds, s>>>(a);
    if (grid_out) *grid_out = grid;
    return check_launch(what);
  }
}

template <int EPI, int K, int N>
int launch_ws_epi(const WsArgs& a, hipStream_t s, const char* what, int64_t* grid_out) {
  const bool r1 = a.r1 != nullptr, z = a.z != nullptr, r2 = a.r2 != nullptr;
  if constexpr (EPI == 1) {
    if (r1 && z) return launch_ws_kn<K, N, 1, true, true, false>(a, s, what, grid_out);
    if (r1) return launch_ws_kn<K, N, 1, true, false, false>(a, s, what, grid_out);
    if (z) return launch_ws_kn<K, N, 1, false, true, false>(a, s, what, grid_out);
    return launch_ws_kn<K, N, 1, false, false, false>(a, s, what, grid_out);
  } else if constexpr (EPI == 4) {
    if (z && r2) return launch_ws_kn<K, N, 4, true, true, true>(a, s, what, grid_out);
    if (z) return launch_ws_kn<K, N, 4, true, true, false>(a, s, what, grid_out);
    return launch_ws_kn<K, N, 4, true, false, false>(a, s, what, grid_out);
  } else {
    return launch_ws_kn<K, N, EPI, false, false, false>(a, s, what, grid_out);
  }
}

// Returns -1 when the weight-stationary form does not apply (the caller launches the tiled kernel).
template <int EPI, typename OutT>
int try_ws_bf16(const Src2h& a, const Src2h& b, int64_t M, int64_t N, int64_t K, const float* bias,
                const float* prelu, const OutT* accum, OutT* z, OutT* y, int64_t ldc, const CombEpi& ce,
                hipStream_t s, const char* what, int64_t* grid_out) {
  if constexpr (!std::is_same<OutT, uint16_t>::value || !(EPI == 0 || EPI == 1 || EPI == 4)) {
    return -1;
  } else {
    if (!ws_enabled() || M < 1 || (N != 128 && N != 256) || (K != 128 && K != 256 && K != 512)) return -1;
    // (16-B aligned rows; ld < 2^24 keeps the kernel's per-lane 32-bit offsets in range within a block)
    auto ok = [](const void* p, int64_t ld) {
      return p == nullptr || (aligned16(p) && ld % 8 == 0 && ld < (int64_t(1) << 24));
    };
    if (a.k1 % 8 || b.ld1 != K || !aligned16(b.p1) || !ok(y, ldc)) return -1;
    if (a.k1 > 0 && !ok(a.p1, a.ld1)) return -1;
    if (a.k1 < K && !ok(a.p2, a.ld2)) return -1;
    WsArgs w{a.p1, a.ld1, a.p2, a.ld2, a.k1, a.eps2, b.p1, bias, prelu,
             nullptr, 0, nullptr, 0, y, ldc, nullptr, 0, nullptr, nullptr, M, ce.nt_io, ws_nt_in()};
    if constexpr (EPI == 1) {
      if (ldc != N || !ok(z, N) || !ok(accum, N)) return -1;
      w.r1 = accum;
      w.ldr1 = N;
      w.z = z;
      w.ldz = N;
      w.zy = ce.zy && z && !accum;
    } else if constexpr (EPI == 4) {
      const uint16_t* xd = static_cast<const uint16_t*>(ce.xd);
      uint16_t* gd = static_cast<uint16_t*>(ce.gd);
      const uint16_t* gp = static_cast<const uint16_t*>(ce.gp);
      if (ce.cs != 0 || !xd || !ok(xd, ce.ldxd) || !ok(gd, ce.ldgd) || !ok(gp, ce.ldgp)) return -1;
      w.r1 = xd;
      w.ldr1 = ce.ldxd;
      w.z = gd;
      w.ldz = ce.ldgd;
      w.r2 = gd ? gp : nullptr;
      w.ldr2 = ce.ldgp;
      w.eps = ce.eps;
      w.part = ce.part;
    }
#define HGIN_WS(KV, NV) \
  if (K == KV && N == NV) return launch_ws_epi<EPI, KV, NV>(w, s, what, grid_out);
    HGIN_WS(512, 256) HGIN_WS(256, 256) HGIN_WS(128, 256) HGIN_WS(512, 128) HGIN_WS(256, 128) HGIN_WS(128, 128)
#undef HGIN_WS
    return -1;
  }
}

// ---------------------------------------------------------------------------------------------------
// k_ws_f32 — the fp32 forward MLP GEMM (EPI 1) and the dX GEMM with the self-term backward (EPI 4: x_dst rows in
// the r1 buffer, g_prev rows DMA'd into the block's A slot once the split pass has consumed it), split mode, in the
// weight-stationary streaming form, for the square layers K = N = 256 (cfg3's layers above the first; an
// instantiation at K = N = 128 measured slower than the tiled kernel, 600k rows: 0.279 vs 0.243 ms, so there is
// none):
//   * N/32 waves; wave w holds the three bf16 planes of W[32 w .. 32 w + 31][0, K) in registers as its MFMA B
//     fragments (3K/4 VGPRs: 192 at K = 256), split once per launch;
//   * 32-row blocks of A (fp32) stream HBM -> LDS by DMA into a 2-slot ring (one block in flight while one is
//     computed; 3 slots measured equal); the block's accum rows are DMA'd into a single buffer at the top of its
//     own iteration (read only by its epilogue, after the split pass and the MFMAs); counted vmcnt waits as in
//     k_ws_bf16;
//   * one split pass per block turns the fp32 A image into three bf16 plane images (each element split once per
//     CU, one barrier); plane rows are 2K bytes of 16-B chunks, chunk c of row r stored at c ^ (r & SW)
//     (conflict-free fragment reads);
//   * per 16-wide k-step six v_mfma_f32_32x32x16_bf16 products in k_gemm_nt's order (smallest terms first), k
//     ascending, one accumulator per wave — the tiled kernel's per-output arithmetic, so the results are
//     bit-identical to it (tests/test_gpu_gemm_switch.py);
//   * epilogue: the 32 x N results staged at once in the dead plane images, then row-contiguous float4 stores of
//     z and y with epilogue<1>'s bias / PReLU / accum arithmetic (four barriers per block in all).
template <int K, int N>
struct Ws32Cfg {
  static constexpr int NW = N / 32;
  static constexpr int NT = NW * 64;
  static constexpr int KS = K / 16;
  static constexpr int BM = 32;
  static constexpr int A_BYTES = BM * K * 4;          // fp32 image; later planes 0 and 1 (BM * K * 2 each)
  static constexpr int C_BYTES = BM * N * 4;          // accum image
  static constexpr int PL = BM * K * 2;               // one bf16 plane
  static constexpr int PROW = K * 2;                  // plane row bytes
  static constexpr int SW = (PROW / 16 < 32 ? PROW / 16 : 32) - 1;
  static constexpr int PA = A_BYTES / 1024 / NW, PC = C_BYTES / 1024 / NW;
  static constexpr int G4 = BM * K / 4 / NT;          // float4 groups per thread in the split pass
  static_assert(A_BYTES % (1024 * NW) == 0 && C_BYTES % (1024 * NW) == 0, "shape");
  static_assert(16 * N * 4 <= A_BYTES && G4 * NT * 4 == BM * K, "staging / split pass");
};

template <int K, int N, bool kR1>
struct Ws32Ring {
  static constexpr int NST = 2;                                          // A ring depth
  static constexpr int ACC = NST * Ws32Cfg<K, N>::A_BYTES;               // accum buffer
  static constexpr int PLANES = ACC + (kR1 ? Ws32Cfg<K, N>::C_BYTES : 0);  // the three bf16 planes
  static constexpr int BIAS = PLANES + 3 * Ws32Cfg<K, N>::PL;            // the bias row
  static constexpr int BYTES = BIAS + N * 4;
  static_assert(32 * N * 4 <= 3 * Ws32Cfg<K, N>::PL, "the 32-row staging fits the plane images");
};

template <int K, int N, int EPI, bool kR1, bool kZ, bool kR2>
__global__ __launch_bounds__((Ws32Cfg<K, N>::NT), 1) void k_ws_f32(WsArgs32 g) {
  static_assert(K == N, "square layers");
  using C = Ws32Cfg<K, N>;
  using R = Ws32Ring<K, N, kR1>;
  static_assert((EPI == 1 && !kR2) || (EPI == 4 && kR1 && (kZ || !kR2)), "epilogue operands");
  constexpr int PA = C::PA, PC = kR1 ? C::PC : 0;              // DMA instructions per wave per block (A, r1)
  constexpr int PR2 = kR2 ? C::PC : 0;                           // (r2)
  constexpr int S = 4 * (kZ ? 2 : 1);                            // stores per lane per block
  constexpr int QPR = N / 4;
  extern __shared__ __attribute__((aligned(16))) char ws32_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int64_t M = g.M;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;
  char* const planes = ws32_smem + R::PLANES;

  // this wave's W slice as split B fragments: lane (li, lh) holds W[32 wave + li][16 t + 8 lh .. + 7]
  uint4 wf[C::KS][3];
  {
    const float* wr = g.w + (int64_t)(wave * 32 + li) * K + lh * 8;
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
      const float4 v0 = *reinterpret_cast<const float4*>(wr + t * 16);
      const float4 v1 = *reinterpret_cast<const float4*>(wr + t * 16 + 4);
      uint2 o0[3], o1[3];
      split4(v0, o0);
      split4(v1, o1);
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[t][p] = make_uint4(o0[p].x, o0[p].y, o1[p].x, o1[p].y);
    }
  }
  // the bias row goes to LDS once (read per row pass: no VGPRs held across the loop); the PReLU slope is uniform
  float* const bias_lds = reinterpret_cast<float*>(ws32_smem + R::BIAS);
  if (EPI == 1 && tid < N / 4) {
    const float4 b4 = *reinterpret_cast<const float4*>(g.bias + tid * 4);
    asm volatile("" ::"v"(b4.x), "v"(b4.y), "v"(b4.z), "v"(b4.w));
    *reinterpret_cast<float4*>(bias_lds + tid * 4) = b4;
  }
  const float a_slope = EPI == 1 ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(g.prelu[0]))) : 0.0f;
  const float sc_self = EPI == 4 ? __fadd_rn(1.0f, __int_as_float(__builtin_amdgcn_readfirstlane(
                                                        __float_as_int(g.eps[0])))) : 0.0f;
  float ep = 0.0f;                                               // EPI 4: this thread's eps-gradient partial
#pragma unroll
  for (int t = 0; t < C::KS; ++t)
#pragma unroll
    for (int p = 0; p < 3; ++p) asm volatile("" ::"v"(wf[t][p].x), "v"(wf[t][p].y), "v"(wf[t][p].z), "v"(wf[t][p].w));

  auto dma = [&](const void* src, void* dst) {
    if (g.nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  auto tid_o = [&]() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto rows_of = [&](int64_t i, int64_t& r0, int& rmax) {
    r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
  };
  auto issue_a = [&](int64_t i) {
    char* base = ws32_smem + (int)(i % R::NST) * C::A_BYTES;
    int64_t r0;
    int rmax;
    rows_of(i, r0, rmax);
    const float* ab = g.a + r0 * g.lda;
    const int ln = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (K * 4);
      r = r < rmax ? r : rmax;
      dma(ab + (r * (int)g.lda + (off % (K * 4)) / 4), base + piece * 1024);
    }
  };
  auto issue_rows = [&](int64_t i, const float* src, int64_t ld, char* img) {   // N-wide rows of block i
    int64_t r0;
    int rmax;
    rows_of(i, r0, rmax);
    const float* cb = src + r0 * ld;
    const int ln = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < C::PC; ++q) {
      const int piece = wave * C::PC + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (N * 4);
      r = r < rmax ? r : rmax;
      dma(cb + (r * (int)ld + (off % (N * 4)) / 4), img + piece * 1024);
    }
  };

  issue_a(0);
  for (int64_t i = 0; i < my; ++i) {
    // wait for A(i).  Issue order: A(0); then per iteration j: r1(j), A(j + 1), [r2(j) after the split pass], the
    // stores of j.  Exact when every block is full (only a grid's last block is partial, and it is the last
    // iteration of its workgroup).
    if (i > 0) wait_vm<S + PR2>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();   // A(i) landed for every wave; the slot of A(i - 1), r1 and planes are free
    asm volatile("" ::: "memory");
    if constexpr (kR1) issue_rows(i, g.r1, g.ldr1, ws32_smem + R::ACC);
    if (i + 1 < my) issue_a(i + 1);
    const char* abase = ws32_smem + (int)(i % R::NST) * C::A_BYTES;
    {   // split pass: the fp32 image -> the three plane images
      const int t = tid_o();
#pragma unroll
      for (int j = 0; j < C::G4; ++j) {
        const int grp = j * C::NT + t;
        const float4 v = *reinterpret_cast<const float4*>(abase + grp * 16);
        const int r = grp / (K / 4), k = (grp % (K / 4)) * 4;
        uint2 o[3];
        split4(v, o);
        const int off = r * C::PROW + 16 * ((k >> 3) ^ (r & C::SW)) + 8 * ((k >> 2) & 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(planes + p * C::PL + off) = o[p];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    // g_prev rows into the block's A slot, dead after the split pass (refilled by A(i + 2) only after the next
    // iteration's barrier)
    if constexpr (kR2) issue_rows(i, g.r2, g.ldr2, ws32_smem + (int)(i % R::NST) * C::A_BYTES);
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
    // A fragments double-buffered one k-step ahead; the scheduling fences keep the compiler from hoisting every
    // k-step's fragment reads to the top of the block (3 x 4 x KS VGPRs on top of the W slice)
    const int fl = tid_o() & 63;
    const int frow = (fl & 31) * C::PROW;
    const int fsw = ((fl >> 5) ^ (fl & 31)) & C::SW;          // (2t + lh) ^ (li & SW) = 2t ^ fsw for 2t even
    auto frag = [&](int t, uint4 (&f)[3]) {
      const int off = frow + ((2 * t ^ fsw) << 4);
      f[0] = *reinterpret_cast<const uint4*>(planes + off);
      f[1] = *reinterpret_cast<const uint4*>(planes + C::PL + off);
      f[2] = *reinterpret_cast<const uint4*>(planes + 2 * C::PL + off);
    };
    uint4 fa[2][3];
    frag(0, fa[0]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
      if (t + 1 < C::KS) frag(t + 1, fa[(t + 1) & 1]);
      const uint4(&f)[3] = fa[t & 1];
      const bf16x8 a0 = __builtin_bit_cast(bf16x8, f[0]), a1 = __builtin_bit_cast(bf16x8, f[1]),
                   a2 = __builtin_bit_cast(bf16x8, f[2]);
      const bf16x8 b0 = __builtin_bit_cast(bf16x8, wf[t][0]), b1 = __builtin_bit_cast(bf16x8, wf[t][1]),
                   b2 = __builtin_bit_cast(bf16x8, wf[t][2]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);   // k_gemm_nt's order
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // r1(i) [and r2(i)] landed (A(i + 1) may stay in flight unless r2 was issued after it); every wave's share, so a
    // barrier follows below
    if constexpr (kR2) {
      wait_vm<0>();
    } else if constexpr (kR1) {
      if (i + 1 < my) wait_vm<PA>(); else wait_vm<0>();
    }
    float* stg = reinterpret_cast<float*>(planes);               // the dead plane images: all 32 rows at once
    const float* img1 = reinterpret_cast<const float*>(ws32_smem + R::ACC);
    const float* img2 = reinterpret_cast<const float*>(ws32_smem + (int)(i % R::NST) * C::A_BYTES);
    const int ldy = EPI == 1 ? N : (int)g.ldy, ldz = EPI == 1 ? N : (int)g.ldz;
    float* yb = g.y + r0 * ldy;
    float* zb = kZ ? g.z + r0 * ldz : nullptr;
    __builtin_amdgcn_s_barrier();                 // every wave's plane reads are done (and its accum pieces landed)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * lh;
      stg[row * N + ((wave * 32 + li) ^ (((row >> 2) & 1) << 5))] = acc[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int tq = tid_o();
      const int cq = (tq % QPR) * 4;
      const int brow = pass * 8 + tq / QPR;
      const int64_t grow = r0 + brow;
      const float4 v4 = *reinterpret_cast<const float4*>(stg + brow * N + (cq ^ (((brow >> 2) & 1) << 5)));
      float o[4] = {v4.x, v4.y, v4.z, v4.w};
      float zz[4] = {0.f, 0.f, 0.f, 0.f};
      float in1[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (kR1) {
        const float4 c4 = *reinterpret_cast<const float4*>(img1 + brow * N + cq);
        in1[0] = c4.x; in1[1] = c4.y; in1[2] = c4.z; in1[3] = c4.w;
      }
      if constexpr (EPI == 1) {
        const float4 b4 = *reinterpret_cast<const float4*>(bias_lds + cq);
        const float bcol[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          zz[t] = __fadd_rn(o[t], bcol[t]);
          const float y = zz[t] > 0.0f ? zz[t] : __fmul_rn(a_slope, zz[t]);
          o[t] = kR1 ? __fadd_rn(in1[t], y) : y;
        }
      }
      if (grow < M) {
        if constexpr (EPI == 4) {   // epilogue<4>'s self-term backward on C (every column is a self column)
          float in2[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (kR2) {
            const float4 p4 = *reinterpret_cast<const float4*>(img2 + brow * N + cq);
            in2[0] = p4.x; in2[1] = p4.y; in2[2] = p4.z; in2[3] = p4.w;
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            ep = __fadd_rn(ep, __fmul_rn(o[t], in1[t]));
            zz[t] = __fmul_rn(sc_self, o[t]);
            if (kR2) zz[t] = __fadd_rn(in2[t], zz[t]);
          }
        }
        const int oy = brow * ldy + cq, oz = brow * ldz + cq;
        if (g.nt_io) {
          Out4<float>::st_nt(yb + oy, o, true, 4);
          if constexpr (kZ) Out4<float>::st_nt(zb + oz, zz, true, 4);
        } else {
          Out4<float>::st(yb + oy, o, true, 4);
          if constexpr (kZ) Out4<float>::st(zb + oz, zz, true, 4);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (EPI == 4) tile_partial(reinterpret_cast<float*>(ws32_smem), ep, g.part, blockIdx.x);
}

// HGIN_NT_WS32 = 0 keeps the tiled kernel for the fp32 forward GEMM.
bool ws32_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_NT_WS32");
    return !(v && v[0] == '0');
  }();
  return on;
}

template <int K, int N, int EPI, bool kR1, bool kZ, bool kR2>
int launch_ws32(const WsArgs32& a, hipStream_t s, const char* what, int64_t* grid_out = nullptr) {
  constexpr int lds = Ws32Ring<K, N, kR1>::BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = k_ws_f32<K, N, EPI, kR1, kZ, kR2>;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (attr != hipSuccess) {
    set_error("%s: hipFuncSetAttribute failed: %s", what, hipGetErrorString(attr));
    return (int)attr;
  }
  const int64_t nblk = ceil_div(a.M, (int64_t)Ws32Cfg<K, N>::BM);
  const int64_t grid = nblk < ws_grid() ? nblk : ws_grid();
  HGIN_TRACE("k_ws_f32<%d,%d,EPI%d>", K, N, EPI);
  kern<<<(unsigned)grid, Ws32Cfg<K, N>::NT, lds, s>>>(a);
  if (grid_out) *grid_out = grid;
  return check_launch(what);
}

// k_wss_f32 — k_ws_f32 (K = N = 256) as a two-stage software pipeline with the two waves of a SIMD staggered
// (every K = N = 256 call k_ws_f32 does not need for g_prev): iteration i runs the MFMAs of block i on plane buffer i & 1 and
// the split of block i + 1 into buffer (i + 1) & 1, one barrier per block.  Waves 0-3 (one per SIMD) run the
// epilogue of block i - 1 and the split of block i + 1, then their MFMAs; waves 4-7 run their MFMAs first, then the
// epilogue of block i and the split — so each SIMD's VALU work sits beside the other wave's MFMAs instead of every
// wave splitting, then multiplying, then storing in lockstep.
//   * EPI 1: the forward MLP GEMM (z = acc + b, y = prelu(z) [+ accum]); EPI 4 (round 5): the dX GEMM with the
//     self-term backward (C = g_comb, g_x_dst = (1 + eps) C, the eps-gradient partial sum of C x_dst), every column a
//     self column, no g_prev (that call keeps k_ws_f32, whose g_prev rows arrive in the block's dead A slot);
//   * LDS: one 32 KB fp32 A slot in per-wave slices (a wave splits exactly the 4 KB its own DMA wrote, so it waits
//     only on its own vmcnt and refills its slice right after reading it) + two 48 KB plane buffers [+ with a row
//     operand (accum / x_dst) a 32 KB row image: wave w's 32 x 32 column slice, DMA'd by the wave itself right
//     after its epilogue has read the previous block's, read back in the accumulator layout — 160 KB in all];
//   * every wait on the DMA / store stream is counted (a wave's vector-memory ops retire in issue order), so the
//     split waits only for its A slice and the epilogue only for its row slice;
//   * the epilogue works from the accumulators: lane (li, lh) holds column 32 w + li of rows (e & 3) + 8 (e >> 2)
//     + 4 lh — the bias is one register, and y / z go out as 32-lane 128-B row segments by buffer stores from the
//     block's row base (SGPR resources, one lane offset);
//   * same W fragments, A fragments, product order and epilogue arithmetic as k_ws_f32: y / z / C / g_x_dst are
//     bit-identical to it (EPI 4's eps partial sums the same terms in another order, one partial per workgroup).
// Round 4 read the accum rows as 4-byte lane loads in the accumulator layout instead (2.81 vs k_ws_f32's 2.67 ms per
// launch at M = 3M: HBM latency in the epilogue, profiles/r04/gpu_q); the row image replaces that.
// Round 6, the first layer's K = 512 forward ([aggregate | (1 + eps) x_dst] W^T) as two launches
// of this kernel: EPI 5 stores the raw fp32 accumulators of the aggregate half (W[:, 0:256], ldw = 512) into z; then
// kInit starts every accumulator from that partial (the row image, read in the accumulator layout before the MFMAs)
// and continues the same chain over the x_dst half (W[:, 256:512], kScale: A scaled by fl(1 + eps) before the split,
// the tiled kernel's staging arithmetic) with EPI 1's epilogue.  An MFMA chain stored and reloaded in fp32 is the
// same chain: z / y are bit-identical to the tiled K = 512 kernel (tests/test_gpu_gemm_switch.py).
template <int EPI, bool kR1, bool kZ, bool kInit = false, bool kScale = false, int KV = 256>
__global__ __launch_bounds__(512, 1) void k_wss_f32(WsArgs32 g) {
  using C = Ws32Cfg<KV, 256>;
  constexpr int K = KV, N = 256;
  constexpr int PLANES = 3 * C::PL;                                // one plane buffer
  constexpr int PL0 = C::A_BYTES;                                  // plane buffers follow the A slot
  constexpr int R1_OFF = PL0 + 2 * PLANES;                         // row image: 8 per-wave 4 KB slices
  constexpr int PR = kR1 ? 4 : 0;                                  // row-image DMA pieces per wave per block
  constexpr int S = 16 * (kZ ? 2 : 1);                             // dword stores per lane per block
  static_assert(C::BM == 32 && C::NW == 8 && C::G4 == C::PA && (K == 256 || (K == 128 && EPI == 5)),
                "one PA KB slice and PA split groups per wave; K = 128: the plain product only");
  static_assert(EPI == 1 || EPI == 5 || (EPI == 4 && kR1), "EPI 4 reads x_dst");
  static_assert(!kInit || (EPI == 1 && kR1), "kInit: the partial arrives as the row image of an EPI 1 launch");
  static_assert(EPI != 5 || (!kR1 && !kZ), "EPI 5 stores the raw accumulators only");
  static_assert(R1_OFF + (kR1 ? 8 * 4096 : 0) <= 163840 && S + PR <= 63, "LDS / vmcnt");
  extern __shared__ __attribute__((aligned(16))) char wss_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: SGPR arithmetic below
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int64_t M = g.M;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;

  uint4 wf[C::KS][3];   // W[32 wave + li][16 t + 8 lh .. + 7] as three bf16 planes (k_ws_f32's B fragments)
  {
    const float* wr = g.w + (int64_t)(wave * 32 + li) * (g.ldw ? g.ldw : K) + lh * 8;
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
      const float4 v0 = *reinterpret_cast<const float4*>(wr + t * 16);
      const float4 v1 = *reinterpret_cast<const float4*>(wr + t * 16 + 4);
      uint2 o0[3], o1[3];
      split4(v0, o0);
      split4(v1, o1);
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[t][p] = make_uint4(o0[p].x, o0[p].y, o1[p].x, o1[p].y);
    }
  }
  const float bcol = EPI == 1 ? g.bias[wave * 32 + li] : 0.0f;
  const float a_slope = EPI == 1 ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(g.prelu[0]))) : 0.0f;
  const float sc_self = EPI == 4 ? __fadd_rn(1.0f, __int_as_float(__builtin_amdgcn_readfirstlane(
                                                        __float_as_int(g.eps[0])))) : 0.0f;
  const float sc_a = kScale ? __fadd_rn(1.0f, __int_as_float(__builtin_amdgcn_readfirstlane(
                                                  __float_as_int(g.eps2[0])))) : 1.0f;
  float ep = 0.0f;                                               // EPI 4: this thread's eps-gradient partial
#pragma unroll
  for (int t = 0; t < C::KS; ++t)
#pragma unroll
    for (int p = 0; p < 3; ++p) asm volatile("" ::"v"(wf[t][p].x), "v"(wf[t][p].y), "v"(wf[t][p].z), "v"(wf[t][p].w));

  auto tid_o = [&]() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto dma = [&](const void* src, void* dst) {
    if (g.nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  auto issue = [&](int64_t i) {   // this wave's 4 KB slice of block i's A rows
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const float* ab = g.a + r0 * g.lda;
    const int ln = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (K * 4);
      r = r < rmax ? r : rmax;
      dma(ab + (r * (int)g.lda + (off % (K * 4)) / 4), wss_smem + piece * 1024);
    }
  };
  char* const rimg = wss_smem + R1_OFF + wave * 4096;             // this wave's row slice: [32 rows][32 columns]
  auto issue_rows = [&](int64_t i) {   // block i's rows, columns 32 w .. 32 w + 31 (rows past M clamped to the last)
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const float* src = g.r1 + r0 * g.ldr1 + wave * 32;
    const int ln = tid_o() & 63;
#pragma unroll
    for (int q = 0; q < PR; ++q) {
      int r = q * 8 + (ln >> 3);
      r = r < rmax ? r : rmax;
      dma(src + (r * (int)g.ldr1 + (ln & 7) * 4), rimg + q * 1024);
    }
  };
  // block j (in this wave's slice, landed) -> plane buffer j & 1; the slice is then refilled with block j + 1
  auto split = [&](int64_t j) {
    char* pl = wss_smem + PL0 + (int)(j & 1) * PLANES;
    const int ln = tid_o() & 63;
    float4 v[C::G4];
#pragma unroll
    for (int q = 0; q < C::G4; ++q) v[q] = *reinterpret_cast<const float4*>(wss_smem + (wave * C::PA + q) * 1024 + ln * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (j + 1 < my) issue(j + 1);
    if constexpr (kScale) {
#pragma unroll
      for (int q = 0; q < C::G4; ++q)
        v[q] = make_float4(__fmul_rn(sc_a, v[q].x), __fmul_rn(sc_a, v[q].y), __fmul_rn(sc_a, v[q].z),
                           __fmul_rn(sc_a, v[q].w));
    }
#pragma unroll
    for (int q = 0; q < C::G4; ++q) {
      const int grp = ((wave * C::PA + q) * 1024 + ln * 16) / 16;
      const int r = grp / (K / 4), k = (grp % (K / 4)) * 4;
      uint2 o[3];
      split4(v[q], o);
      const int off = r * C::PROW + 16 * ((k >> 3) ^ (r & C::SW)) + 8 * ((k >> 2) & 1);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(pl + p * C::PL + off) = o[p];
    }
  };
  f32x16 acc;
  auto mfma = [&](int64_t i) {   // k_ws_f32's fragments and product order
    const char* planes = wss_smem + PL0 + (int)(i & 1) * PLANES;
    if constexpr (kInit) {   // the partial of the first K half, this wave's 32 columns in the accumulator layout
      const int il = tid_o() & 63;
      const float* img = reinterpret_cast<const float*>(rimg) + 4 * (il >> 5) * 32 + (il & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = img[((e & 3) + 8 * (e >> 2)) * 32];
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
    }
    const int fl = tid_o() & 63;
    const int frow = (fl & 31) * C::PROW;
    const int fsw = ((fl >> 5) ^ (fl & 31)) & C::SW;
    auto frag = [&](int t, uint4 (&f)[3]) {
      const int off = frow + ((2 * t ^ fsw) << 4);
      f[0] = *reinterpret_cast<const uint4*>(planes + off);
      f[1] = *reinterpret_cast<const uint4*>(planes + C::PL + off);
      f[2] = *reinterpret_cast<const uint4*>(planes + 2 * C::PL + off);
    };
    uint4 fa[2][3];
    frag(0, fa[0]);
#pragma unroll
    for (int t = 0; t < C::KS; ++t) {
      if (t + 1 < C::KS) frag(t + 1, fa[(t + 1) & 1]);
      const uint4(&f)[3] = fa[t & 1];
      const bf16x8 a0 = __builtin_bit_cast(bf16x8, f[0]), a1 = __builtin_bit_cast(bf16x8, f[1]),
                   a2 = __builtin_bit_cast(bf16x8, f[2]);
      const bf16x8 b0 = __builtin_bit_cast(bf16x8, wf[t][0]), b1 = __builtin_bit_cast(bf16x8, wf[t][1]),
                   b2 = __builtin_bit_cast(bf16x8, wf[t][2]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // the epilogue of block i from the accumulators (k_ws_f32's epilogue<1> / <4> arithmetic).  Buffer stores from the
  // block's row base (SGPR resources, one lane offset per output): no per-row 64-bit addresses held in VGPRs.
  constexpr int kRsrc = 0x00020000;
  const int ldy = EPI == 1 ? N : (int)g.ldy, ldz = EPI == 1 ? N : (int)g.ldz;
  auto epilogue = [&](int64_t i) {
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int nr = M - r0 < C::BM ? (int)(M - r0) : C::BM;
    const auto ry = __builtin_amdgcn_make_buffer_rsrc(g.y + r0 * ldy, 0, C::BM * ldy * 4, kRsrc);
    const auto rz = __builtin_amdgcn_make_buffer_rsrc(kZ ? g.z + r0 * ldz : g.y, 0, C::BM * ldz * 4, kRsrc);
    // lane offsets recomputed per block (tid_o hides tid's value): nothing of the epilogue stays live in VGPRs
    const int el = tid_o() & 63, eli = el & 31, elh = el >> 5;
    const int voy = (4 * elh * ldy + wave * 32 + eli) * 4, voz = (4 * elh * ldz + wave * 32 + eli) * 4;
    const float* img = reinterpret_cast<const float*>(rimg) + 4 * elh * 32 + eli;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rb = (e & 3) + 8 * (e >> 2);                     // this lane's row: rb + 4 lh
      constexpr bool kAcc = kR1 && !kInit;                        // the row image is the accum (EPI 1) / x_dst
      const float in1 = kAcc ? img[rb * 32] : 0.0f;
      if ((e & 3) == 3) __builtin_amdgcn_sched_barrier(0);       // at most 4 row values in flight
      float o, zz;
      if constexpr (EPI == 5) {
        o = acc[e];
        zz = 0.0f;
      } else if constexpr (EPI == 1) {
        zz = __fadd_rn(acc[e], bcol);
        const float y = zz > 0.0f ? zz : __fmul_rn(a_slope, zz);
        o = kAcc ? __fadd_rn(in1, y) : y;
      } else {
        o = acc[e];
        zz = __fmul_rn(sc_self, o);
      }
      if (rb + 4 * elh < nr) {
        if constexpr (EPI == 4) ep = __fadd_rn(ep, __fmul_rn(o, in1));
        const int aux = g.nt_io ? 2 : 0;
        if (aux) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), ry, voy, rb * ldy * 4, 2);
          if constexpr (kZ) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zz), rz, voz, rb * ldz * 4, 2);
        } else {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), ry, voy, rb * ldy * 4, 0);
          if constexpr (kZ) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(zz), rz, voz, rb * ldz * 4, 0);
        }
      }
    }
    if constexpr (kR1 && !kInit) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the row slice is read: refill it
  };

  // Per wave the vector-memory stream is: A(0), A(1) [split(0)], R(0), then per block j the epilogue's stores E(j),
  // R(j + 1), A(j + 2) [split(j + 1)] (waves 4-7 run E(j) after block j's MFMAs, waves 0-3 before block j + 1's).
  // Hence the split of block j + 1 waits until at most S + PR ops issued after A(j + 1) are pending (PR at waves
  // 0-3's first split, which no epilogue precedes), and the epilogue of block j until at most PA are pending after
  // R(j): the A pieces that follow it — of block j + 2 at waves 0-3, of block j + 1 at waves 4-7 (R(0): none yet) —
  // when that block exists.
  issue(0);
  wait_vm<0>();
  split(0);
  if constexpr (kR1) issue_rows(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  auto wait_rows = [&](int64_t j, bool first) {   // before the epilogue of block j (first: waves 0-3)
    if constexpr (kR1 && !kInit) {
      if (first ? j + 2 < my : (j >= 1 && j + 1 < my)) wait_vm<C::PA>(); else wait_vm<0>();
    }
  };
  // kInit: block i's rows must have landed before its MFMAs, and its slice is free once they have read it, so R(i + 1)
  // is issued right after block i's MFMAs (a whole epilogue + split earlier than R(j + 1) above).  Younger than R(i)
  // at block i's MFMAs: waves 0-3 — E(i - 1) and A(i + 2) [split(i + 1)] (R(0), issued after A(1) in the prologue: only
  // A(2)); waves 4-7 — E(i - 1) and A(i + 1) [split(i)] (R(0): nothing).  The splits' waits count the same ops as above
  // (R and E swap places).
  auto wait_init = [&](int64_t i, bool first) {
    if constexpr (kInit) {
      const bool a_next = first ? i + 2 < my : i + 1 < my;
      if (i == 0) {
        if (first && a_next) wait_vm<C::PA>(); else wait_vm<0>();
      } else {
        if (a_next) wait_vm<S + C::PA>(); else wait_vm<S>();
      }
    }
  };
  auto issue_rows_next = [&](int64_t i) {   // kInit: block i + 1's rows, once block i's MFMAs have read the slice
    if constexpr (kInit) {
      if (i + 1 < my) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_rows(i + 1);
      }
    }
  };
  // one loop per wave group (the same barrier count: s_barrier counts arrivals, not program points), so the
  // accumulators are dead during each group's split
  if (wave < 4) {
    for (int64_t i = 0; i < my; ++i) {
      __builtin_amdgcn_s_barrier();   // block i's planes written by every wave; block i - 1's read by every wave
      asm volatile("" ::: "memory");
      if (i > 0) {
        wait_rows(i - 1, true);
        epilogue(i - 1);
        if (kR1 && !kInit) issue_rows(i);
      }
      if (i + 1 < my) {
        if (i == 0) wait_vm<PR>(); else wait_vm<S + PR>();
        split(i + 1);
      }
      wait_init(i, true);
      mfma(i);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's plane writes and fragment reads are done
      issue_rows_next(i);
    }
    wait_rows(my - 1, true);
    epilogue(my - 1);
  } else {
    for (int64_t i = 0; i < my; ++i) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      wait_init(i, false);
      mfma(i);
      __builtin_amdgcn_sched_barrier(0);
      issue_rows_next(i);
      wait_rows(i, false);
      epilogue(i);
      if (i + 1 < my) {
        if (kR1 && !kInit) issue_rows(i + 1);
        wait_vm<S + PR>();
        split(i + 1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if constexpr (EPI == 4) {
    wait_vm<0>();
    tile_partial(reinterpret_cast<float*>(wss_smem), ep, g.part, blockIdx.x);
  }
}

// Always on (round 6: the A/B switch is gone): fwd256 at M = 6M 4.95 -> 4.49 ms per launch, the cfg3 step
// 183.3 -> 179.4 ms (profiles/r04/gpu_s).
constexpr bool wss_enabled() { return true; }

template <int EPI, bool kR1, bool kZ, bool kInit = false, bool kScale = false, int KV = 256>
int launch_wss(const WsArgs32& a, hipStream_t s, const char* what, int64_t* grid_out = nullptr) {
  constexpr int lds = Ws32Cfg<KV, 256>::A_BYTES + 2 * 3 * Ws32Cfg<KV, 256>::PL + (kR1 ? 8 * 4096 : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = k_wss_f32<EPI, kR1, kZ, kInit, kScale, KV>;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (attr != hipSuccess) {
    set_error("%s: hipFuncSetAttribute failed: %s", what, hipGetErrorString(attr));
    return (int)attr;
  }
  const int64_t nblk = ceil_div(a.M, (int64_t)Ws32Cfg<KV, 256>::BM);
  const int64_t grid = nblk < ws_grid() ? nblk : ws_grid();
  HGIN_TRACE("k_wss_f32<EPI%d,%d,%d%s%s>", EPI, (int)kR1, (int)kZ, kInit ? ",init" : "", KV == 128 ? ",K128" : "");
  kern<<<(unsigned)grid, 512, lds, s>>>(a);
  if (grid_out) *grid_out = grid;
  return check_launch(what);
}

// Returns -1 when the fp32 weight-stationary form does not apply (the caller launches the tiled kernel): split
// mode, K = N = 256 with one A source, or (round 6) the first layer's K = 512 = [a1 | (1 + eps) a2] with 256 + 256
// columns and no accum as two k_wss_f32 launches through z (or y when z is not kept); 16-B aligned rows, packed W /
// z / y / accum.
int try_ws_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2, const float* a2_eps,
               const float* w, const float* bias, const float* prelu, const float* accum, float* z, float* y,
               int64_t M, int64_t N, int64_t K, hipStream_t s, const char* what) {
  if (!ws32_enabled() || !gemm_split_enabled() || M < 1) return -1;
  if (K == 512 && N == 256 && k1 == 256 && a2 && a2_eps && !accum && wss_enabled()) {
    // (the relation that adds another's output keeps the tiled kernel: the partial and accum row images do not
    // both fit beside the plane buffers)
    auto ok = [](const void* p, int64_t ld) { return aligned16(p) && ld % 4 == 0 && ld < (int64_t(1) << 24); };
    if (!ok(a1, lda1) || !ok(a2, lda2) || !aligned16(w) || !aligned16(y) || (z && !aligned16(z))) return -1;
    float* part = z ? z : y;
    const bool nt_io = gemm_nt_io(M, N, 4);
    WsArgs32 g1{a1, lda1, w, nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, part, N, nullptr, nullptr, M,
                nt_io, ws_nt_in(), 512, nullptr};
    if (int rc = launch_wss<5, false, false>(g1, s, what)) return rc;
    WsArgs32 g2{a2, lda2, w + 256, bias, prelu, part, N, nullptr, 0, z, N, y, N, nullptr, nullptr, M, nt_io,
                ws_nt_in(), 512, a2_eps};
    if (z) return launch_wss<1, true, true, true, true>(g2, s, what);
    return launch_wss<1, true, false, true, true>(g2, s, what);
  }
  // (profiles/r02/gemm_ws_f32.txt)
  if (K != N || K != 256 || k1 != K || a2_eps != nullptr) return -1;
  if (!aligned16(a1) || lda1 % 4 || lda1 >= (int64_t(1) << 24) || !aligned16(w) || !aligned16(y) ||
      (z && !aligned16(z)) || (accum && !aligned16(accum)))
    return -1;
  WsArgs32 g{a1, lda1, w, bias, prelu, accum, N, nullptr, 0, z, N, y, N, nullptr, nullptr, M, gemm_nt_io(M, N, 4),
             ws_nt_in()};
  if (wss_enabled()) {
    if (accum && z) return launch_wss<1, true, true>(g, s, what);
    if (accum) return launch_wss<1, true, false>(g, s, what);
    if (z) return launch_wss<1, false, true>(g, s, what);
    return launch_wss<1, false, false>(g, s, what);
  }
  if (accum && z) return launch_ws32<256, 256, 1, true, true, false>(g, s, what);
  if (accum) return launch_ws32<256, 256, 1, true, false, false>(g, s, what);
  if (z) return launch_ws32<256, 256, 1, false, true, false>(g, s, what);
  return launch_ws32<256, 256, 1, false, false, false>(g, s, what);
}

// The plain fp32 NT GEMM (hgin_gemm_nt_f32: C = A B^T, B packed [N, K]) at N = 256, K = 128 / 256 as k_wss_f32's
// raw-accumulator epilogue (EPI 5) — the readout's dX through its first Linear(512, 128) has K = 128.  Same W / A
// fragments and product order as the tiled kernel, so C is bit-identical to it.  Returns -1 when it does not apply.
int try_wss_plain(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc, int64_t M, int64_t N,
                  int64_t K, hipStream_t s, const char* what) {
  if (!ws32_enabled() || !gemm_split_enabled() || M < 1 || N != 256 || (K != 128 && K != 256) || ldb != K) return -1;
  auto ok = [](const void* p, int64_t ld) { return aligned16(p) && ld % 4 == 0 && ld < (int64_t(1) << 20); };
  if (!ok(a, lda) || !ok(c, ldc) || !aligned16(b)) return -1;
  WsArgs32 g{a, lda, b, nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, 0, c, ldc, nullptr, nullptr, M,
             gemm_nt_io(M, N, 4), ws_nt_in()};
  if (K == 128) return launch_wss<5, false, false, false, false, 128>(g, s, what);
  return launch_wss<5, false, false>(g, s, what);
}

// The dX GEMM with the self-term backward (EPI 4, hgin_gemm_nt_combine_f32) in the same form: C = A B^T with
// B packed [N, K], K = N = 256, the self term on every column (cs = 0); x_dst [, g_x_dst, g_prev] rows of any
// 16-B aligned stride.  Returns -1 when it does not apply; *grid_out = the workgroups (= eps partials).
int try_ws_f32_comb(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc, int64_t M,
                    int64_t N, int64_t K, const CombEpi& ce, hipStream_t s, const char* what, int64_t* grid_out) {
  if (!ws32_enabled() || !gemm_split_enabled() || M < 1 || K != N || K != 256 || ldb != K || ce.cs != 0) return -1;
  auto ok = [](const void* p, int64_t ld) {
    return p == nullptr || (aligned16(p) && ld % 4 == 0 && ld < (int64_t(1) << 24));
  };
  const float* xd = static_cast<const float*>(ce.xd);
  float* gd = static_cast<float*>(ce.gd);
  const float* gp = static_cast<const float*>(ce.gp);
  if (!xd || !aligned16(b) || !ok(a, lda) || !ok(c, ldc) || !ok(xd, ce.ldxd) || !ok(gd, ce.ldgd) ||
      !ok(gp, ce.ldgp) || (gp && !gd))
    return -1;
  WsArgs32 g{a, lda, b, nullptr, nullptr, xd, ce.ldxd, gp, ce.ldgp, gd, ce.ldgd, c, ldc, ce.eps, ce.part, M,
             gemm_nt_io(M, N, 4), ws_nt_in()};
  if (wss_enabled() && !gp) {   // (with g_prev: k_ws_f32, whose g_prev rows arrive in the block's dead A slot)
    if (gd) return launch_wss<4, true, true>(g, s, what, grid_out);
    return launch_wss<4, true, false>(g, s, what, grid_out);
  }
  if (gd && gp) return launch_ws32<256, 256, 4, true, true, true>(g, s, what, grid_out);
  if (gd) return launch_ws32<256, 256, 4, true, true, false>(g, s, what, grid_out);
  return launch_ws32<256, 256, 4, true, false, false>(g, s, what, grid_out);
}

template <int EPI, typename OutT>
int launch_nt_bf16(const Src2h& a, const Src2h& b, int64_t M, int64_t N, int64_t K, const float* bias,
                   const float* prelu, const OutT* accum, OutT* z, OutT* y, int64_t ldc, hipStream_t s,
                   const char* what, const CombEpi& ce_in = CombEpi{}, int64_t* tiles_out = nullptr) {
  CombEpi ce = ce_in;
  ce.nt_io = gemm_nt_io(M, N, (int64_t)sizeof(OutT));
  {
    const int rc = try_ws_bf16<EPI, OutT>(a, b, M, N, K, bias, prelu, accum, z, y, ldc, ce, s, what, tiles_out);
    if (rc >= 0) return rc;   // (EPI 4: *tiles_out = the grid, one eps-gradient partial per workgroup)
  }
  const bool al = aligned16(a.p1) && a.ld1 % 8 == 0 && (a.k1 == K || (aligned16(a.p2) && a.ld2 % 8 == 0)) &&
                  aligned16(b.p1) && b.ld1 % 8 == 0;
  const bool vec = al && K % kBKh == 0 && a.k1 % kBKh == 0;
  // K a multiple of 32 only (the readout's dX through Linear(128, 32): K = 32), N > 32: 32-wide K tiles with 16-B
  // loads instead of the element-wise kClean = false loads over a half-empty 64-wide tile (1.10 ms per cfg5 step)
  const bool vec32 = al && !vec && K % 32 == 0 && a.k1 % 32 == 0;
  const bool vec_out = ldc % 4 == 0 && aligned16(y) && (z == nullptr || aligned16(z)) &&
                       (accum == nullptr || aligned16(accum)) &&
                       (EPI != 4 || (aligned16(ce.xd) && ce.ldxd % 4 == 0 &&
                                     (ce.gd == nullptr || (aligned16(ce.gd) && ce.ldgd % 4 == 0))));
#define HGIN_NT_BF16(TNV, WNV)                                                                                \
  {                                                                                                          \
    constexpr int BM = (4 / WNV) * 64;                                                                       \
    constexpr int BN = WNV * TNV * 32;                                                                       \
    const int64_t tiles = ceil_div(N, BN) * ceil_div(M, BM);                                                 \
    const bool xcd = xcd_remap_enabled();                                                                    \
    dim3 grid((unsigned)(xcd ? round_up8(tiles) : tiles));                                                   \
    HGIN_TRACE("k_gemm_nt_bf16<EPI%d,%dx%d,N%lld,K%lld%s>", EPI, BM, BN, (long long)N, (long long)K,        \
               (vec32 && EPI == 0 && BN >= TileH<32>::kRp) ? ",k32" : "");                                   \
    bool k32 = false;                                                                                        \
    if constexpr (BN >= TileH<32>::kRp) { /* (a 32-wide K tile loads 64 rows per pass) */                    \
      if (vec32 && EPI == 0) {                                                                               \
        k_gemm_nt_bf16<0, true, TNV, WNV, OutT, 32><<<grid, 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum,   \
                                                                         z, y, ldc, vec_out, tiles, xcd, ce); \
        k32 = true;                                                                                          \
      }                                                                                                      \
    }                                                                                                        \
    if (k32) {                                                                                               \
    } else if (vec)                                                                                          \
      k_gemm_nt_bf16<EPI, true, TNV, WNV, OutT><<<grid, 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z, y, \
                                                                     ldc, vec_out, tiles, xcd, ce);          \
    else                                                                                                     \
      k_gemm_nt_bf16<EPI, false, TNV, WNV, OutT><<<grid, 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z,  \
                                                                      y, ldc, vec_out, tiles, xcd, ce);      \
    if (tiles_out) *tiles_out = tiles;                                                                       \
  }
  if (N <= 32)
    HGIN_NT_BF16(1, 1)
  else if (use_bm64_bf16<EPI == 4 ? 0 : EPI, OutT>(M, N))
    HGIN_NT_BF16(1, 4)
  else
    HGIN_NT_BF16(2, 2)
#undef HGIN_NT_BF16
  return check_launch(what);
}

int check_a_h(const char* what, const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
              int64_t K) {
  HGIN_ARG_CHECK(k1 >= 0 && k1 <= K, "%s: k1 out of [0, K]", what);
  HGIN_ARG_CHECK(k1 == 0 || (a1 && lda1 >= k1), "%s: bad A1", what);
  HGIN_ARG_CHECK(k1 == K || (a2 && lda2 >= K - k1), "%s: bad A2", what);
  return HGIN_OK;
}

// ---------------------------------------------------------------------------------------------------
// Pre-split weight planes (hgin_nt_planes_*): the B operand of the split-mode NT GEMMs ([N, K], small) converted once
// per call into the per-K-stage LDS image of the kBdma kernels — fp32: the three bf16 split planes, bf16: one plane —
// laid out [stage][plane][N][stage k] with XOR-swizzled 16-B chunks, so a stage is a plain contiguous copy (LDS-DMA)
// and no workgroup re-splits W.  (An LDS-DMA restructuring of the whole NT GEMM around these planes, k_nt2, was
// measured slower and removed: DESIGN.md §3.)
//   B fp32 planes (64-B rows of 32 k): chunk c of column n at c ^ ((n >> 2) & 3)
//   B bf16 (128-B rows of 64 k):       chunk c of column n at c ^ ((n >> 1) & 7)
template <typename T>
struct Nt2 {
  static constexpr bool kF32 = sizeof(T) == 4;
  static constexpr int KS = kF32 ? 32 : 64;       // K elements per stage
  static constexpr int NP = kF32 ? 3 : 1;         // B planes
  static constexpr int BROW = kF32 ? 64 : 128;    // bytes of one B plane row per stage
};

// B planes, global layout [K / KS][NP][N][KS] (2-B elements), chunks swizzled as in the LDS image.
template <typename T>
__global__ __launch_bounds__(256) void k_nt_planes(const T* __restrict__ b, int64_t ldb, int64_t N, int64_t K,
                                                   uint16_t* __restrict__ out) {
  using P = Nt2<T>;
  constexpr int CH = P::BROW / 16;                     // 16-B chunks per plane row
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (stage, n, chunk)
  const int64_t stages = K / P::KS;
  if (i >= stages * N * CH) return;
  const int q = (int)(i % CH);
  const int64_t n = (i / CH) % N;
  const int64_t s = i / (CH * N);
  const int c = P::kF32 ? (q ^ (int)((n >> 2) & 3)) : (q ^ (int)((n >> 1) & 7));   // logical chunk at slot q
  const int64_t k0 = s * P::KS + c * 8;
  uint4 o[P::NP];
  if constexpr (P::kF32) {
    const float* src = reinterpret_cast<const float*>(b) + n * ldb + k0;
    const float4 v0 = *reinterpret_cast<const float4*>(src);
    const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
    uint2 a[3], bb[3];
    split4(v0, a);
    split4(v1, bb);
#pragma unroll
    for (int p = 0; p < 3; ++p) o[p] = make_uint4(a[p].x, a[p].y, bb[p].x, bb[p].y);
  } else {
    o[0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(b) + n * ldb + k0);
  }
#pragma unroll
  for (int p = 0; p < P::NP; ++p)
    *reinterpret_cast<uint4*>(out + (((s * P::NP + p) * N + n) * P::BROW + q * 16) / 2) = o[p];
}

template <typename T>
size_t nt_planes_bytes(int64_t N, int64_t K) {
  return (size_t)N * (size_t)K * Nt2<T>::NP * 2;
}

template <typename T>
int nt_planes(const T* b, int64_t ldb, int64_t N, int64_t K, void* out, hipStream_t s, const char* what) {
  using P = Nt2<T>;
  HGIN_ARG_CHECK(N > 0 && K > 0 && K % P::KS == 0, "%s: K must be a positive multiple of %d", what, P::KS);
  HGIN_ARG_CHECK(b && out && ldb >= K && aligned16(b) && ldb % (16 / (int)sizeof(T)) == 0 && aligned16(out),
                 "%s: bad operand / alignment", what);
  const int64_t work = (K / P::KS) * N * (P::BROW / 16);
  k_nt_planes<T><<<(unsigned)ceil_div(work, 256), 256, 0, s>>>(b, ldb, N, K, static_cast<uint16_t*>(out));
  return check_launch(what);
}

// Fixed-order sum of the EPI 4 tile partials: level 1 (k_part_sum over kPartChunk-long chunks, one workgroup
// each), level 2 (one workgroup over the level-1 sums).  cfg5 launches ~94k tiles: one workgroup alone took 0.1 ms.
constexpr int64_t kPartChunk = 4096;

__global__ __launch_bounds__(256) void k_part_sum(const float* __restrict__ part, int64_t n, float* __restrict__ out) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kPartChunk;
  const int64_t b1 = b0 + kPartChunk < n ? b0 + kPartChunk : n;
  float s = 0.0f;
  for (int64_t i = b0 + t; i < b1; i += 256) s = __fadd_rn(s, part[i]);
  red[t] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
    __syncthreads();
  }
  if (t == 0) out[blockIdx.x] = red[0];
}

int64_t combine_max_tiles(int64_t M, int64_t N) {   // the most tiles any tile shape launches (64-row x 32-col)
  return ceil_div(M > 0 ? M : 1, 64) * ceil_div(N > 0 ? N : 1, 32);
}

size_t combine_ws_bytes(int64_t M, int64_t N) {
  const int64_t t = combine_max_tiles(M, N);
  return align_up(sizeof(float) * (size_t)t, 256) + align_up(sizeof(float) * (size_t)ceil_div(t, kPartChunk), 256);
}

template <typename T>
int gemm_nt_combine(const char* what, const T* a, int64_t lda, const T* b, int64_t ldb, T* c, int64_t ldc, int64_t M,
                    int64_t N, int64_t K, const T* x_dst, int64_t ld_xd, T* g_dst, int64_t ld_gd, const T* g_prev,
                    int64_t ld_gp, int64_t cs,
                    const float* eps, float* g_eps, void* workspace, size_t workspace_bytes, const void* b_planes,
                    void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0 && cs >= 0 && cs <= N, "%s: bad sizes", what);
  HGIN_ARG_CHECK(N <= 65535 * 128 && M < (int64_t(1) << 31), "%s: size too large", what);
  HGIN_ARG_CHECK(cs % 4 == 0, "%s: the self columns must start at a multiple of 4", what);
  HGIN_ARG_CHECK(eps && g_eps, "%s: NULL eps / g_eps", what);
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == cs) return memset_async(g_eps, 0, sizeof(float), s, what);
  HGIN_ARG_CHECK(a && b && c && x_dst, "%s: NULL operand", what);
  HGIN_ARG_CHECK(lda >= K && ldb >= K && ldc >= N && ld_xd >= N - cs && (!g_dst || ld_gd >= N - cs),
                 "%s: leading dimension too small", what);
  const size_t need = combine_ws_bytes(M, N);
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  float* part = static_cast<float*>(workspace);
  HGIN_ARG_CHECK(!g_prev || (g_dst && ld_gp >= N - cs && aligned16(g_prev) == aligned16(g_dst) &&
                              (ld_gp % 4 == 0) == (ld_gd % 4 == 0)),
                 "%s: g_prev needs g_dst and a matching layout", what);
  CombEpi ce{x_dst, ld_xd, g_dst, ld_gd, cs, eps, part};
  ce.gp = g_prev;
  ce.ldgp = ld_gp;
  int64_t tiles = 0;
  int rc;
  if constexpr (sizeof(T) == 2)
    rc = launch_nt_bf16<4, uint16_t>(Src2h{a, lda, nullptr, 0, K}, Src2h{b, ldb, nullptr, 0, K}, M, N, K, nullptr,
                                     nullptr, nullptr, nullptr, c, ldc, s, what, ce, &tiles);
  else if constexpr (sizeof(T) == 4) {
    ce.nt_io = gemm_nt_io(M, N, 4);
    rc = try_ws_f32_comb(a, lda, b, ldb, c, ldc, M, N, K, ce, s, what, &tiles);
    if (rc < 0)
      rc = launch_nt<4>(Src2{a, lda, nullptr, 0, K}, Src2{b, ldb, nullptr, 0, K}, M, N, K, nullptr, nullptr, nullptr,
                        nullptr, c, ldc, s, what, ce, &tiles, b_planes);
  }
  if (rc) return rc;
  const int64_t nb = ceil_div(tiles, kPartChunk);
  if (nb == 1) {
    k_part_sum<<<1, 256, 0, s>>>(part, tiles, g_eps);
  } else {
    float* part2 = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                            align_up(sizeof(float) * (size_t)combine_max_tiles(M, N), 256));
    k_part_sum<<<(unsigned)nb, 256, 0, s>>>(part, tiles, part2);
    k_part_sum<<<1, 256, 0, s>>>(part2, nb, g_eps);   // nb <= kPartChunk for any M < 2^31
  }
  return check_launch(what);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_gemm_nt_combine_workspace_size(int64_t M, int64_t N, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && M >= 0 && N >= 0, "hgin_gemm_nt_combine_workspace_size: bad args");
  *bytes = combine_ws_bytes(M, N);
  return HGIN_OK;
}

extern "C" int hgin_gemm_nt_combine_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c,
                                        int64_t ldc, int64_t M, int64_t N, int64_t K, const float* x_dst,
                                        int64_t ld_xd, float* g_dst, int64_t ld_gd, const float* g_prev,
                                        int64_t ld_gp, int64_t cs, const float* eps, float* g_eps, void* workspace,
                                        size_t workspace_bytes, const void* b_planes, void* stream) {
  return gemm_nt_combine<float>("hgin_gemm_nt_combine_f32", a, lda, b, ldb, c, ldc, M, N, K, x_dst, ld_xd, g_dst,
                                ld_gd, g_prev, ld_gp, cs, eps, g_eps, workspace, workspace_bytes, b_planes, stream);
}

extern "C" int hgin_gemm_nt_combine_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, uint16_t* c,
                                         int64_t ldc, int64_t M, int64_t N, int64_t K, const uint16_t* x_dst,
                                         int64_t ld_xd, uint16_t* g_dst, int64_t ld_gd, const uint16_t* g_prev,
                                         int64_t ld_gp, int64_t cs, const float* eps, float* g_eps, void* workspace,
                                         size_t workspace_bytes, const void* b_planes, void* stream) {
  return gemm_nt_combine<uint16_t>("hgin_gemm_nt_combine_bf16", a, lda, b, ldb, c, ldc, M, N, K, x_dst, ld_xd, g_dst,
                                   ld_gd, g_prev, ld_gp, cs, eps, g_eps, workspace, workspace_bytes, b_planes, stream);
}

extern "C" int hgin_gin_mlp_fwd_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                                     const float* a2_eps, const uint16_t* w, const float* bias, const float* prelu,
                                     const uint16_t* accum, uint16_t* z, uint16_t* y, int64_t M, int64_t N, int64_t K,
                                     const void* w_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gin_mlp_fwd_bf16: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * 128, "hgin_gin_mlp_fwd_bf16: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && prelu && y, "hgin_gin_mlp_fwd_bf16: NULL operand");
  if (int rc = check_a_h("hgin_gin_mlp_fwd_bf16", a1, lda1, k1, a2, lda2, K)) return rc;
  return launch_nt_bf16<1, uint16_t>(Src2h{a1, lda1, a2, lda2, k1, a2_eps}, Src2h{w, K, nullptr, 0, K}, M, N, K, bias, prelu,
                                     accum, z, y, N, as_stream(stream), "hgin_gin_mlp_fwd_bf16");
}

extern "C" int hgin_gin_mlp_fwd_zy_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                                        const float* a2_eps, const uint16_t* w, const float* bias, const float* prelu,
                                        uint16_t* z, uint16_t* y, int64_t M, int64_t N, int64_t K, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gin_mlp_fwd_zy_bf16: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * 128, "hgin_gin_mlp_fwd_zy_bf16: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && prelu && z && y, "hgin_gin_mlp_fwd_zy_bf16: NULL operand");
  if (int rc = check_a_h("hgin_gin_mlp_fwd_zy_bf16", a1, lda1, k1, a2, lda2, K)) return rc;
  CombEpi ce{};
  ce.zy = true;
  return launch_nt_bf16<1, uint16_t>(Src2h{a1, lda1, a2, lda2, k1, a2_eps}, Src2h{w, K, nullptr, 0, K}, M, N, K, bias,
                                     prelu, nullptr, z, y, N, as_stream(stream), "hgin_gin_mlp_fwd_zy_bf16", ce);
}

extern "C" int hgin_linear_fwd_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                                    const uint16_t* w, const float* bias, float* y, int64_t M, int64_t N, int64_t K,
                                    const void* w_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_linear_fwd_bf16: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * 128, "hgin_linear_fwd_bf16: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && y, "hgin_linear_fwd_bf16: NULL operand");
  if (int rc = check_a_h("hgin_linear_fwd_bf16", a1, lda1, k1, a2, lda2, K)) return rc;
  return launch_nt_bf16<2, float>(Src2h{a1, lda1, a2, lda2, k1}, Src2h{w, K, nullptr, 0, K}, M, N, K, bias, nullptr,
                                  nullptr, nullptr, y, N, as_stream(stream), "hgin_linear_fwd_bf16");
}

extern "C" int hgin_gemm_nt_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, uint16_t* c,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, const void* b_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gemm_nt_bf16: negative size");
  HGIN_ARG_CHECK(N <= 65535 * 128, "hgin_gemm_nt_bf16: N too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(a && b && c, "hgin_gemm_nt_bf16: NULL operand");
  HGIN_ARG_CHECK(lda >= K && ldb >= K && ldc >= N, "hgin_gemm_nt_bf16: leading dimension too small");
  return launch_nt_bf16<0, uint16_t>(Src2h{a, lda, nullptr, 0, K}, Src2h{b, ldb, nullptr, 0, K}, M, N, K, nullptr,
                                     nullptr, nullptr, nullptr, c, ldc, as_stream(stream), "hgin_gemm_nt_bf16");
}

extern "C" int hgin_gin_mlp_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                                    const float* a2_eps, const float* w, const float* bias, const float* prelu,
                                    const float* accum, float* z, float* y, int64_t M, int64_t N, int64_t K,
                                    const void* w_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gin_mlp_fwd_f32: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * 128, "hgin_gin_mlp_fwd_f32: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && prelu && y, "hgin_gin_mlp_fwd_f32: NULL operand");
  if (int rc = check_a("hgin_gin_mlp_fwd_f32", a1, lda1, k1, a2, lda2, K)) return rc;
  {
    const int rc = try_ws_f32(a1, lda1, k1, a2, lda2, a2_eps, w, bias, prelu, accum, z, y, M, N, K,
                              as_stream(stream), "hgin_gin_mlp_fwd_f32");
    if (rc >= 0) return rc;
  }
  return launch_nt<1>(Src2{a1, lda1, a2, lda2, k1, a2_eps}, Src2{w, K, nullptr, 0, K}, M, N, K, bias, prelu, accum, z, y,
                      N, as_stream(stream), "hgin_gin_mlp_fwd_f32", CombEpi{}, nullptr, w_planes);
}

extern "C" int hgin_linear_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                                   const float* w, const float* bias, float* y, int64_t M, int64_t N, int64_t K,
                                   const void* w_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_linear_fwd_f32: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * 128, "hgin_linear_fwd_f32: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && y, "hgin_linear_fwd_f32: NULL operand");
  if (int rc = check_a("hgin_linear_fwd_f32", a1, lda1, k1, a2, lda2, K)) return rc;
  return launch_nt<2>(Src2{a1, lda1, a2, lda2, k1}, Src2{w, K, nullptr, 0, K}, M, N, K, bias, nullptr, nullptr,
                      nullptr, y, N, as_stream(stream), "hgin_linear_fwd_f32", CombEpi{}, nullptr, w_planes);
}

extern "C" int hgin_gemm_nt_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
                                int64_t M, int64_t N, int64_t K, const void* b_planes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gemm_nt_f32: negative size");
  HGIN_ARG_CHECK(N <= 65535 * 128, "hgin_gemm_nt_f32: N too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(a && b && c, "hgin_gemm_nt_f32: NULL operand");
  HGIN_ARG_CHECK(lda >= K && ldb >= K && ldc >= N, "hgin_gemm_nt_f32: leading dimension too small");
  {
    const int rc = try_wss_plain(a, lda, b, ldb, c, ldc, M, N, K, as_stream(stream), "hgin_gemm_nt_f32");
    if (rc >= 0) return rc;
  }
  return launch_nt<0>(Src2{a, lda, nullptr, 0, K}, Src2{b, ldb, nullptr, 0, K}, M, N, K, nullptr, nullptr, nullptr,
                      nullptr, c, ldc, as_stream(stream), "hgin_gemm_nt_f32", CombEpi{}, nullptr, b_planes);
}

extern "C" int hgin_nt_planes_size(int64_t N, int64_t K, int elem_bytes, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && N >= 0 && K >= 0 && (elem_bytes == 4 || elem_bytes == 2), "hgin_nt_planes_size: bad args");
  *bytes = elem_bytes == 4 ? nt_planes_bytes<float>(N, K) : nt_planes_bytes<uint16_t>(N, K);
  return HGIN_OK;
}

extern "C" int hgin_nt_planes_f32(const float* b, int64_t ldb, int64_t N, int64_t K, void* out, void* stream) {
  return nt_planes<float>(b, ldb, N, K, out, as_stream(stream), "hgin_nt_planes_f32");
}

extern "C" int hgin_nt_planes_bf16(const uint16_t* b, int64_t ldb, int64_t N, int64_t K, void* out, void* stream) {
  return nt_planes<uint16_t>(b, ldb, N, K, out, as_stream(stream), "hgin_nt_planes_bf16");
}


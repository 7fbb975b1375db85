// A5 — GIN MLP update on MFMA, the readout Linear(+PReLU) layers, and the plain NT
// GEMM of the input-gradient backward.
//
// Reference: GINLayer.mlp = Sequential(Linear(K, N), PReLU()) (models.py:236-239) applied at
// models.py:217 (addmm + prelu as two kernels), HeteroConv's torch.stack(outs).sum(0) for the second
// relation into a node type (models.py:286-298), and the readout Sequential(Linear, PReLU) layers applied
// to cat(x_path, raw path features) (models.py:300-330, :362-374).  One kernel computes
//     z = [A1 | A2] W^T + b ;  y = prelu(z) [+ accum]          (EPI 1; EPI 2: y = z; EPI 0: no bias)
// with fp32 operands on the f32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, 157 TF/s chip peak).
// The two A sources remove the readout's torch.cat: columns [0, K1) come from A1, [K1, K) from A2.
//
// Tiling: 256 threads = 4 waves as 2 x 2; a workgroup owns a 128 x 128 output tile, a wave 64 x 64
// (2 x 2 MFMA tiles, 64 accumulator registers).  A and W are both K-contiguous (torch Linear.weight is
// [N, K]), so inside a K-chunk of 8 the MFMA k-step t (0..3) of lane half h (0/1) uses k = 8c + 4h + t:
// every lane reads its operands for four k-steps with ONE ds_read_b128 from a [row][BK + 4] LDS image
// (row stride 36 floats puts the 16 rows of a ds_read_b128 lane group on 16 distinct 4-bank slots).
// Pipelining: the next K-tile's global loads (float4, 8 per thread) are issued into registers before the
// current tile's 64 MFMAs per wave and written to LDS after them, so HBM latency hides under the matrix
// work; 2 barriers per K-tile.
// C/D map of the 32x32 f32 MFMA (gfx950): col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
#include "hgin_common.h"

namespace hgin {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kBM = 128;
constexpr int kBN = 128;
constexpr int kBK = 32;
constexpr int kLds = kBK + 4;

struct Src2 {
  const float* p1;
  int64_t ld1;
  const float* p2;
  int64_t ld2;
  int64_t k1;
};

// 128 rows x 32 floats of [p1 | p2] starting at (row0, k0) -> 4 float4 per thread:
// thread t owns column chunk q = t & 7 of rows (t >> 3) + 32 i.
template <bool kVec>
__device__ __forceinline__ void load_tile(float4 (&r)[4], const Src2& s, int64_t row0, int64_t rows, int64_t k0,
                                          int64_t K, int tid) {
  const int64_t kk = k0 + (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t gr = row0 + (tid >> 3) + 32 * i;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gr < rows) {
      if (kVec && kk + 3 < K && (kk + 3 < s.k1 || kk >= s.k1)) {
        const float* p = kk < s.k1 ? s.p1 + gr * s.ld1 + kk : s.p2 + gr * s.ld2 + (kk - s.k1);
        v = *reinterpret_cast<const float4*>(p);
      } else {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int64_t k = kk + c;
          t[c] = k < K ? (k < s.k1 ? s.p1[gr * s.ld1 + k] : s.p2[gr * s.ld2 + (k - s.k1)]) : 0.0f;
        }
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
    r[i] = v;
  }
}

__device__ __forceinline__ void store_tile(float* __restrict__ dst, const float4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<float4*>(dst + ((tid >> 3) + 32 * i) * kLds + (tid & 7) * 4) = r[i];
}

template <int EPI, bool kVec, bool kPF, int kOcc, bool kPersist>
__global__ __launch_bounds__(256, kOcc) void k_gemm_nt(Src2 A, Src2 B, int64_t M, int64_t N, int64_t K,
                                                    const float* __restrict__ bias, const float* __restrict__ prelu,
                                                    const float* __restrict__ accum, float* __restrict__ Z,
                                                    float* __restrict__ Y, int64_t ldc, bool vec_out) {
  __shared__ __attribute__((aligned(16))) float smem[(kBM + kBN) * kLds];
  float* As = smem;
  float* Bs = smem + kBM * kLds;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1;
  const int wn = wave & 1;
  const int li = lane & 31;
  const int lh = lane >> 5;
  // Persistent: a workgroup walks output tiles tile, tile + gridDim.x, ... (M-tiles inner, so workgroups
  // running together share the W tile in L2).  The first K-tile of the NEXT output tile is fetched into
  // registers during the last K-tile's MFMAs and lands in LDS after the epilogue, so the z / y store tail
  // overlaps the next tile's HBM reads.
  const int64_t tiles_m = (M + kBM - 1) / kBM;
  const int64_t n_tiles = tiles_m * ((N + kBN - 1) / kBN);
  float4 ra[4], rb[4];
  int64_t tile = blockIdx.x;
  if (tile < n_tiles) {
    load_tile<kVec>(ra, A, (tile % tiles_m) * kBM, M, 0, K, tid);
    load_tile<kVec>(rb, B, (tile / tiles_m) * kBN, N, 0, K, tid);
    store_tile(As, ra, tid);
    store_tile(Bs, rb, tid);
  }
  __syncthreads();
  for (; tile < n_tiles; tile += gridDim.x) {
  const int64_t m0 = (tile % tiles_m) * kBM;
  const int64_t n0 = (tile / tiles_m) * kBN;
  const int64_t next = tile + gridDim.x;
  const bool has_next = kPersist && next < n_tiles;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  for (int64_t k0 = 0; k0 < K; k0 += kBK) {
    const bool more = k0 + kBK < K;
    if (kPF && more) {   // next K-tile's global loads stay in flight under this K-tile's MFMAs
      load_tile<kVec>(ra, A, m0, M, k0 + kBK, K, tid);
      load_tile<kVec>(rb, B, n0, N, k0 + kBK, K, tid);
    } else if (kPF && has_next) {   // last K-tile: fetch the next output tile's first K-tile
      load_tile<kVec>(ra, A, (next % tiles_m) * kBM, M, 0, K, tid);
      load_tile<kVec>(rb, B, (next / tiles_m) * kBN, N, 0, K, tid);
    }
#pragma unroll
    for (int c = 0; c < kBK / 8; ++c) {
      float4 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[t] = *reinterpret_cast<const float4*>(As + (wm * 64 + t * 32 + li) * kLds + c * 8 + lh * 4);
        fb[t] = *reinterpret_cast<const float4*>(Bs + (wn * 64 + t * 32 + li) * kLds + c * 8 + lh * 4);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].x, fb[tn].x, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].y, fb[tn].y, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].z, fb[tn].z, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].w, fb[tn].w, acc[tm][tn], 0, 0, 0);
        }
    }
    if (more) {
      __syncthreads();
      if (!kPF) {
        load_tile<kVec>(ra, A, m0, M, k0 + kBK, K, tid);
        load_tile<kVec>(rb, B, n0, N, k0 + kBK, K, tid);
      }
      store_tile(As, ra, tid);
      store_tile(Bs, rb, tid);
      __syncthreads();
    }
  }

  // Epilogue through LDS: the 32x32 C/D layout gives each lane one column, so direct stores are 4 B per
  // lane (store-issue bound: 2 x 64 instructions per wave for z and y).  Each wave instead parks 32 rows x
  // 64 columns of its tile in LDS and writes them back as row-contiguous float4s (8 dwordx4 per lane for
  // each output), reading `accum` the same way.
  constexpr int kLc = 64 + 4;
  const float a_slope = EPI == 1 ? prelu[0] : 0.0f;
  float* Cw = smem + wave * 32 * kLc;
  __syncthreads();   // every wave is done with the A/B tiles
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) Cw[((e & 3) + 8 * (e >> 2) + 4 * lh) * kLc + tn * 32 + li] = acc[tm][tn][e];
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < 8; ++j) {
      const int q = lane + 64 * j;
      const int r = q >> 4;
      const int c = (q & 15) * 4;
      const int64_t row = m0 + wm * 64 + tm * 32 + r;
      const int64_t col = n0 + wn * 64 + c;
      if (row >= M || col >= N) continue;
      const float4 v4 = *reinterpret_cast<const float4*>(Cw + r * kLc + c);
      float o[4] = {v4.x, v4.y, v4.z, v4.w};
      float zz[4];
      const bool full = vec_out && col + 3 < N;
      float acc_in[4] = {0.f, 0.f, 0.f, 0.f};
      if (EPI == 1 && accum) {
        if (full) {
          const float4 a4 = *reinterpret_cast<const float4*>(accum + row * ldc + col);
          acc_in[0] = a4.x; acc_in[1] = a4.y; acc_in[2] = a4.z; acc_in[3] = a4.w;
        } else {
          for (int t = 0; t < 4 && col + t < N; ++t) acc_in[t] = accum[row * ldc + col + t];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bcol = (EPI >= 1 && col + t < N) ? bias[col + t] : 0.0f;
        if (EPI == 2) {
          o[t] = __fadd_rn(o[t], bcol);
        } else if (EPI == 1) {
          zz[t] = __fadd_rn(o[t], bcol);
          float y = zz[t] > 0.0f ? zz[t] : __fmul_rn(a_slope, zz[t]);
          o[t] = accum ? __fadd_rn(acc_in[t], y) : y;
        }
      }
      if (full) {
        *reinterpret_cast<float4*>(Y + row * ldc + col) = make_float4(o[0], o[1], o[2], o[3]);
        if (EPI == 1 && Z) *reinterpret_cast<float4*>(Z + row * ldc + col) = make_float4(zz[0], zz[1], zz[2], zz[3]);
      } else {
        for (int t = 0; t < 4 && col + t < N; ++t) {
          Y[row * ldc + col + t] = o[t];
          if (EPI == 1 && Z) Z[row * ldc + col + t] = zz[t];
        }
      }
    }
    if (tm == 0) __syncthreads();
  }
  if (has_next) {
    __syncthreads();   // every wave has read its C tile out of LDS
    if (!kPF) {
      load_tile<kVec>(ra, A, (next % tiles_m) * kBM, M, 0, K, tid);
      load_tile<kVec>(rb, B, (next / tiles_m) * kBN, N, 0, K, tid);
    }
    store_tile(As, ra, tid);
    store_tile(Bs, rb, tid);
    __syncthreads();
  }
  }  // tile loop
}

// Resident workgroups of one instantiation on this device (VGPR / LDS limited), for the persistent grid.
template <typename Kern>
int64_t resident_blocks(Kern kernel) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess)
    return 1024;
  return (int64_t)cus * (per_cu > 0 ? per_cu : 1);
}

template <int EPI>
int launch_nt(const Src2& a, const Src2& b, int64_t M, int64_t N, int64_t K, const float* bias, const float* prelu,
              const float* accum, float* z, float* y, int64_t ldc, hipStream_t s, const char* what) {
  const bool vec = aligned16(a.p1) && a.ld1 % 4 == 0 && a.k1 % 4 == 0 && (a.k1 == K || (aligned16(a.p2) &&
                   a.ld2 % 4 == 0)) && aligned16(b.p1) && b.ld1 % 4 == 0;
  const bool vec_out = ldc % 4 == 0 && aligned16(y) && (z == nullptr || aligned16(z)) &&
                       (accum == nullptr || aligned16(accum));
  const int64_t n_tiles = ceil_div(M, kBM) * ceil_div(N, kBN);
  static const int variant = [] {
    const char* v = getenv("HGIN_NT_VARIANT");
    return v ? atoi(v) : 0;
  }();
#define HGIN_NT_LAUNCH(PF, OCC, PERSIST)                                                                         \
  do {                                                                                                        \
    auto kern = vec ? k_gemm_nt<EPI, true, PF, OCC, PERSIST> : k_gemm_nt<EPI, false, PF, OCC, PERSIST>;        \
    static int64_t resident[2] = {0, 0};                                                                      \
    if (PERSIST && !resident[vec]) resident[vec] = resident_blocks(kern);                                     \
    const int64_t g = (PERSIST && n_tiles > resident[vec]) ? resident[vec] : n_tiles;                         \
    kern<<<dim3((unsigned)(g > 0 ? g : 1)), 256, 0, s>>>(a, b, M, N, K, bias, prelu, accum, z, y, ldc, vec_out); \
  } while (0)
  // Measured on MI355X (tools/gemm_bench.py, profiles/r01_gemm_variants.txt): register prefetch at 3 waves
  // per SIMD (160 VGPRs) beats 2 waves (172 VGPRs) by 7-14 % and the unpipelined loop by 3-6 %; forcing 4
  // waves spills.  The other variants stay selectable for re-measurement (HGIN_NT_VARIANT).
  switch (variant) {
    case 1: HGIN_NT_LAUNCH(true, 2, true); break;
    case 2: HGIN_NT_LAUNCH(true, 2, false); break;
    default: HGIN_NT_LAUNCH(true, 3, false); break;
  }
#undef HGIN_NT_LAUNCH
  return check_launch(what);
}

int check_a(const char* what, const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2, int64_t K) {
  HGIN_ARG_CHECK(k1 >= 0 && k1 <= K, "%s: k1 out of [0, K]", what);
  HGIN_ARG_CHECK(k1 == 0 || (a1 && lda1 >= k1), "%s: bad A1", what);
  HGIN_ARG_CHECK(k1 == K || (a2 && lda2 >= K - k1), "%s: bad A2", what);
  return HGIN_OK;
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_gin_mlp_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                                    const float* w, const float* bias, const float* prelu, const float* accum, float* z,
                                    float* y, int64_t M, int64_t N, int64_t K, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gin_mlp_fwd_f32: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * (int64_t)kBN, "hgin_gin_mlp_fwd_f32: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && prelu && y, "hgin_gin_mlp_fwd_f32: NULL operand");
  if (int rc = check_a("hgin_gin_mlp_fwd_f32", a1, lda1, k1, a2, lda2, K)) return rc;
  return launch_nt<1>(Src2{a1, lda1, a2, lda2, k1}, Src2{w, K, nullptr, 0, K}, M, N, K, bias, prelu, accum, z, y,
                      N, as_stream(stream), "hgin_gin_mlp_fwd_f32");
}

extern "C" int hgin_linear_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                                   const float* w, const float* bias, float* y, int64_t M, int64_t N, int64_t K,
                                   void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_linear_fwd_f32: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) && N <= 65535 * (int64_t)kBN, "hgin_linear_fwd_f32: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(w && bias && y, "hgin_linear_fwd_f32: NULL operand");
  if (int rc = check_a("hgin_linear_fwd_f32", a1, lda1, k1, a2, lda2, K)) return rc;
  return launch_nt<2>(Src2{a1, lda1, a2, lda2, k1}, Src2{w, K, nullptr, 0, K}, M, N, K, bias, nullptr, nullptr,
                      nullptr, y, N, as_stream(stream), "hgin_linear_fwd_f32");
}

extern "C" int hgin_gemm_nt_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
                                int64_t M, int64_t N, int64_t K, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gemm_nt_f32: negative size");
  HGIN_ARG_CHECK(N <= 65535 * (int64_t)kBN, "hgin_gemm_nt_f32: N too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(a && b && c, "hgin_gemm_nt_f32: NULL operand");
  HGIN_ARG_CHECK(lda >= K && ldb >= K && ldc >= N, "hgin_gemm_nt_f32: leading dimension too small");
  return launch_nt<0>(Src2{a, lda, nullptr, 0, K}, Src2{b, ldb, nullptr, 0, K}, M, N, K, nullptr, nullptr, nullptr,
                      nullptr, c, ldc, as_stream(stream), "hgin_gemm_nt_f32");
}

// A5 — GIN MLP update on MFMA and the plain NT GEMM used by the backward.
//
// Reference: GINLayer.mlp = Sequential(Linear(K, N), PReLU()) (models.py:236-239) applied at
// models.py:217 (addmm + prelu as two kernels), and HeteroConv's torch.stack(outs).sum(0) for the second
// relation into a node type (models.py:286-298).  Here one kernel computes
//     z = A W^T + b ;  y = prelu(z) [+ accum]
// with fp32 operands on the f32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, 64 FLOP/clk/SIMD,
// 157 TF/s chip peak).
//
// Tiling: 256 threads = 4 waves as 2 x 2; a block owns a 128 x 128 output tile, a wave 64 x 64
// (2 x 2 MFMA tiles, 64 accumulator registers).  A and W are both K-contiguous (torch Linear.weight is
// [N, K]), so a K-chunk of 8 is laid out as: MFMA k-step t (0..3), lane half h (0/1) holds k = 8c+4h+t.
// Every lane then reads its A and B operands for four k-steps as ONE ds_read_b128 from a [row][BK+4]
// LDS image (row stride 36 floats: the 16 rows a ds_read_b128 lane group touches land on 16 distinct
// 4-bank slots — conflict-free).  Tiles are staged global -> LDS with float4 loads, BK = 32.
// C/D map of the 32x32 f32 MFMA (gfx950): col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
#include "hgin_common.h"

namespace hgin {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kBM = 128;
constexpr int kBN = 128;
constexpr int kBK = 32;
constexpr int kLds = kBK + 4;

template <bool kVecA, bool kVecB>
__device__ __forceinline__ void stage_tile(float* __restrict__ dst, const float* __restrict__ src, int64_t ld,
                                           int64_t row0, int64_t rows, int64_t k0, int64_t K, int tid) {
  // 128 rows x 32 floats = 1024 float4; 4 per thread.  thread t: q = t & 7, row = (t >> 3) + 32 i
  const int q = tid & 7;
  const int64_t kk = k0 + q * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int64_t gr = row0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gr < rows) {
      const float* p = src + gr * ld + kk;
      if (kVecA && kk + 3 < K) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        if (kk + 0 < K) v.x = p[0];
        if (kk + 1 < K) v.y = p[1];
        if (kk + 2 < K) v.z = p[2];
        if (kk + 3 < K) v.w = p[3];
      }
    }
    *reinterpret_cast<float4*>(dst + r * kLds + q * 4) = v;
  }
  (void)kVecB;
}

// EPI: 0 = plain store of A B^T into Y;  1 = GIN MLP epilogue (bias, PReLU, optional accum, optional Z)
template <int EPI, bool kVec>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ B, int64_t ldb,
                                                    int64_t M, int64_t N, int64_t K,
                                                    const float* __restrict__ bias, const float* __restrict__ prelu,
                                                    const float* __restrict__ accum, float* __restrict__ Z,
                                                    float* __restrict__ Y, int64_t ldc) {
  __shared__ __attribute__((aligned(16))) float smem[(kBM + kBN) * kLds];
  float* As = smem;
  float* Bs = smem + kBM * kLds;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1;
  const int wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const int64_t n0 = (int64_t)blockIdx.y * kBN;
  const int li = lane & 31;
  const int lh = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  for (int64_t k0 = 0; k0 < K; k0 += kBK) {
    stage_tile<kVec, kVec>(As, A, lda, m0, M, k0, K, tid);
    stage_tile<kVec, kVec>(Bs, B, ldb, n0, N, k0, K, tid);
    __syncthreads();
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
    __syncthreads();
  }

  const float a_slope = EPI == 1 ? prelu[0] : 0.0f;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int64_t col = n0 + wn * 64 + tn * 32 + li;
      if (col >= N) continue;
      const float bcol = EPI == 1 ? bias[col] : 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (row >= M) continue;
        const float v = acc[tm][tn][e];
        if (EPI == 0) {
          Y[row * ldc + col] = v;
        } else {
          const float z = __fadd_rn(v, bcol);
          float y = z > 0.0f ? z : __fmul_rn(a_slope, z);
          if (accum) y = __fadd_rn(accum[row * ldc + col], y);
          if (Z) Z[row * ldc + col] = z;
          Y[row * ldc + col] = y;
        }
      }
    }
}

template <int EPI>
int launch_gemm(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t M, int64_t N, int64_t K,
                const float* bias, const float* prelu, const float* accum, float* z, float* y, int64_t ldc,
                hipStream_t s) {
  const bool vec = aligned16(a) && aligned16(b) && lda % 4 == 0 && ldb % 4 == 0;
  dim3 grid((unsigned)ceil_div(M, kBM), (unsigned)ceil_div(N, kBN));
  if (vec)
    k_gemm_nt<EPI, true><<<grid, 256, 0, s>>>(a, lda, b, ldb, M, N, K, bias, prelu, accum, z, y, ldc);
  else
    k_gemm_nt<EPI, false><<<grid, 256, 0, s>>>(a, lda, b, ldb, M, N, K, bias, prelu, accum, z, y, ldc);
  return check_launch(EPI == 1 ? "hgin_gin_mlp_fwd_f32" : "hgin_gemm_nt_f32");
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_gin_mlp_fwd_f32(const float* a, int64_t lda, const float* w, const float* bias,
                                    const float* prelu, const float* accum, float* z, float* y, int64_t M, int64_t N,
                                    int64_t K, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gin_mlp_fwd_f32: negative size");
  HGIN_ARG_CHECK(M < (int64_t(1) << 31) / 1 && N <= 65535 * (int64_t)kBN, "hgin_gin_mlp_fwd_f32: size too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(a && w && bias && prelu && y, "hgin_gin_mlp_fwd_f32: NULL operand");
  HGIN_ARG_CHECK(lda >= K, "hgin_gin_mlp_fwd_f32: lda < K");
  return launch_gemm<1>(a, lda, w, K, M, N, K, bias, prelu, accum, z, y, N, as_stream(stream));
}

extern "C" int hgin_gemm_nt_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
                                int64_t M, int64_t N, int64_t K, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0, "hgin_gemm_nt_f32: negative size");
  HGIN_ARG_CHECK(N <= 65535 * (int64_t)kBN, "hgin_gemm_nt_f32: N too large");
  if (M == 0 || N == 0) return HGIN_OK;
  HGIN_ARG_CHECK(a && b && c, "hgin_gemm_nt_f32: NULL operand");
  HGIN_ARG_CHECK(lda >= K && ldb >= K && ldc >= N, "hgin_gemm_nt_f32: leading dimension too small");
  return launch_gemm<0>(a, lda, b, ldb, M, N, K, nullptr, nullptr, nullptr, nullptr, c, ldc, as_stream(stream));
}

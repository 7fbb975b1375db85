// F3 — fused readout head + MAPE loss.
//
// Reference: the readout head Linear(mlp_layers[-1], 1) (models.py:326-330, applied at :373-374), then
// train.py:38-43: label = y.reshape(-1, 1); loss_value = mape(out, label) = 100 * mean(|(out - y) / y|)
// (train.py:12-13); loss = sqrt(loss_value); loss.backward().  On the GPU that is an addmm with one output
// column plus ~6 elementwise / reduction kernels forward and as many backward, and the reference's
// per-step `mape(out, label).item()` (train.py:50) synchronises the host.
//
// Here: forward = one pass over the [M, K] hidden rows computing out = h·w + b, q = (out - y) / y and
// per-block partial sums of |q| in a fixed order, then one workgroup that adds the partials in block order
// and writes loss_value to device memory — no host sync.  Backward = one pass that
// forms g_out = (100 g / M) * sgn(q) / y per row (the autograd of mape's mul / mean / abs / div), writes
// g_h = g_out w and accumulates g_w = sum g_out h, g_b = sum g_out as fixed-order block partials, then a
// fixed-order final pass.  Deterministic; h may be fp32 or bf16 (cfg5), everything else fp32.
// m_valid (device int32, optional): only rows < *m_valid are labelled — the loss is their mean and the
// other rows get zero gradient (static-shape padded batches replayed from a hipGraph, hgin/graphs.py).
#include "hgin_common.h"

namespace hgin {
namespace {

constexpr int kHeadRows = 256;   // rows per block (both passes)

__device__ __forceinline__ float block_sum_tree(float v, float* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

__device__ __forceinline__ int64_t valid_rows(const int32_t* m_valid, int64_t M) {
  if (!m_valid) return M;
  const int64_t v = m_valid[0];
  return v < M ? (v < 0 ? 0 : v) : M;
}

// thread per row: out[m] = sum_k h[m, k] w[k] (sequential fmaf) + b;  part[blk] = sum |(out - y) / y|
template <typename T>
__global__ __launch_bounds__(256) void k_head_fwd(const T* __restrict__ h, int64_t ldh, int64_t M, int K,
                                                  const float* __restrict__ w, const float* __restrict__ b,
                                                  const float* __restrict__ y, const int32_t* __restrict__ m_valid,
                                                  float* __restrict__ out, float* __restrict__ part) {
  __shared__ float red[256];
  const int64_t m = (int64_t)blockIdx.x * kHeadRows + threadIdx.x;
  const int64_t mv = valid_rows(m_valid, M);
  float a = 0.0f;
  if (m < M) {
    float s = 0.0f;
    const T* row = h + m * ldh;
    for (int k = 0; k < K; ++k) s = __fmaf_rn(Elem<T>::ld(row + k), w[k], s);
    const float o = __fadd_rn(s, b[0]);
    out[m] = o;
    if (m < mv) a = fabsf(__fdiv_rn(__fsub_rn(o, y[m]), y[m]));
  }
  const float tot = block_sum_tree(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Vector variant (K a multiple of the 16-B quad, aligned rows): 8 lanes per row, each lane a 16-B quad of
// columns per pass, so one load instruction covers 8 full 128-B row segments (coalesced) instead of 64
// scattered 4-B reads; the 8 lane partials are combined by a fixed xor butterfly.  A block still owns 256
// rows (each 8-lane group walks 8 of them), so the partial-sum layout matches k_head_fwd.
template <typename T>
struct HQuad;
template <>
struct HQuad<float> {
  static constexpr int E = 4;
  static __device__ __forceinline__ float dot(const float* p, const float* w, float acc) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    acc = __fmaf_rn(v.x, w[0], acc);
    acc = __fmaf_rn(v.y, w[1], acc);
    acc = __fmaf_rn(v.z, w[2], acc);
    return __fmaf_rn(v.w, w[3], acc);
  }
};
template <>
struct HQuad<uint16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ float dot(const uint16_t* p, const float* w, float acc) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc = __fmaf_rn(bf_lo(q[i]), w[2 * i], acc);
      acc = __fmaf_rn(bf_hi(q[i]), w[2 * i + 1], acc);
    }
    return acc;
  }
};

template <typename T>
__global__ __launch_bounds__(256) void k_head_fwd_vec(const T* __restrict__ h, int64_t ldh, int64_t M, int K,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      const float* __restrict__ y, const int32_t* __restrict__ m_valid,
                                                      float* __restrict__ out, float* __restrict__ part) {
  constexpr int E = HQuad<T>::E;
  __shared__ float red[256];
  const int t = threadIdx.x;
  const int grp = t >> 3, gl = t & 7;
  const int64_t mv = valid_rows(m_valid, M);
  float a = 0.0f;
  for (int i = 0; i < kHeadRows / 32; ++i) {
    const int64_t m = (int64_t)blockIdx.x * kHeadRows + grp + 32 * i;
    float s = 0.0f;
    if (m < M)
      for (int c = gl * E; c < K; c += 8 * E) s = HQuad<T>::dot(h + m * ldh + c, w + c, s);
    s = __fadd_rn(s, __shfl_xor(s, 1, 8));
    s = __fadd_rn(s, __shfl_xor(s, 2, 8));
    s = __fadd_rn(s, __shfl_xor(s, 4, 8));
    if (m < M && gl == 0) {
      const float o = __fadd_rn(s, b[0]);
      out[m] = o;
      if (m < mv) a = __fadd_rn(a, fabsf(__fdiv_rn(__fsub_rn(o, y[m]), y[m])));
    }
  }
  const float tot = block_sum_tree(a, red);
  if (t == 0) part[blockIdx.x] = tot;
}

// loss_value = 100 * (sum of the partials in block order) / M
__global__ __launch_bounds__(256) void k_head_loss_final(const float* __restrict__ part, int64_t nblk, int64_t M,
                                                         const int32_t* __restrict__ m_valid,
                                                         float* __restrict__ loss_value) {
  __shared__ float red[256];
  float s = 0.0f;
  for (int64_t i = threadIdx.x; i < nblk; i += 256) s = __fadd_rn(s, part[i]);
  const float tot = block_sum_tree(s, red);
  if (threadIdx.x == 0) {
    loss_value[0] = __fmul_rn(100.0f, __fdiv_rn(tot, (float)valid_rows(m_valid, M)));
  }
}

// 256 threads = 8 row lanes x 32 columns.  Phase 1: thread t computes g_out of row t of the block's chunk
// into LDS.  Phase 2: thread (r, c) walks columns k = k0 + c, rows r, r + 8, ... writing g_h and summing
// g_out * h in order; the 8 row lanes are then added in lane order.  part_w: [K][nblk], part_b: [nblk].
template <typename T>
__global__ __launch_bounds__(256) void k_head_bwd(const T* __restrict__ h, int64_t ldh, int64_t M, int K,
                                                  const float* __restrict__ w, const float* __restrict__ y,
                                                  const float* __restrict__ out, const float* __restrict__ g_loss,
                                                  const int32_t* __restrict__ m_valid, T* __restrict__ g_h, int64_t ldg,
                                                  float* __restrict__ part_w, float* __restrict__ part_b) {
  __shared__ float gbuf[kHeadRows];
  __shared__ float red[256];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kHeadRows;
  const int64_t n = M - r0 < kHeadRows ? M - r0 : kHeadRows;
  {
    const int64_t m = r0 + t;
    const int64_t mv = valid_rows(m_valid, M);
    float g = 0.0f;
    if (m < mv) {
      const float q = __fdiv_rn(__fsub_rn(out[m], y[m]), y[m]);
      const float gm = __fdiv_rn(__fmul_rn(100.0f, g_loss[0]), (float)mv);  // d(100 * mean)
      g = __fdiv_rn(__fmul_rn(gm, sgn(q)), y[m]);                               // abs, then the / y
    }
    gbuf[t] = g;
  }
  const float gb = block_sum_tree(gbuf[t], red);   // also orders the gbuf writes before phase 2
  if (t == 0) part_b[blockIdx.x] = gb;
  const int rl = t >> 5, c = t & 31;
  for (int k0 = 0; k0 < K; k0 += 32) {
    const int k = k0 + c;
    float acc = 0.0f;
    if (k < K) {
      const float wk = w[k];
      for (int64_t i = rl; i < n; i += 8) {
        const float g = gbuf[i];
        const int64_t m = r0 + i;
        acc = __fmaf_rn(g, Elem<T>::ld(h + m * ldh + k), acc);
        if (g_h) Elem<T>::st(g_h + m * ldg + k, __fmul_rn(g, wk));
      }
    }
    red[t] = acc;
    __syncthreads();
    if (rl == 0 && k < K) {
      float s = 0.0f;
      for (int j = 0; j < 8; ++j) s = __fadd_rn(s, red[j * 32 + c]);
      part_w[(int64_t)k * gridDim.x + blockIdx.x] = s;
    }
    __syncthreads();
  }
}

// one workgroup per output (K weights + the bias): fixed-order sum of the block partials
__global__ __launch_bounds__(256) void k_head_bwd_final(const float* __restrict__ part_w,
                                                        const float* __restrict__ part_b, int64_t nblk, int K,
                                                        float* __restrict__ g_w, float* __restrict__ g_b) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  const float* p = j < K ? part_w + (int64_t)j * nblk : part_b;
  float s = 0.0f;
  for (int64_t i = threadIdx.x; i < nblk; i += 256) s = __fadd_rn(s, p[i]);
  const float tot = block_sum_tree(s, red);
  if (threadIdx.x == 0) {
    if (j < K) g_w[j] = tot;
    else g_b[0] = tot;
  }
}

template <typename T>
int head_fwd(const char* what, const T* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* b,
             const float* y, const int32_t* m_valid, float* out, float* loss_value, void* ws, size_t ws_bytes,
             void* stream) {
  HGIN_ARG_CHECK(M > 0 && K > 0 && K <= 4096 && ldh >= K, "%s: bad sizes (M %lld, K %lld)", what, (long long)M,
                 (long long)K);
  HGIN_ARG_CHECK(h && w && b && y && out && loss_value, "%s: NULL operand", what);
  size_t need = 0;
  hgin_head_mape_workspace_size(M, K, &need);
  if (!ws || ws_bytes < need) {
    set_error("%s: workspace %zu < %zu", what, ws_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  const int64_t nblk = ceil_div(M, kHeadRows);
  float* part = static_cast<float*>(ws);
  constexpr int E = HQuad<T>::E;
  if (K % E == 0 && ldh % E == 0 && aligned16(h))
    k_head_fwd_vec<T><<<(unsigned)nblk, 256, 0, s>>>(h, ldh, M, (int)K, w, b, y, m_valid, out, part);
  else
    k_head_fwd<T><<<(unsigned)nblk, 256, 0, s>>>(h, ldh, M, (int)K, w, b, y, m_valid, out, part);
  k_head_loss_final<<<1, 256, 0, s>>>(part, nblk, M, m_valid, loss_value);
  return check_launch(what);
}

template <typename T>
int head_bwd(const char* what, const T* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* y,
             const float* out, const float* g_loss, const int32_t* m_valid, T* g_h, int64_t ldg, float* g_w,
             float* g_b, void* ws, size_t ws_bytes, void* stream) {
  HGIN_ARG_CHECK(M > 0 && K > 0 && K <= 4096 && ldh >= K, "%s: bad sizes", what);
  HGIN_ARG_CHECK(h && w && y && out && g_loss && g_w && g_b, "%s: NULL operand", what);
  HGIN_ARG_CHECK(!g_h || ldg >= K, "%s: ldg < K", what);
  size_t need = 0;
  hgin_head_mape_workspace_size(M, K, &need);
  if (!ws || ws_bytes < need) {
    set_error("%s: workspace %zu < %zu", what, ws_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  const int64_t nblk = ceil_div(M, kHeadRows);
  float* part_w = static_cast<float*>(ws);
  float* part_b = part_w + nblk * K;
  k_head_bwd<T><<<(unsigned)nblk, 256, 0, s>>>(h, ldh, M, (int)K, w, y, out, g_loss, m_valid, g_h, ldg, part_w,
                                               part_b);
  k_head_bwd_final<<<(unsigned)(K + 1), 256, 0, s>>>(part_w, part_b, nblk, (int)K, g_w, g_b);
  return check_launch(what);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_head_mape_workspace_size(int64_t M, int64_t K, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && M >= 0 && K >= 0, "hgin_head_mape_workspace_size: bad args");
  const int64_t nblk = ceil_div(M > 0 ? M : 1, kHeadRows);
  *bytes = sizeof(float) * (size_t)(nblk * (K + 1)) + 256;
  return HGIN_OK;
}

extern "C" int hgin_head_mape_fwd_f32(const float* h, int64_t ldh, int64_t M, int64_t K, const float* w,
                                      const float* b, const float* y, const int32_t* m_valid, float* out,
                                      float* loss_value, void* ws, size_t ws_bytes, void* stream) {
  return head_fwd<float>("hgin_head_mape_fwd_f32", h, ldh, M, K, w, b, y, m_valid, out, loss_value, ws, ws_bytes,
                         stream);
}

extern "C" int hgin_head_mape_fwd_bf16(const uint16_t* h, int64_t ldh, int64_t M, int64_t K, const float* w,
                                       const float* b, const float* y, const int32_t* m_valid, float* out,
                                       float* loss_value, void* ws, size_t ws_bytes, void* stream) {
  return head_fwd<uint16_t>("hgin_head_mape_fwd_bf16", h, ldh, M, K, w, b, y, m_valid, out, loss_value, ws,
                            ws_bytes, stream);
}

extern "C" int hgin_head_mape_bwd_f32(const float* h, int64_t ldh, int64_t M, int64_t K, const float* w,
                                      const float* y, const float* out, const float* g_loss, const int32_t* m_valid,
                                      float* g_h, int64_t ldg, float* g_w, float* g_b, void* ws, size_t ws_bytes,
                                      void* stream) {
  return head_bwd<float>("hgin_head_mape_bwd_f32", h, ldh, M, K, w, y, out, g_loss, m_valid, g_h, ldg, g_w, g_b, ws,
                         ws_bytes, stream);
}

extern "C" int hgin_head_mape_bwd_bf16(const uint16_t* h, int64_t ldh, int64_t M, int64_t K, const float* w,
                                       const float* y, const float* out, const float* g_loss,
                                       const int32_t* m_valid, uint16_t* g_h, int64_t ldg, float* g_w, float* g_b,
                                       void* ws, size_t ws_bytes, void* stream) {
  return head_bwd<uint16_t>("hgin_head_mape_bwd_bf16", h, ldh, M, K, w, y, out, g_loss, m_valid, g_h, ldg, g_w, g_b,
                            ws, ws_bytes, stream);
}

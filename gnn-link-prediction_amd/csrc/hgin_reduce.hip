// A9 — backward of the GIN update's elementwise parts, with deterministic reductions.
//
// Reference: autograd of PReLU (models.py:238), Linear's bias (models.py:237) and of the self term
// `(1 + eps) * x_r` (models.py:212-215), reached from loss.backward() at train.py:43.  On the GPU,
// PyTorch reduces these with atomics / split reductions whose order varies; here every reduction has a
// fixed shape — per block: a fixed per-thread order over a 256-row chunk, then an LDS combine in fixed
// order; then one pass that adds the block partials in block order — so gradients are bitwise
// reproducible run to run.  The element type of the row streams is fp32 or bf16 (cfg5); reductions and
// arithmetic are fp32 either way.
#include "hgin_common.h"

namespace hgin {
namespace {

constexpr int kMinRowsPerBlock = 64;   // workspace sizing: the most blocks any variant launches

// Rows per block / rows in flight per thread (tools/rows_bench.py, profiles/r01_rows_variants.txt): 256-row blocks;
// 4 rows in flight for fp32 rows (2-4 % faster), 1 for bf16 (4 in flight was 20-40 % slower there): u = 0 chooses by
// element type; non-temporal inputs for fp32 (nt -1), outputs by size (nt_out -1).  (The round-1 switches that set
// these are gone: the defaults are the measured choices.)
struct RowsCfg {
  int rpb = 256;
  int u = 0;
  int nt = -1;       // -1: fp32 on, bf16 off (measured)
  int nt_out = -1;   // -1: by output size
};
const RowsCfg& rows_cfg() {
  static const RowsCfg c{};
  return c;
}

__device__ __forceinline__ float block_sum_fixed(float v, float* red) {
  // fixed-order tree over 256 threads (same pairing every launch)
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

// VEC = 4: each thread owns 4 consecutive columns (16-B fp32 / 8-B bf16 accesses; needs N % 4 == 0 and
// aligned rows).
template <int VEC, typename T>
struct RowVec {
  static __device__ __forceinline__ void load(const T* p, float (&v)[VEC]) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = Elem<T>::ld(p + q);
  }
  static __device__ __forceinline__ void store(T* p, const float (&v)[VEC]) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) Elem<T>::st(p + q, v[q]);
  }
};
template <>
struct RowVec<4, float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <>
struct RowVec<4, uint16_t> {
  static __device__ __forceinline__ void load(const uint16_t* p, float (&v)[4]) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = bf_lo(t.x); v[1] = bf_hi(t.x); v[2] = bf_lo(t.y); v[3] = bf_hi(t.y);
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float (&v)[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
  }
};

// Read-once operand streams (g_y / z, g / x_dst) loaded non-temporally so they do not displace the output,
// which the dW / dX GEMMs read next.  fp32: row kernel 5-15 % faster, cfg2 step -0.8 %; bf16: mixed in
// isolation, cfg5 step equal, so off (HGIN_ROWS_NT=0/1 forces; profiles/r01/s6/rows_nt.txt).
typedef float rows_f4v __attribute__((ext_vector_type(4)));
typedef unsigned rows_u2v __attribute__((ext_vector_type(2)));
template <bool NT, int VEC, typename T>
__device__ __forceinline__ void rows_load(const T* p, float (&v)[VEC]) {
  if constexpr (NT && VEC == 4 && sizeof(T) == 4) {
    const rows_f4v t = __builtin_nontemporal_load(reinterpret_cast<const rows_f4v*>(p));
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (NT && VEC == 4 && sizeof(T) == 2) {
    const rows_u2v t = __builtin_nontemporal_load(reinterpret_cast<const rows_u2v*>(p));
    v[0] = bf_lo(t.x); v[1] = bf_hi(t.x); v[2] = bf_lo(t.y); v[3] = bf_hi(t.y);
  } else {
    RowVec<VEC, T>::load(p, v);
  }
}

// MODE 0: PReLU backward.  in0 = g_y, in1 = z; out = g_z; colsum(g_z) -> part_col; sum(z<=0 ? z*g : 0) -> part_s
//         (the column sums and the slope sum use the fp32 g_z before any bf16 rounding of the output)
// MODE 1: combine backward.  in0 = g (self-term columns), in1 = x_dst; out = s*g (optional);
//         part_s = sum(g * x_dst); no column sums.
// Non-temporal store of one output group (nt_out: outputs far beyond the caches, read back by a later kernel).
template <int VEC, typename T>
__device__ __forceinline__ void rows_store(T* p, const float (&v)[VEC], bool nt) {
  if constexpr (VEC == 4 && sizeof(T) == 4) {
    if (nt) {
      __builtin_nontemporal_store(rows_f4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<rows_f4v*>(p));
      return;
    }
  } else if constexpr (VEC == 4 && sizeof(T) == 2) {
    if (nt) {
      __builtin_nontemporal_store(rows_u2v{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])}, reinterpret_cast<rows_u2v*>(p));
      return;
    }
  }
  RowVec<VEC, T>::store(p, v);
}

template <int MODE, int VEC, typename T, int kU, bool NT = false>
__global__ __launch_bounds__(256) void k_rows_bwd(const T* __restrict__ in0, int64_t ld0, const T* __restrict__ in1,
                                                  int64_t ld1, int64_t M, int N, const float* __restrict__ scalar,
                                                  T* __restrict__ out, int64_t ldo, float* __restrict__ part_col,
                                                  float* __restrict__ part_s, int rows_per_block, bool nt_out) {
  __shared__ float red[256 * VEC];
  const int t = threadIdx.x;
  const int NU = N / VEC;                 // column units
  const int CW = NU < 256 ? NU : 256;
  const int RL = 256 / CW;
  const bool active = t < CW * RL;
  const int u0 = t % CW;
  const int rl = t / CW;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  float sc = 0.0f;
  if (MODE == 0) sc = scalar[0];
  else sc = __fadd_rn(1.0f, scalar[0]);
  float ssum = 0.0f;
  const int iters = (NU + CW - 1) / CW;
  for (int it = 0; it < iters; ++it) {
    const int c = (u0 + it * CW) * VEC;
    float csum[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) csum[q] = 0.0f;
    if (active && c < N) {
      // one row: fixed per-thread order (rows r0 + rl, r0 + rl + RL, ...), identical for any unrolling
      auto row = [&](int64_t r, const float (&g)[VEC], const float (&x)[VEC]) {
        float o[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          if (MODE == 0) {
            const bool pos = x[q] > 0.0f;
            o[q] = pos ? g[q] : __fmul_rn(sc, g[q]);
            csum[q] = __fadd_rn(csum[q], o[q]);
            if (!pos) ssum = __fadd_rn(ssum, __fmul_rn(x[q], g[q]));
          } else {
            o[q] = __fmul_rn(sc, g[q]);
            ssum = __fadd_rn(ssum, __fmul_rn(g[q], x[q]));
          }
        }
        if (MODE == 0 || out) rows_store<VEC, T>(out + r * ldo + c, o, nt_out);
      };
      int64_t r = r0 + rl;     // kU rows' loads in flight together
      for (; r + (kU - 1) * RL < r1; r += kU * RL) {
        float g[kU][VEC], x[kU][VEC];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          rows_load<NT, VEC, T>(in0 + (r + u * RL) * ld0 + c, g[u]);
          rows_load<NT, VEC, T>(in1 + (r + u * RL) * ld1 + c, x[u]);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) row(r + u * RL, g[u], x[u]);
      }
      for (; r < r1; r += RL) {
        float g[VEC], x[VEC];
        rows_load<NT, VEC, T>(in0 + r * ld0 + c, g);
        rows_load<NT, VEC, T>(in1 + r * ld1 + c, x);
        row(r, g, x);
      }
    }
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) red[t * VEC + q] = csum[q];
      __syncthreads();
      if (active && rl == 0 && c < N) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          float tot = 0.0f;
          for (int j = 0; j < RL; ++j) tot = __fadd_rn(tot, red[(j * CW + u0) * VEC + q]);
          part_col[(int64_t)(c + q) * gridDim.x + blockIdx.x] = tot;   // [N][nblk]: coalesced final pass
        }
      }
      __syncthreads();
    }
  }
  const float bs = block_sum_fixed(ssum, red);
  if (t == 0) part_s[blockIdx.x] = bs;
}

template <int MODE, typename T>
void launch_rows_bwd(bool vec, unsigned nblk, int rpb, hipStream_t s, const T* in0, int64_t ld0, const T* in1,
                     int64_t ld1, int64_t M, int N, const float* scalar, T* out, int64_t ldo, float* part_col,
                     float* part_s) {
  const bool u4 = rows_cfg().u == 4 || (rows_cfg().u == 0 && sizeof(T) == 4);
  const bool nt = rows_cfg().nt < 0 ? sizeof(T) == 4 : rows_cfg().nt == 1;
  // non-temporal output stores once the output exceeds 512 MiB (HGIN_ROWS_NT_OUT = 0 / 1 forces)
  const bool nt_out = rows_cfg().nt_out < 0 ? M * N * (int64_t)sizeof(T) > (int64_t(512) << 20) : rows_cfg().nt_out == 1;
  HGIN_TRACE("k_rows_bwd<%d,%s,N%d>", MODE, sizeof(T) == 4 ? "f32" : "bf16", N);
  if (vec && nt) {
    if (u4)
      k_rows_bwd<MODE, 4, T, 4, true><<<nblk, 256, 0, s>>>(in0, ld0, in1, ld1, M, N, scalar, out, ldo, part_col, part_s, rpb, nt_out);
    else
      k_rows_bwd<MODE, 4, T, 1, true><<<nblk, 256, 0, s>>>(in0, ld0, in1, ld1, M, N, scalar, out, ldo, part_col, part_s, rpb, nt_out);
  } else if (vec && u4)
    k_rows_bwd<MODE, 4, T, 4><<<nblk, 256, 0, s>>>(in0, ld0, in1, ld1, M, N, scalar, out, ldo, part_col, part_s, rpb, nt_out);
  else if (vec)
    k_rows_bwd<MODE, 4, T, 1><<<nblk, 256, 0, s>>>(in0, ld0, in1, ld1, M, N, scalar, out, ldo, part_col, part_s, rpb, nt_out);
  else
    k_rows_bwd<MODE, 1, T, 1><<<nblk, 256, 0, s>>>(in0, ld0, in1, ld1, M, N, scalar, out, ldo, part_col, part_s, rpb, nt_out);
}

template <typename T>
bool rows_vec_ok(int64_t N, const T* a, int64_t lda, const T* b, int64_t ldb, const T* c, int64_t ldc) {
  const uintptr_t align = 4 * sizeof(T);
  auto ok = [&](const T* p) { return (reinterpret_cast<uintptr_t>(p) & (align - 1)) == 0; };
  return N % 4 == 0 && ok(a) && lda % 4 == 0 && ok(b) && ldb % 4 == 0 && (c == nullptr || (ok(c) && ldc % 4 == 0));
}

// Sum block partials in a fixed order (one workgroup): strided per-thread sums + fixed tree.
__global__ __launch_bounds__(256) void k_final_scalar(const float* __restrict__ part, int64_t nblk,
                                                      float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.0f;
  for (int64_t b = threadIdx.x; b < nblk; b += 256) s = __fadd_rn(s, part[b]);
  const float tot = block_sum_fixed(s, red);
  if (threadIdx.x == 0) out[0] = tot;
}

// Per-column sums (workgroups 0..N-1, one per column) and the slope sum (workgroup N) of the block partials in
// one launch: strided per-thread sums + the fixed tree, so the order is fixed.
__global__ __launch_bounds__(256) void k_final_cols_scalar(const float* __restrict__ part_col,
                                                           const float* __restrict__ part_s, int64_t nblk, int N,
                                                           float* __restrict__ out_col, float* __restrict__ out_s) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  const float* p = c < N ? part_col + (int64_t)c * nblk : part_s;
  float s = 0.0f;
  for (int64_t b = threadIdx.x; b < nblk; b += 256) s = __fadd_rn(s, p[b]);
  const float tot = block_sum_fixed(s, red);
  if (threadIdx.x == 0) {
    if (c < N) out_col[c] = tot;
    else out_s[0] = tot;
  }
}

size_t prelu_ws_bytes(int64_t M, int64_t N) {
  const int64_t nblk = ceil_div(M > 0 ? M : 1, kMinRowsPerBlock);
  return align_up(sizeof(float) * (size_t)(nblk * N), 256) + align_up(sizeof(float) * (size_t)nblk, 256);
}

template <typename T>
int prelu_bwd(const char* what, const T* g_y, int64_t ld_gy, const T* z, int64_t M, int64_t N, const float* prelu,
              T* g_z, float* g_prelu, float* g_bias, void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && N < (1 << 24), "%s: bad sizes", what);
  HGIN_ARG_CHECK(g_prelu && g_bias && prelu, "%s: NULL output", what);
  const size_t need = prelu_ws_bytes(M, N);
  if (workspace_bytes < need || !workspace) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == 0) {
    int rc = N ? memset_async(g_bias, 0, sizeof(float) * (size_t)N, s, what) : HGIN_OK;
    if (rc == HGIN_OK) rc = memset_async(g_prelu, 0, sizeof(float), s, what);
    return rc;
  }
  HGIN_ARG_CHECK(g_y && z && g_z && ld_gy >= N, "%s: NULL operand or ld_gy < N", what);
  const int rpb = rows_cfg().rpb;
  const int64_t nblk = ceil_div(M, rpb);
  float* part_col = static_cast<float*>(workspace);
  float* part_s = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                           align_up(sizeof(float) * (size_t)(nblk * N), 256));
  launch_rows_bwd<0, T>(rows_vec_ok<T>(N, g_y, ld_gy, z, N, g_z, N), (unsigned)nblk, rpb, s, g_y, ld_gy, z, N, M, (int)N,
                        prelu, g_z, N, part_col, part_s);
  k_final_cols_scalar<<<(unsigned)N + 1, 256, 0, s>>>(part_col, part_s, nblk, (int)N, g_bias, g_prelu);
  return check_launch(what);
}

template <typename T>
int combine_bwd(const char* what, const T* g, int64_t ld_g, const T* x_dst, int64_t ld_dst, int64_t n_rows,
                int64_t f_dst, const float* eps, T* g_x_dst, int64_t ld_gx, float* g_eps, void* workspace,
                size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(n_rows >= 0 && f_dst >= 0 && f_dst < (1 << 24), "%s: bad sizes", what);
  HGIN_ARG_CHECK(eps && g_eps, "%s: NULL eps/g_eps", what);
  const size_t need = align_up(sizeof(float) * (size_t)ceil_div(n_rows > 0 ? n_rows : 1, kMinRowsPerBlock), 256);
  if (workspace_bytes < need || !workspace) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if (n_rows == 0 || f_dst == 0) return memset_async(g_eps, 0, sizeof(float), s, what);
  HGIN_ARG_CHECK(g && x_dst, "%s: NULL operand", what);
  const int rpb = rows_cfg().rpb;
  const int64_t nblk = ceil_div(n_rows, rpb);
  float* part_s = static_cast<float*>(workspace);
  launch_rows_bwd<1, T>(rows_vec_ok<T>(f_dst, g, ld_g, x_dst, ld_dst, g_x_dst, ld_gx), (unsigned)nblk, rpb, s, g, ld_g,
                        x_dst, ld_dst, n_rows, (int)f_dst, eps, g_x_dst, ld_gx, nullptr, part_s);
  k_final_scalar<<<1, 256, 0, s>>>(part_s, nblk, g_eps);
  return check_launch(what);
}

// Self-term weight gradient of a GINConv whose inputs are data (ops._GINConvFn's one-TN-pass form, first
// layer; models.py:210-217 reached from train.py:43): G [N, KG] = g_z^T [aggregate | x_dst] from the dW GEMM.
//   g_w[:, :f] = G[:, :f];   concat: g_w[:, f:] = (1 + eps) G[:, f:]   (add: g_w is G[:, :f] only)
//   g_eps = sum_{n, j < KG - f} W[n, w0 + j] G[n, f + j]          (concat: w0 = f; add: w0 = 0)
// Element i of the flattened G goes to thread i % (blocks * 256) in a fixed order; per-block fixed trees,
// then k_final_scalar over the block partials.  Replaces 3-5 torch launches (scale, cat, product, sum).
constexpr int kSelfPerThread = 8;

int64_t self_wgrad_blocks(int64_t N, int64_t KG) {
  const int64_t b = ceil_div(N * KG > 0 ? N * KG : 1, (int64_t)256 * kSelfPerThread);
  return b < 512 ? b : 512;
}

__global__ __launch_bounds__(256) void k_self_wgrad(const float* __restrict__ G, int64_t ldg,
                                                    const float* __restrict__ W, int64_t ldw, int64_t N, int64_t KG,
                                                    int64_t f, int64_t w0, int concat, const float* __restrict__ eps,
                                                    float* __restrict__ gw, int64_t ldgw, float* __restrict__ part) {
  __shared__ float red[256];
  const float sc = __fadd_rn(1.0f, eps[0]);
  const int64_t total = N * KG;
  const int64_t stride = (int64_t)gridDim.x * 256;
  float s = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const int64_t n = i / KG, k = i - n * KG;
    const float v = G[n * ldg + k];
    if (k < f) {
      gw[n * ldgw + k] = v;
    } else {
      s = __fadd_rn(s, __fmul_rn(W[n * ldw + w0 + (k - f)], v));
      if (concat) gw[n * ldgw + k] = __fmul_rn(sc, v);
    }
  }
  const float bs = block_sum_fixed(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = bs;
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_self_wgrad_workspace_size(int64_t N, int64_t KG, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && N >= 0 && KG >= 0, "hgin_self_wgrad_workspace_size: bad args");
  *bytes = align_up(sizeof(float) * (size_t)self_wgrad_blocks(N, KG), 256);
  return HGIN_OK;
}

extern "C" int hgin_self_wgrad_f32(const float* G, int64_t ldg, const float* W, int64_t ldw, int64_t N, int64_t KG,
                                   int64_t f, int concat, const float* eps, float* g_w, int64_t ld_gw, float* g_eps,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(N >= 0 && KG >= 0 && f >= 0 && f <= KG, "hgin_self_wgrad_f32: bad sizes");
  HGIN_ARG_CHECK(G && W && eps && g_w && g_eps, "hgin_self_wgrad_f32: NULL operand");
  HGIN_ARG_CHECK(ldg >= KG && ld_gw >= (concat ? KG : f), "hgin_self_wgrad_f32: leading dimension too small");
  HGIN_ARG_CHECK(ldw >= (concat ? KG : KG - f), "hgin_self_wgrad_f32: W narrower than the self block");
  const int64_t nblk = self_wgrad_blocks(N, KG);
  if (!workspace || workspace_bytes < sizeof(float) * (size_t)nblk) {
    set_error("hgin_self_wgrad_f32: workspace %zu < %zu", workspace_bytes, sizeof(float) * (size_t)nblk);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  k_self_wgrad<<<(unsigned)nblk, 256, 0, s>>>(G, ldg, W, ldw, N, KG, f, concat ? f : 0, concat, eps, g_w, ld_gw, part);
  k_final_scalar<<<1, 256, 0, s>>>(part, nblk, g_eps);
  return check_launch("hgin_self_wgrad_f32");
}

extern "C" int hgin_prelu_bwd_workspace_size(int64_t M, int64_t N, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && M >= 0 && N >= 0, "hgin_prelu_bwd_workspace_size: bad args");
  *bytes = prelu_ws_bytes(M, N);
  return HGIN_OK;
}

extern "C" int hgin_prelu_bwd_f32(const float* g_y, int64_t ld_gy, const float* z, int64_t M, int64_t N,
                                  const float* prelu, float* g_z, float* g_prelu, float* g_bias, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  return prelu_bwd<float>("hgin_prelu_bwd_f32", g_y, ld_gy, z, M, N, prelu, g_z, g_prelu, g_bias, workspace,
                          workspace_bytes, stream);
}

extern "C" int hgin_prelu_bwd_bf16(const uint16_t* g_y, int64_t ld_gy, const uint16_t* z, int64_t M, int64_t N,
                                   const float* prelu, uint16_t* g_z, float* g_prelu, float* g_bias, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  return prelu_bwd<uint16_t>("hgin_prelu_bwd_bf16", g_y, ld_gy, z, M, N, prelu, g_z, g_prelu, g_bias, workspace,
                             workspace_bytes, stream);
}

extern "C" int hgin_combine_bwd_workspace_size(int64_t n_rows, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && n_rows >= 0, "hgin_combine_bwd_workspace_size: bad args");
  *bytes = align_up(sizeof(float) * (size_t)ceil_div(n_rows > 0 ? n_rows : 1, kMinRowsPerBlock), 256);
  return HGIN_OK;
}

extern "C" int hgin_combine_bwd_f32(const float* g, int64_t ld_g, const float* x_dst, int64_t ld_dst, int64_t n_rows,
                                    int64_t f_dst, const float* eps, float* g_x_dst, int64_t ld_gx, float* g_eps,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  return combine_bwd<float>("hgin_combine_bwd_f32", g, ld_g, x_dst, ld_dst, n_rows, f_dst, eps, g_x_dst, ld_gx, g_eps,
                            workspace, workspace_bytes, stream);
}

extern "C" int hgin_combine_bwd_bf16(const uint16_t* g, int64_t ld_g, const uint16_t* x_dst, int64_t ld_dst,
                                     int64_t n_rows, int64_t f_dst, const float* eps, uint16_t* g_x_dst, int64_t ld_gx,
                                     float* g_eps, void* workspace, size_t workspace_bytes, void* stream) {
  return combine_bwd<uint16_t>("hgin_combine_bwd_bf16", g, ld_g, x_dst, ld_dst, n_rows, f_dst, eps, g_x_dst, ld_gx,
                               g_eps, workspace, workspace_bytes, stream);
}

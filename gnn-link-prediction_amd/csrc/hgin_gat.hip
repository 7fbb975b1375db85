// F4 widening — HetroGAT's graph attention (models.py:380-506: PyG 2.0.2 GATConv inside the same HeteroConv),
// on the CSR / CSC machinery of the GIN path.  Per relation, with x_s = x_src W_src^T, x_d = x_dst W_dst^T viewed as
// [N, H, C] (the projections are the NT GEMMs of hgin_gemm_nt.hip) and the edge list already self-loop adjusted
// (GATConv removes (i, i) edges and adds (i, i) for i < min(N_src, N_dst), bipartite relations included):
//   a_s[n, h] = sum_c x_s[n, h, c] att_src[h, c]          (k_gat_logits; a_d likewise)
//   e_k       = leaky_relu(a_s[j_k, h] + a_d[i, h], 0.2)   for edge k = (j_k -> i)
//   alpha_k   = exp(e_k - max_row e) / (sum_row exp(e - max_row e) + 1e-16)        (PyG softmax, per dst and head)
//   out[i, h, :] = sum_k alpha_k x_s[j_k, h, :] + bias [+ accum]                  (k_gat_fwd, CSR by destination)
// Backward (autograd of the same expression, train.py:43):
//   g_alpha_k = <g_out[i, h, :], x_s[j_k, h, :]>,  S_i = sum_k alpha_k g_alpha_k,  g_e_k = alpha_k (g_alpha_k - S_i),
//   g_pre_k = g_e_k * (pre_k > 0 ? 1 : 0.2),  g_a_d[i, h] = sum_k g_pre_k,  g_x_d[i, h, :] = g_a_d[i, h] att_dst[h, :]
//                                                                                  (k_gat_bwd_dst, CSR)
//   g_x_s[j, h, :] = sum_k alpha_k g_out[i_k, h, :] + g_a_s[j, h] att_src[h, :],  g_a_s[j, h] = sum_k g_pre_k
//                                                                                  (k_gat_bwd_src, CSC)
//   g_att_src[h, c] = sum_j g_a_s[j, h] x_s[j, h, c], g_att_dst likewise, g_bias = sum_i g_out[i, :]  (k_gat_wsum)
// Deterministic: every sum runs in a fixed order (edges in CSR / CSC order = the edge list's order within a row, as
// the reference's scatter_add; column sums by fixed row blocks, then blocks in order); no atomics.  One thread per
// (row, head): the GAT widths are small (H * C = 64 .. 128 here), and the walk over a row's edges is short.
#include "hgin_common.h"

namespace hgin {
namespace {

__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.0f ? x : __fmul_rn(slope, x); }

__global__ __launch_bounds__(256) void k_gat_logits(const float* __restrict__ x, int64_t ldx, int64_t n, int H, int C,
                                                    const float* __restrict__ att, float* __restrict__ a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * H) return;
  const int64_t r = t / H;
  const int h = (int)(t % H);
  const float* xr = x + r * ldx + (int64_t)h * C;
  const float* at = att + h * C;
  float s = 0.0f;
  for (int c = 0; c < C; ++c) s = __fadd_rn(s, __fmul_rn(xr[c], at[c]));
  a[t] = s;
}

__global__ __launch_bounds__(256) void k_gat_fwd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                 int64_t n_dst, int H, int C, const float* __restrict__ xs,
                                                 int64_t ldxs, const float* __restrict__ as,
                                                 const float* __restrict__ ad, float slope,
                                                 const float* __restrict__ bias, const float* __restrict__ accum,
                                                 int64_t ld_acc, float* __restrict__ alpha, float* __restrict__ out,
                                                 int64_t ldo) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_dst * H) return;
  const int64_t i = t / H;
  const int h = (int)(t % H);
  const int rb = rowptr[i], re = rowptr[i + 1];
  const float adv = ad ? ad[t] : 0.0f;
  float m = -INFINITY;
  for (int k = rb; k < re; ++k) m = fmaxf(m, lrelu(__fadd_rn(as[(int64_t)col[k] * H + h], adv), slope));
  float ssum = 0.0f;
  for (int k = rb; k < re; ++k)
    ssum = __fadd_rn(ssum, expf(__fsub_rn(lrelu(__fadd_rn(as[(int64_t)col[k] * H + h], adv), slope), m)));
  const float den = __fadd_rn(ssum, 1e-16f);
  for (int k = rb; k < re; ++k) {
    const float e = expf(__fsub_rn(lrelu(__fadd_rn(as[(int64_t)col[k] * H + h], adv), slope), m));
    alpha[(int64_t)k * H + h] = __fdiv_rn(e, den);
  }
  float* o = out + i * ldo + (int64_t)h * C;
  const float* acc = accum ? accum + i * ld_acc + (int64_t)h * C : nullptr;
  const float* bh = bias ? bias + h * C : nullptr;
  for (int c = 0; c < C; ++c) {
    float s = 0.0f;
    for (int k = rb; k < re; ++k)
      s = __fadd_rn(s, __fmul_rn(xs[(int64_t)col[k] * ldxs + (int64_t)h * C + c], alpha[(int64_t)k * H + h]));
    if (bh) s = __fadd_rn(s, bh[c]);
    if (acc) s = __fadd_rn(acc[c], s);
    o[c] = s;
  }
}

// g_pre (per CSR edge and head) and g_a_d; g_x_d = g_a_d att_dst when requested.
__global__ __launch_bounds__(256) void k_gat_bwd_dst(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                     int64_t n_dst, int H, int C, const float* __restrict__ xs,
                                                     int64_t ldxs, const float* __restrict__ g_out, int64_t ldg,
                                                     const float* __restrict__ alpha, const float* __restrict__ as,
                                                     const float* __restrict__ ad, float slope,
                                                     const float* __restrict__ att_dst, float* __restrict__ g_pre,
                                                     float* __restrict__ g_ad, float* __restrict__ g_xd, int64_t ldgxd) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_dst * H) return;
  const int64_t i = t / H;
  const int h = (int)(t % H);
  const int rb = rowptr[i], re = rowptr[i + 1];
  const float* go = g_out + i * ldg + (int64_t)h * C;
  float S = 0.0f;
  for (int k = rb; k < re; ++k) {
    const float* xr = xs + (int64_t)col[k] * ldxs + (int64_t)h * C;
    float ga = 0.0f;
    for (int c = 0; c < C; ++c) ga = __fadd_rn(ga, __fmul_rn(go[c], xr[c]));
    g_pre[(int64_t)k * H + h] = ga;   // g_alpha for now
    S = __fadd_rn(S, __fmul_rn(alpha[(int64_t)k * H + h], ga));
  }
  const float adv = ad ? ad[t] : 0.0f;
  float gsum = 0.0f;
  for (int k = rb; k < re; ++k) {
    const int64_t q = (int64_t)k * H + h;
    const float ge = __fmul_rn(alpha[q], __fsub_rn(g_pre[q], S));
    const float pre = __fadd_rn(as[(int64_t)col[k] * H + h], adv);
    const float gp = pre > 0.0f ? ge : __fmul_rn(ge, slope);
    g_pre[q] = gp;
    gsum = __fadd_rn(gsum, gp);
  }
  if (g_ad) g_ad[t] = gsum;
  if (g_xd) {
    float* gx = g_xd + i * ldgxd + (int64_t)h * C;
    for (int c = 0; c < C; ++c) gx[c] = __fmul_rn(gsum, att_dst[h * C + c]);
  }
}

// CSC walk: cptr / cdst = the relation's CSC (rows = sources, entries = destinations), cpos = the CSR position of
// each CSC entry (where alpha / g_pre of that edge live).
__global__ __launch_bounds__(256) void k_gat_bwd_src(const int32_t* __restrict__ cptr, const int32_t* __restrict__ cdst,
                                                     const int32_t* __restrict__ cpos, int64_t n_src, int H, int C,
                                                     const float* __restrict__ g_out, int64_t ldg,
                                                     const float* __restrict__ alpha, const float* __restrict__ g_pre,
                                                     const float* __restrict__ att_src, float* __restrict__ g_as,
                                                     float* __restrict__ g_xs, int64_t ldgxs) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_src * H) return;
  const int64_t j = t / H;
  const int h = (int)(t % H);
  const int rb = cptr[j], re = cptr[j + 1];
  float gas = 0.0f;
  for (int k = rb; k < re; ++k) gas = __fadd_rn(gas, g_pre[(int64_t)cpos[k] * H + h]);
  g_as[t] = gas;
  float* gx = g_xs + j * ldgxs + (int64_t)h * C;
  for (int c = 0; c < C; ++c) {
    float s = 0.0f;
    for (int k = rb; k < re; ++k)
      s = __fadd_rn(s, __fmul_rn(g_out[(int64_t)cdst[k] * ldg + (int64_t)h * C + c], alpha[(int64_t)cpos[k] * H + h]));
    gx[c] = __fadd_rn(s, __fmul_rn(gas, att_src[h * C + c]));
  }
}

// out[h * C + c] = sum_n w[n, h] x[n, h * C + c] (w NULL: weight 1), n in fixed 256-row blocks, then blocks in order.
constexpr int kWsumRows = 256;
__global__ __launch_bounds__(256) void k_gat_wsum_part(const float* __restrict__ x, int64_t ldx, int64_t n, int H,
                                                       int C, const float* __restrict__ w, float* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kWsumRows;
  const int64_t r1 = r0 + kWsumRows < n ? r0 + kWsumRows : n;
  const int HC = H * C;
  for (int f = threadIdx.x; f < HC; f += 256) {
    const int h = f / C;
    float s = 0.0f;
    for (int64_t r = r0; r < r1; ++r) {
      const float v = x[r * ldx + f];
      s = __fadd_rn(s, w ? __fmul_rn(w[r * H + h], v) : v);
    }
    part[(int64_t)blockIdx.x * HC + f] = s;
  }
}
__global__ __launch_bounds__(256) void k_gat_wsum_final(const float* __restrict__ part, int64_t nb, int HC,
                                                        float* __restrict__ out) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= HC) return;
  float s = 0.0f;
  for (int64_t b = 0; b < nb; ++b) s = __fadd_rn(s, part[b * HC + f]);
  out[f] = s;
}

inline unsigned blocks_for(int64_t n) { return (unsigned)ceil_div(n > 0 ? n : 1, 256); }

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_gat_logits_f32(const float* x, int64_t ldx, int64_t n, int64_t H, int64_t C, const float* att,
                                   float* a, void* stream) {
  HGIN_ARG_CHECK(n >= 0 && H >= 1 && C >= 1 && ldx >= H * C, "hgin_gat_logits_f32: bad sizes");
  if (n == 0) return HGIN_OK;
  HGIN_ARG_CHECK(x && att && a, "hgin_gat_logits_f32: NULL operand");
  HGIN_TRACE("k_gat_logits");
  k_gat_logits<<<blocks_for(n * H), 256, 0, as_stream(stream)>>>(x, ldx, n, (int)H, (int)C, att, a);
  return check_launch("hgin_gat_logits_f32");
}

extern "C" int hgin_gat_fwd_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                                const float* xs, int64_t ldxs, const float* as, const float* ad, float slope,
                                const float* bias, const float* accum, int64_t ld_acc, float* alpha, float* out,
                                int64_t ldo, void* stream) {
  HGIN_ARG_CHECK(n_dst >= 0 && H >= 1 && C >= 1 && ldxs >= H * C && ldo >= H * C && (!accum || ld_acc >= H * C),
                 "hgin_gat_fwd_f32: bad sizes");
  if (n_dst == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr && col && xs && as && alpha && out, "hgin_gat_fwd_f32: NULL operand");
  HGIN_TRACE("k_gat_fwd");
  k_gat_fwd<<<blocks_for(n_dst * H), 256, 0, as_stream(stream)>>>(rowptr, col, n_dst, (int)H, (int)C, xs, ldxs, as, ad,
                                                                  slope, bias, accum, ld_acc, alpha, out, ldo);
  return check_launch("hgin_gat_fwd_f32");
}

extern "C" int hgin_gat_bwd_dst_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                                    const float* xs, int64_t ldxs, const float* g_out, int64_t ldg, const float* alpha,
                                    const float* as, const float* ad, float slope, const float* att_dst, float* g_pre,
                                    float* g_ad, float* g_xd, int64_t ldgxd, void* stream) {
  HGIN_ARG_CHECK(n_dst >= 0 && H >= 1 && C >= 1 && ldxs >= H * C && ldg >= H * C && (!g_xd || ldgxd >= H * C),
                 "hgin_gat_bwd_dst_f32: bad sizes");
  if (n_dst == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr && col && xs && g_out && alpha && as && g_pre && (!g_xd || (att_dst && ad)),
                 "hgin_gat_bwd_dst_f32: NULL operand");
  HGIN_TRACE("k_gat_bwd_dst");
  k_gat_bwd_dst<<<blocks_for(n_dst * H), 256, 0, as_stream(stream)>>>(rowptr, col, n_dst, (int)H, (int)C, xs, ldxs,
                                                                      g_out, ldg, alpha, as, ad, slope, att_dst, g_pre,
                                                                      g_ad, g_xd, ldgxd);
  return check_launch("hgin_gat_bwd_dst_f32");
}

extern "C" int hgin_gat_bwd_src_f32(const int32_t* cptr, const int32_t* cdst, const int32_t* cpos, int64_t n_src,
                                    int64_t H, int64_t C, const float* g_out, int64_t ldg, const float* alpha,
                                    const float* g_pre, const float* att_src, float* g_as, float* g_xs, int64_t ldgxs,
                                    void* stream) {
  HGIN_ARG_CHECK(n_src >= 0 && H >= 1 && C >= 1 && ldg >= H * C && ldgxs >= H * C, "hgin_gat_bwd_src_f32: bad sizes");
  if (n_src == 0) return HGIN_OK;
  HGIN_ARG_CHECK(cptr && cdst && cpos && g_out && alpha && g_pre && att_src && g_as && g_xs,
                 "hgin_gat_bwd_src_f32: NULL operand");
  HGIN_TRACE("k_gat_bwd_src");
  k_gat_bwd_src<<<blocks_for(n_src * H), 256, 0, as_stream(stream)>>>(cptr, cdst, cpos, n_src, (int)H, (int)C, g_out,
                                                                      ldg, alpha, g_pre, att_src, g_as, g_xs, ldgxs);
  return check_launch("hgin_gat_bwd_src_f32");
}

extern "C" int hgin_gat_wsum_workspace_size(int64_t n, int64_t H, int64_t C, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && n >= 0 && H >= 1 && C >= 1, "hgin_gat_wsum_workspace_size: bad args");
  *bytes = sizeof(float) * (size_t)ceil_div(n > 0 ? n : 1, kWsumRows) * (size_t)(H * C);
  return HGIN_OK;
}

extern "C" int hgin_gat_wsum_f32(const float* x, int64_t ldx, int64_t n, int64_t H, int64_t C, const float* w,
                                 float* out, void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(n >= 0 && H >= 1 && C >= 1 && ldx >= H * C && out, "hgin_gat_wsum_f32: bad args");
  hipStream_t s = as_stream(stream);
  if (n == 0) return memset_async(out, 0, sizeof(float) * (size_t)(H * C), s, "hgin_gat_wsum_f32");
  const int64_t nb = ceil_div(n, kWsumRows);
  const size_t need = sizeof(float) * (size_t)nb * (size_t)(H * C);
  if (!workspace || workspace_bytes < need) {
    set_error("hgin_gat_wsum_f32: workspace %zu < %zu", workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  HGIN_ARG_CHECK(x, "hgin_gat_wsum_f32: NULL x");
  float* part = static_cast<float*>(workspace);
  HGIN_TRACE("k_gat_wsum");
  k_gat_wsum_part<<<(unsigned)nb, 256, 0, s>>>(x, ldx, n, (int)H, (int)C, w, part);
  k_gat_wsum_final<<<blocks_for(H * C), 256, 0, s>>>(part, nb, (int)(H * C), out);
  return check_launch("hgin_gat_wsum_f32");
}

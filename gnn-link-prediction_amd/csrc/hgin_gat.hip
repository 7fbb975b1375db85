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
// the reference's scatter_add; column sums by fixed row blocks, then blocks in order); no atomics.  Two forms: a
// G-lane group per row with lanes across the H * C columns (the default, below: coalesced 16-B row reads, several
// rows in flight, online softmax statistics), and one thread per (row, head) for the shapes it does not take
// (C not a multiple of 4 with C / 4 a power of two, H * C > 256, unaligned rows; HGIN_GAT_WAVE = 0 forces it).
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

// out[h * C + c] = sum_n w[n, h] x[n, h * C + c] (w NULL: weight 1): per 256-row block a partial per column
// (k_gat_wsum_part, a thread per column walking the block's rows in order), stored column-major [HC][nb]; then one
// workgroup per column adds its nb partials — thread t the blocks t, t + 256, ... in order (coalesced), then a fixed
// tree (k_gat_wsum_final).  Round 4's final pass had one thread per column walk all nb partials (5.4 ms per call at
// 6M rows).
constexpr int kWsumRows = 256;
inline int64_t wsum_blocks(int64_t n) { return ceil_div(n > 0 ? n : 1, (int64_t)kWsumRows); }
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
    part[(int64_t)f * gridDim.x + blockIdx.x] = s;
  }
}
__global__ __launch_bounds__(256) void k_gat_wsum_final(const float* __restrict__ part, int64_t nb,
                                                        float* __restrict__ out) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  const float* p = part + (int64_t)blockIdx.x * nb;
  float s = 0.0f;
  for (int64_t b = t; b < nb; b += 256) s = __fadd_rn(s, p[b]);
  red[t] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
    __syncthreads();
  }
  if (t == 0) out[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------------------------------------------
// Wave-group forms (round 5; the default wherever C % 4 == 0, C / 4 a power of two, H * C <= 256, 16-B aligned rows):
// a G-lane group per row, G = the next power of two >= H * C / 4 (G = 32 for the reference's HEADS 16 x C 8: two rows
// per wave), lane gl owning the float4 of columns 4 gl .. 4 gl + 3 (head hq = 4 gl / C), so every gathered x_s / g_out
// row is one contiguous G x 16-B read and up to kGatU rows are in flight per group; the per-head work runs on the
// group's lanes as (edge slot, head) pairs or on each head's first column lane.  No LDS, no atomics; every sum in a
// fixed order (per-column sums over a row's edges in CSR / CSC order, as the thread-per-(row, head) kernels).
constexpr int kGatU = 8;
constexpr int kGatElds = 32;   // k_gat_attn_w: edges per row whose logits wait in LDS for the alpha pass

template <int G>
__device__ __forceinline__ float group_sum_pow2(float v, int width) {   // xor butterfly over `width` aligned lanes
  for (int off = 1; off < width; off <<= 1) v = __fadd_rn(v, __shfl_xor(v, off, G));
  return v;
}

// a[n, h] = sum_c x[n, h C + c] att[h C + c]: each lane its 4 columns in order, then the head's C / 4 lanes.
template <int G>
__global__ __launch_bounds__(256) void k_gat_logits_w(const float* __restrict__ x, int64_t ldx, int64_t n, int H,
                                                      int C, const float* __restrict__ att, float* __restrict__ a) {
  const int gl = threadIdx.x % G;
  const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (r >= n) return;
  const int HC4 = H * C / 4;
  float s = 0.0f;
  if (gl < HC4) {
    const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + 4 * gl);
    const float4 w = *reinterpret_cast<const float4*>(att + 4 * gl);
    s = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(v.x, w.x), __fmul_rn(v.y, w.y)), __fmul_rn(v.z, w.z)),
                  __fmul_rn(v.w, w.w));
  }
  s = group_sum_pow2<G>(s, C / 4);
  if (gl < HC4 && (4 * gl) % C == 0) a[r * H + (4 * gl) / C] = s;
}

// Forward.  The row's first G edge sources come in one coalesced load (lane gl: col[rb + gl]) and reach the other
// lanes by ds_bpermute, and the x_s rows of its first kGatU edges are requested before any softmax arithmetic, so a
// row of up to G edges costs two dependent memory round trips instead of one per phase and batch.  Phase 1 on
// (slot, head) lanes (ES = G / H slots): the online max / exp-sum of the head's logits over the slot's edges (rb + slot,
// + ES, ...), merged over the slots in slot order -> m_h, den_h = sum + 1e-16; the logits of the first ES * kGatU
// edges stay in registers.  Phase 2 on column lanes, in CSR order: alpha = exp(e - m_h) / den_h with e taken from the
// phase-1 lane that holds it (stored by the head's first lane: the backward's alpha) and out += x_s[j] * alpha; then
// + bias, accum + (the thread-per-(row, head) kernel's order).
template <int G>
__global__ __launch_bounds__(256) void k_gat_fwd_w(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                   int64_t n_dst, int H, int C, const float* __restrict__ xs,
                                                   int64_t ldxs, const float* __restrict__ as,
                                                   const float* __restrict__ ad, float slope,
                                                   const float* __restrict__ bias, const float* __restrict__ accum,
                                                   int64_t ld_acc, float* __restrict__ alpha, float* __restrict__ out,
                                                   int64_t ldo) {
  constexpr int U = kGatU;
  const int gl = threadIdx.x % G;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (i >= n_dst) return;
  const int rb = rowptr[i], re = rowptr[i + 1];
  const int deg = re - rb;
  const int cj = gl < deg ? col[rb + gl] : 0;                    // the sources of edges 0 .. G - 1
  // source of edge k (< deg) of the row; every lane of the group runs the shuffle (k may differ per lane)
  auto src = [&](int k) -> int64_t {
    const int sh = __shfl(cj, k & (G - 1), G);
    return k < G ? (int64_t)sh : (int64_t)col[rb + k];
  };
  const int HC4 = H * C / 4;
  const bool col_lane = gl < HC4;
  // the first U edges' x_s rows, in flight during phase 1
  float4 xv0[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t j = src(u < deg ? u : 0);
    xv0[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col_lane && u < deg) xv0[u] = *reinterpret_cast<const float4*>(xs + j * ldxs + 4 * gl);
  }
  const int ES = G / H;
  const int slot = gl / H, h1 = gl % H;
  const bool ph1 = slot < ES;
  const float adv = ph1 && ad ? ad[i * H + h1] : 0.0f;
  float m = -INFINITY, s = 0.0f;
  auto online = [&](float e) {
    if (e > m) {
      s = __fadd_rn(__fmul_rn(s, expf(__fsub_rn(m, e))), 1.0f);
      m = e;
    } else {
      s = __fadd_rn(s, expf(__fsub_rn(e, m)));
    }
  };
  float e0[U];   // logits of this lane's edges slot + ES t, t < U (phase-1 lanes)
  {
    float av[U];
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const int k = slot + ES * t;
      const int64_t j = src(k < deg ? k : 0);
      av[t] = ph1 && k < deg ? as[j * H + h1] : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < U; ++t) {
      e0[t] = lrelu(__fadd_rn(av[t], adv), slope);
      if (ph1 && slot + ES * t < deg) online(e0[t]);
    }
  }
  if (ph1) {   // rows longer than ES * U: the rest of the slot's edges
    for (int k0 = rb + slot + ES * U; k0 < re; k0 += ES * U) {
      float av[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * ES;
        av[u] = k < re ? as[(int64_t)col[k] * H + h1] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k0 + u * ES < re) online(lrelu(__fadd_rn(av[u], adv), slope));
    }
  }
  for (int q = 1; q < ES; ++q) {   // slot 0 merges slots 1 .. ES - 1 in order (every lane runs the shuffles)
    const float m2 = __shfl(m, gl + q * H < G ? gl + q * H : gl, G);
    const float s2 = __shfl(s, gl + q * H < G ? gl + q * H : gl, G);
    if (slot == 0 && m2 != -INFINITY) {
      if (m == -INFINITY) {
        m = m2;
        s = s2;
      } else {
        const float M = fmaxf(m, m2);
        s = __fadd_rn(__fmul_rn(s, expf(__fsub_rn(m, M))), __fmul_rn(s2, expf(__fsub_rn(m2, M))));
        m = M;
      }
    }
  }
  const float den = __fadd_rn(s, 1e-16f);
  const int hq = col_lane ? (4 * gl) / C : 0;
  const float mh = __shfl(m, hq, G), dh = __shfl(den, hq, G);
  const bool first = col_lane && (4 * gl) % C == 0;
  const float adq = ad ? ad[i * H + hq] : 0.0f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](int k, float e, const float4& x) {   // edge k of the row, its logit, its x_s quad
    const float al = __fdiv_rn(expf(__fsub_rn(e, mh)), dh);
    if (first) __builtin_nontemporal_store(al, alpha + (int64_t)(rb + k) * H + hq);   // streamed once
    acc.x = __fadd_rn(acc.x, __fmul_rn(x.x, al));
    acc.y = __fadd_rn(acc.y, __fmul_rn(x.y, al));
    acc.z = __fadd_rn(acc.z, __fmul_rn(x.z, al));
    acc.w = __fadd_rn(acc.w, __fmul_rn(x.w, al));
  };
  // the logit of edge k < ES U: e0[k / ES] of lane (k % ES) H + hq (ES is a runtime value: the register is picked by
  // selects, not by a dynamic index); every lane runs the shuffle
  auto logit = [&](int k) {
    const int t = k / ES;
    float r = 0.0f;
#pragma unroll
    for (int tt = 0; tt < U; ++tt) r = tt == t ? e0[tt] : r;
    return __shfl(r, (k % ES) * H + hq, G);
  };
  // edges 0 .. U - 1: rows and logits already here
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float e = logit(u);
    if (col_lane && u < deg) add(u, e, xv0[u]);
  }
  for (int k0 = U; k0 < deg; k0 += U) {   // the rest, U rows in flight
    float4 xv[U];
    float ev[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      // logits of edges below ES U come from phase 1's registers; beyond, reloaded
      ev[u] = logit(k < ES * U ? k : 0);
      const int64_t j = src(k < deg ? k : 0);
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (col_lane && k < deg) {
        xv[u] = *reinterpret_cast<const float4*>(xs + j * ldxs + 4 * gl);
        if (k >= ES * U) ev[u] = lrelu(__fadd_rn(as[j * H + hq], adq), slope);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (col_lane && k0 + u < deg) add(k0 + u, ev[u], xv[u]);
  }
  if (!col_lane) return;
  if (bias) {
    const float4 b = *reinterpret_cast<const float4*>(bias + 4 * gl);
    acc = make_float4(__fadd_rn(acc.x, b.x), __fadd_rn(acc.y, b.y), __fadd_rn(acc.z, b.z), __fadd_rn(acc.w, b.w));
  }
  if (accum) {
    const float4 c = *reinterpret_cast<const float4*>(accum + i * ld_acc + 4 * gl);
    acc = make_float4(__fadd_rn(c.x, acc.x), __fadd_rn(c.y, acc.y), __fadd_rn(c.z, acc.z), __fadd_rn(c.w, acc.w));
  }
  *reinterpret_cast<float4*>(out + i * ldo + 4 * gl) = acc;
}

// Forward in one pass over the row's edges (hgin_gat_attn_fwd_f32, the default of hgin/gat.py; round 5): the source
// logit a_s[j, h] = x_s[j, h, :] . att_src[h, :] is formed from the x_s row the aggregate gathers anyway (each lane its
// 4 products in order, then the head's C / 4 lanes: k_gat_logits_w's arithmetic, bit for bit), so no a_s table is
// gathered; per edge in CSR order the online softmax keeps (m, s) and the exp-weighted row sum with the rescale
// exp(m_old - m_new) when the maximum moves, out = acc / (s + 1e-16) (+ bias, accum +); the edge logits go into the
// alpha slots on the way and become alpha = exp(e - m) / den in a second, L2-resident pass of the head's first lane over
// its own stores.  Differs from the two-pass form only in rounding (the weighted sum is divided once at the end).
template <int G, int U = kGatU>
__global__ __launch_bounds__(256) void k_gat_attn_w(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                    int64_t n_dst, int H, int C, const float* __restrict__ xs,
                                                    int64_t ldxs, const float* __restrict__ att_src,
                                                    const float* __restrict__ ad, float slope,
                                                    const float* __restrict__ bias, const float* __restrict__ accum,
                                                    int64_t ld_acc, float* __restrict__ alpha, float* __restrict__ out,
                                                    int64_t ldo) {
  extern __shared__ float gat_elds[];   // per row of the block: the logits of its first kGatElds edges, [edge][head]
  const int gl = threadIdx.x % G;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (i >= n_dst) return;
  float* const el = gat_elds + (threadIdx.x / G) * kGatElds * H;
  const int rb = rowptr[i], re = rowptr[i + 1];
  const int deg = re - rb;
  const int cj = gl < deg ? col[rb + gl] : 0;                    // the sources of edges 0 .. G - 1
  const int HC4 = H * C / 4;
  const bool col_lane = gl < HC4;
  const int hq = col_lane ? (4 * gl) / C : 0;
  const bool first = col_lane && (4 * gl) % C == 0;
  const float4 at = col_lane ? *reinterpret_cast<const float4*>(att_src + 4 * gl) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float adq = col_lane && ad ? ad[i * H + hq] : 0.0f;
  float m = -INFINITY, s = 0.0f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k0 = 0; k0 < deg; k0 += U) {
    float4 xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u < deg ? k0 + u : 0;
      const int sh = __shfl(cj, k & (G - 1), G);                 // every lane runs the shuffle
      const int64_t j = k < G ? (int64_t)sh : (int64_t)col[rb + k];
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (col_lane && k0 + u < deg) xv[u] = *reinterpret_cast<const float4*>(xs + j * ldxs + 4 * gl);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + u < deg) {   // uniform over the group
        float p = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(xv[u].x, at.x), __fmul_rn(xv[u].y, at.y)),
                                      __fmul_rn(xv[u].z, at.z)), __fmul_rn(xv[u].w, at.w));
        p = group_sum_pow2<G>(p, C / 4);                         // a_s[j, hq]
        const float e = lrelu(__fadd_rn(p, adq), slope);
        if (first) {   // the logit, until the alpha pass: in LDS for the first kGatElds edges, else in alpha
          if (k0 + u < kGatElds) el[(k0 + u) * H + hq] = e;
          else alpha[(int64_t)(rb + k0 + u) * H + hq] = e;
        }
        if (e > m) {
          const float sc = expf(__fsub_rn(m, e));
          s = __fadd_rn(__fmul_rn(s, sc), 1.0f);
          acc = make_float4(__fadd_rn(__fmul_rn(acc.x, sc), xv[u].x), __fadd_rn(__fmul_rn(acc.y, sc), xv[u].y),
                            __fadd_rn(__fmul_rn(acc.z, sc), xv[u].z), __fadd_rn(__fmul_rn(acc.w, sc), xv[u].w));
          m = e;
        } else {
          const float w = expf(__fsub_rn(e, m));
          s = __fadd_rn(s, w);
          acc = make_float4(__fadd_rn(acc.x, __fmul_rn(w, xv[u].x)), __fadd_rn(acc.y, __fmul_rn(w, xv[u].y)),
                            __fadd_rn(acc.z, __fmul_rn(w, xv[u].z)), __fadd_rn(acc.w, __fmul_rn(w, xv[u].w)));
        }
      }
    }
  }
  if (!col_lane) return;
  const float den = __fadd_rn(s, 1e-16f);
  if (first) {   // the logits stored above -> alpha (this lane's own stores, read back in order)
    const int kl = deg < kGatElds ? deg : kGatElds;
    for (int k = 0; k < kl; ++k)
      __builtin_nontemporal_store(__fdiv_rn(expf(__fsub_rn(el[k * H + hq], m)), den), alpha + (int64_t)(rb + k) * H + hq);
    for (int k0 = rb + kGatElds; k0 < re; k0 += U) {
      float ev[U];
#pragma unroll
      for (int u = 0; u < U; ++u) ev[u] = k0 + u < re ? alpha[(int64_t)(k0 + u) * H + hq] : 0.0f;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k0 + u < re)
          __builtin_nontemporal_store(__fdiv_rn(expf(__fsub_rn(ev[u], m)), den), alpha + (int64_t)(k0 + u) * H + hq);
    }
  }
  acc = make_float4(__fdiv_rn(acc.x, den), __fdiv_rn(acc.y, den), __fdiv_rn(acc.z, den), __fdiv_rn(acc.w, den));
  if (bias) {
    const float4 b = *reinterpret_cast<const float4*>(bias + 4 * gl);
    acc = make_float4(__fadd_rn(acc.x, b.x), __fadd_rn(acc.y, b.y), __fadd_rn(acc.z, b.z), __fadd_rn(acc.w, b.w));
  }
  if (accum) {
    const float4 c = *reinterpret_cast<const float4*>(accum + i * ld_acc + 4 * gl);
    acc = make_float4(__fadd_rn(c.x, acc.x), __fadd_rn(c.y, acc.y), __fadd_rn(c.z, acc.z), __fadd_rn(c.w, acc.w));
  }
  *reinterpret_cast<float4*>(out + i * ldo + 4 * gl) = acc;
}

// Backward, destination side.  Phase A (column lanes, CSR order, U rows in flight): g_alpha_k = <g_out[i, h, :],
// x_s[j_k, h, :]> (each lane its 4 products, then the head's C / 4 lanes), S_h = sum_k alpha_k g_alpha_k; the head's
// first lane stores g_alpha_k.  Phase B (the head's first lane, CSR order): g_pre_k = leaky'(pre_k) alpha_k
// (g_alpha_k - S_h) over its own stores, g_a_d = sum_k g_pre_k; g_x_d = g_a_d att_dst on the column lanes.  The row's
// first G edge sources come in one coalesced load and reach the lanes by ds_bpermute (k_gat_attn_w's scheme), so a
// batch of U edges costs one dependent round trip (both phases run their loops on every lane of the group: the
// shuffles need them).
template <int G, int U>
__global__ __launch_bounds__(256) void k_gat_bwd_dst_w(const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col, int64_t n_dst, int H, int C,
                                                       const float* __restrict__ xs, int64_t ldxs,
                                                       const float* __restrict__ g_out, int64_t ldg,
                                                       const float* __restrict__ alpha, const float* __restrict__ as,
                                                       const float* __restrict__ ad, float slope,
                                                       const float* __restrict__ att_dst, float* __restrict__ g_pre,
                                                       float* __restrict__ g_ad, float* __restrict__ g_xd,
                                                       int64_t ldgxd) {
  const int gl = threadIdx.x % G;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (i >= n_dst) return;
  const int rb = rowptr[i], re = rowptr[i + 1];
  const int deg = re - rb;
  const int cj = gl < deg ? col[rb + gl] : 0;   // the sources of edges 0 .. G - 1
  auto src = [&](int k) -> int64_t {           // (every lane of the group runs the shuffle)
    const int sh = __shfl(cj, k & (G - 1), G);
    return k < G ? (int64_t)sh : (int64_t)col[rb + k];
  };
  const int HC4 = H * C / 4;
  const bool lane_on = gl < HC4;
  const int hq = lane_on ? (4 * gl) / C : 0;
  const bool first = lane_on && (4 * gl) % C == 0;
  const float4 go = lane_on ? *reinterpret_cast<const float4*>(g_out + i * ldg + 4 * gl) : make_float4(0.f, 0.f, 0.f, 0.f);
  float S = 0.0f;
  for (int k0 = 0; k0 < deg; k0 += U) {
    float av[U];
    float4 xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = src(k0 + u < deg ? k0 + u : 0);
      av[u] = 0.0f;
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (lane_on && k0 + u < deg) {
        av[u] = alpha[(int64_t)(rb + k0 + u) * H + hq];
        xv[u] = *reinterpret_cast<const float4*>(xs + j * ldxs + 4 * gl);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + u < deg) {   // (uniform over the group: the shuffles below run on every lane)
        float p = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(go.x, xv[u].x), __fmul_rn(go.y, xv[u].y)),
                                      __fmul_rn(go.z, xv[u].z)), __fmul_rn(go.w, xv[u].w));
        p = group_sum_pow2<G>(p, C / 4);
        S = __fadd_rn(S, __fmul_rn(av[u], p));
        if (first) g_pre[(int64_t)(rb + k0 + u) * H + hq] = p;   // g_alpha for now
      }
    }
  }
  float gsum = 0.0f;
  const float adv = first && ad ? ad[i * H + hq] : 0.0f;
  for (int k0 = 0; k0 < deg; k0 += U) {   // U edges' operands loaded together
    float al[U], ga[U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = src(k0 + u < deg ? k0 + u : 0);
      al[u] = ga[u] = av[u] = 0.0f;
      if (first && k0 + u < deg) {
        const int64_t q = (int64_t)(rb + k0 + u) * H + hq;
        al[u] = alpha[q];
        ga[u] = g_pre[q];
        av[u] = as[j * H + hq];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (first && k0 + u < deg) {
        const float ge = __fmul_rn(al[u], __fsub_rn(ga[u], S));
        const float pre = __fadd_rn(av[u], adv);
        const float gp = pre > 0.0f ? ge : __fmul_rn(ge, slope);
        g_pre[(int64_t)(rb + k0 + u) * H + hq] = gp;
        gsum = __fadd_rn(gsum, gp);
      }
    }
  }
  if (first && g_ad) g_ad[i * H + hq] = gsum;
  if (g_xd) {
    const int srcl = lane_on ? hq * (C / 4) : gl;
    gsum = __shfl(gsum, srcl, G);
    if (lane_on) {
      const float4 at = *reinterpret_cast<const float4*>(att_dst + 4 * gl);
      *reinterpret_cast<float4*>(g_xd + i * ldgxd + 4 * gl) =
          make_float4(__fmul_rn(gsum, at.x), __fmul_rn(gsum, at.y), __fmul_rn(gsum, at.z), __fmul_rn(gsum, at.w));
    }
  }
}

// Backward, source side, on the CSC (entries k: destination cdst[k], CSR position cpos[k]), in CSC order:
// g_a_s[j, h] = sum_k g_pre (the head's first lane), g_x_s[j, cols] = sum_k alpha g_out[i_k, cols] + g_a_s att_src.
// The row's first G CSC entries (destination, position) come in one coalesced load each, as in k_gat_bwd_dst_w.
template <int G, int U>
__global__ __launch_bounds__(256) void k_gat_bwd_src_w(const int32_t* __restrict__ cptr, const int32_t* __restrict__ cdst,
                                                       const int32_t* __restrict__ cpos, int64_t n_src, int H, int C,
                                                       const float* __restrict__ g_out, int64_t ldg,
                                                       const float* __restrict__ alpha,
                                                       const float* __restrict__ g_pre,
                                                       const float* __restrict__ att_src, float* __restrict__ g_as,
                                                       float* __restrict__ g_xs, int64_t ldgxs) {
  const int gl = threadIdx.x % G;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (j >= n_src) return;
  const int HC4 = H * C / 4;
  const bool lane_on = gl < HC4;
  const int hq = lane_on ? (4 * gl) / C : 0;
  const bool first = lane_on && (4 * gl) % C == 0;
  const int rb = cptr[j], re = cptr[j + 1];
  const int deg = re - rb;
  const int cd = gl < deg ? cdst[rb + gl] : 0, cp = gl < deg ? cpos[rb + gl] : 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float gas = 0.0f;
  for (int k0 = 0; k0 < deg; k0 += U) {
    float av[U], pv[U];
    float4 gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u < deg ? k0 + u : 0;
      const int sd = __shfl(cd, k & (G - 1), G), sp = __shfl(cp, k & (G - 1), G);   // (every lane)
      const int64_t d = k < G ? sd : cdst[rb + k];
      const int64_t p = (int64_t)(k < G ? sp : cpos[rb + k]) * H + hq;
      av[u] = pv[u] = 0.0f;
      gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (lane_on && k0 + u < deg) {
        av[u] = alpha[p];
        if (first) pv[u] = g_pre[p];
        gv[u] = *reinterpret_cast<const float4*>(g_out + d * ldg + 4 * gl);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (lane_on && k0 + u < deg) {
        gas = __fadd_rn(gas, pv[u]);
        acc.x = __fadd_rn(acc.x, __fmul_rn(gv[u].x, av[u]));
        acc.y = __fadd_rn(acc.y, __fmul_rn(gv[u].y, av[u]));
        acc.z = __fadd_rn(acc.z, __fmul_rn(gv[u].z, av[u]));
        acc.w = __fadd_rn(acc.w, __fmul_rn(gv[u].w, av[u]));
      }
    }
  }
  if (first) g_as[j * H + hq] = gas;
  gas = __shfl(gas, lane_on ? hq * (C / 4) : gl, G);
  if (lane_on) {
    const float4 at = *reinterpret_cast<const float4*>(att_src + 4 * gl);
    *reinterpret_cast<float4*>(g_xs + j * ldgxs + 4 * gl) =
        make_float4(__fadd_rn(acc.x, __fmul_rn(gas, at.x)), __fadd_rn(acc.y, __fmul_rn(gas, at.y)),
                    __fadd_rn(acc.z, __fmul_rn(gas, at.z)), __fadd_rn(acc.w, __fmul_rn(gas, at.w)));
  }
}

// The wave-group form applies: C a multiple of 4 with C / 4 a power of two, H * C <= 256, 16-B aligned rows.
int gat_group(int64_t H, int64_t C) {
  static const bool off = [] {
    const char* v = getenv("HGIN_GAT_WAVE");
    return v && v[0] == '0';
  }();
  if (off || C % 4 || ((C / 4) & (C / 4 - 1)) || H * C > 256) return 0;
  int g = 1;
  while (g < H * C / 4) g <<= 1;
  return g < (int)H ? 0 : g;
}

inline bool al16(const void* p, int64_t ld) { return p == nullptr || (aligned16(p) && ld % 4 == 0); }

// the backward kernels take U edges in flight per group: 4 (8 measured 2 % slower over fwd + bwd at a 30M-edge
// relation, profiles/r05/gat_bwd/)
#define HGIN_GAT_GU(G, U, KERN, ...)                                                                            \
  switch (G) {                                                                                                \
    case 1: KERN<1, U><<<(unsigned)ceil_div(rows, 256 / 1), 256, 0, s>>>(__VA_ARGS__); break;                  \
    case 2: KERN<2, U><<<(unsigned)ceil_div(rows, 256 / 2), 256, 0, s>>>(__VA_ARGS__); break;                  \
    case 4: KERN<4, U><<<(unsigned)ceil_div(rows, 256 / 4), 256, 0, s>>>(__VA_ARGS__); break;                  \
    case 8: KERN<8, U><<<(unsigned)ceil_div(rows, 256 / 8), 256, 0, s>>>(__VA_ARGS__); break;                  \
    case 16: KERN<16, U><<<(unsigned)ceil_div(rows, 256 / 16), 256, 0, s>>>(__VA_ARGS__); break;               \
    case 32: KERN<32, U><<<(unsigned)ceil_div(rows, 256 / 32), 256, 0, s>>>(__VA_ARGS__); break;               \
    default: KERN<64, U><<<(unsigned)ceil_div(rows, 256 / 64), 256, 0, s>>>(__VA_ARGS__); break;               \
  }
#define HGIN_GAT_G(G, KERN, ...)                                                                                \
  switch (G) {                                                                                                \
    case 1: KERN<1><<<(unsigned)ceil_div(rows, 256 / 1), 256, 0, s>>>(__VA_ARGS__); break;                     \
    case 2: KERN<2><<<(unsigned)ceil_div(rows, 256 / 2), 256, 0, s>>>(__VA_ARGS__); break;                     \
    case 4: KERN<4><<<(unsigned)ceil_div(rows, 256 / 4), 256, 0, s>>>(__VA_ARGS__); break;                     \
    case 8: KERN<8><<<(unsigned)ceil_div(rows, 256 / 8), 256, 0, s>>>(__VA_ARGS__); break;                     \
    case 16: KERN<16><<<(unsigned)ceil_div(rows, 256 / 16), 256, 0, s>>>(__VA_ARGS__); break;                  \
    case 32: KERN<32><<<(unsigned)ceil_div(rows, 256 / 32), 256, 0, s>>>(__VA_ARGS__); break;                  \
    default: KERN<64><<<(unsigned)ceil_div(rows, 256 / 64), 256, 0, s>>>(__VA_ARGS__); break;                  \
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
  if (const int G = gat_group(H, C); G && al16(x, ldx) && aligned16(att)) {
    HGIN_TRACE("k_gat_logits_w<%d>", G);
    const int64_t rows = n;
    hipStream_t s = as_stream(stream);
    HGIN_GAT_G(G, k_gat_logits_w, x, ldx, n, (int)H, (int)C, att, a)
    return check_launch("hgin_gat_logits_f32");
  }
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
  if (const int G = gat_group(H, C);
      G && al16(xs, ldxs) && al16(out, ldo) && al16(accum, ld_acc) && (!bias || aligned16(bias))) {
    HGIN_TRACE("k_gat_fwd_w<%d>", G);
    const int64_t rows = n_dst;
    hipStream_t s = as_stream(stream);
    HGIN_GAT_G(G, k_gat_fwd_w, rowptr, col, n_dst, (int)H, (int)C, xs, ldxs, as, ad, slope, bias, accum, ld_acc, alpha,
               out, ldo)
    return check_launch("hgin_gat_fwd_f32");
  }
  HGIN_TRACE("k_gat_fwd");
  k_gat_fwd<<<blocks_for(n_dst * H), 256, 0, as_stream(stream)>>>(rowptr, col, n_dst, (int)H, (int)C, xs, ldxs, as, ad,
                                                                  slope, bias, accum, ld_acc, alpha, out, ldo);
  return check_launch("hgin_gat_fwd_f32");
}

extern "C" int hgin_gat_attn_fwd_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                                     const float* xs, int64_t ldxs, const float* att_src, const float* ad, float slope,
                                     const float* bias, const float* accum, int64_t ld_acc, float* alpha, float* out,
                                     int64_t ldo, void* stream) {
  HGIN_ARG_CHECK(n_dst >= 0 && H >= 1 && C >= 1 && ldxs >= H * C && ldo >= H * C && (!accum || ld_acc >= H * C),
                 "hgin_gat_attn_fwd_f32: bad sizes");
  if (n_dst == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr && col && xs && att_src && alpha && out, "hgin_gat_attn_fwd_f32: NULL operand");
  const int G = gat_group(H, C);
  if (!(G && al16(xs, ldxs) && al16(out, ldo) && al16(accum, ld_acc) && (!bias || aligned16(bias)) &&
        aligned16(att_src))) {
    set_error("hgin_gat_attn_fwd_f32: needs the wave-group shape (C a multiple of 4 with C / 4 a power of two, "
              "H * C <= 256, 16-B aligned rows); use hgin_gat_logits_f32 + hgin_gat_fwd_f32");
    return HGIN_E_ARG;
  }
  HGIN_TRACE("k_gat_attn_w<%d>", G);
  const int64_t rows = n_dst;
  hipStream_t s = as_stream(stream);
  // 4 rows of x_s in flight per group: 52 VGPRs, 8 waves per SIMD (8 rows: 68 VGPRs, 7 waves, 2.3 % slower; 16 rows:
  // 4 waves, 42 % slower — profiles/r05/gat_u_ab.txt)
  const size_t lds = sizeof(float) * (size_t)(256 / G) * kGatElds * (size_t)H;
#define HGIN_GAT_ATTN(GV)                                                                                          \
  case GV:                                                                                                        \
    k_gat_attn_w<GV, 4><<<(unsigned)ceil_div(rows, (int64_t)(256 / GV)), 256, lds, s>>>(                          \
        rowptr, col, n_dst, (int)H, (int)C, xs, ldxs, att_src, ad, slope, bias, accum, ld_acc, alpha, out, ldo);   \
    break;
  switch (G) {
    HGIN_GAT_ATTN(1) HGIN_GAT_ATTN(2) HGIN_GAT_ATTN(4) HGIN_GAT_ATTN(8) HGIN_GAT_ATTN(16) HGIN_GAT_ATTN(32)
    default: HGIN_GAT_ATTN(64)
  }
#undef HGIN_GAT_ATTN
  return check_launch("hgin_gat_attn_fwd_f32");
}

extern "C" int hgin_gat_attn_supported(int64_t H, int64_t C) { return gat_group(H, C) != 0; }

extern "C" int hgin_gat_bwd_dst_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                                    const float* xs, int64_t ldxs, const float* g_out, int64_t ldg, const float* alpha,
                                    const float* as, const float* ad, float slope, const float* att_dst, float* g_pre,
                                    float* g_ad, float* g_xd, int64_t ldgxd, void* stream) {
  HGIN_ARG_CHECK(n_dst >= 0 && H >= 1 && C >= 1 && ldxs >= H * C && ldg >= H * C && (!g_xd || ldgxd >= H * C),
                 "hgin_gat_bwd_dst_f32: bad sizes");
  if (n_dst == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr && col && xs && g_out && alpha && as && g_pre && (!g_xd || (att_dst && ad)),
                 "hgin_gat_bwd_dst_f32: NULL operand");
  if (const int G = gat_group(H, C);
      G && al16(xs, ldxs) && al16(g_out, ldg) && al16(g_xd, ldgxd) && (!g_xd || aligned16(att_dst))) {
    HGIN_TRACE("k_gat_bwd_dst_w<%d>", G);
    const int64_t rows = n_dst;
    hipStream_t s = as_stream(stream);
    HGIN_GAT_GU(G, 4, k_gat_bwd_dst_w, rowptr, col, n_dst, (int)H, (int)C, xs, ldxs, g_out, ldg, alpha, as, ad,
                  slope, att_dst, g_pre, g_ad, g_xd, ldgxd)
    return check_launch("hgin_gat_bwd_dst_f32");
  }
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
  if (const int G = gat_group(H, C); G && al16(g_out, ldg) && al16(g_xs, ldgxs) && aligned16(att_src)) {
    HGIN_TRACE("k_gat_bwd_src_w<%d>", G);
    const int64_t rows = n_src;
    hipStream_t s = as_stream(stream);
    HGIN_GAT_GU(G, 4, k_gat_bwd_src_w, cptr, cdst, cpos, n_src, (int)H, (int)C, g_out, ldg, alpha, g_pre, att_src,
                  g_as, g_xs, ldgxs)
    return check_launch("hgin_gat_bwd_src_f32");
  }
  HGIN_TRACE("k_gat_bwd_src");
  k_gat_bwd_src<<<blocks_for(n_src * H), 256, 0, as_stream(stream)>>>(cptr, cdst, cpos, n_src, (int)H, (int)C, g_out,
                                                                      ldg, alpha, g_pre, att_src, g_as, g_xs, ldgxs);
  return check_launch("hgin_gat_bwd_src_f32");
}

extern "C" int hgin_gat_wsum_workspace_size(int64_t n, int64_t H, int64_t C, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && n >= 0 && H >= 1 && C >= 1, "hgin_gat_wsum_workspace_size: bad args");
  *bytes = sizeof(float) * (size_t)wsum_blocks(n) * (size_t)(H * C);
  return HGIN_OK;
}

extern "C" int hgin_gat_wsum_f32(const float* x, int64_t ldx, int64_t n, int64_t H, int64_t C, const float* w,
                                 float* out, void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(n >= 0 && H >= 1 && C >= 1 && ldx >= H * C && out, "hgin_gat_wsum_f32: bad args");
  hipStream_t s = as_stream(stream);
  if (n == 0) return memset_async(out, 0, sizeof(float) * (size_t)(H * C), s, "hgin_gat_wsum_f32");
  const int64_t nb = wsum_blocks(n);
  const size_t need = sizeof(float) * (size_t)nb * (size_t)(H * C);
  if (!workspace || workspace_bytes < need) {
    set_error("hgin_gat_wsum_f32: workspace %zu < %zu", workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  HGIN_ARG_CHECK(x, "hgin_gat_wsum_f32: NULL x");
  float* part = static_cast<float*>(workspace);
  HGIN_TRACE("k_gat_wsum");
  k_gat_wsum_part<<<(unsigned)nb, 256, 0, s>>>(x, ldx, n, (int)H, (int)C, w, part);
  k_gat_wsum_final<<<(unsigned)(H * C), 256, 0, s>>>(part, nb, out);
  return check_launch("hgin_gat_wsum_f32");
}

// F1 — the reference's real training loop (dataset.py:26, :239-244; train.py:25-44): shuffled batches of a few small
// network graphs.  A batch of 8 RouteNet-sized graphs is a few thousand vertices, so the general path (one launch per
// relation, layer and GEMM family, ~100 per step even as one hipGraph replay) is bound by kernel boundaries, not work.
// Here the whole train step of a HetroGIN over a padded batch (hgin/store.py PaddedBatch) is 3 L + 1 launches (one
// fewer: the first layer needs no input gradient), every one spread over all rows of the batch (the graphs are
// disjoint, but a workgroup per graph leaves all but a handful of CUs idle and serialises each graph's dependent
// gathers — measured 1.15 ms per batch against the general path's 0.71).  Launch boundaries only where a phase reads
// rows another workgroup wrote (the aggregates and the readout); row-local phases share a launch:
//
//   k_sb_fwd    (per layer)   32 rows of one node type per workgroup: the CSR aggregate in edge order and the
//                             (1 + eps) x_dst self term of every relation into the type (concat in the first layer,
//                             add above it: models.py:210-215), then Linear + PReLU per relation (models.py:236-239)
//                             and their sum in relation order (HeteroConv, models.py:286-298);
//   k_sb_readout              tiles of 8 path rows:  the readout MLP (models.py:300-330, :362-376: hidden Linear
//                             + the ONE shared PReLU, Linear head), the MAPE numerator sum_rows |(out - y) / y|
//                             (train.py:12-13) and the readout backward seeded with d sum|u| / d out = sgn(u) / y,
//                             each layer's input and pre-activation gradient rows kept for the weight gradients;
//   k_sb_bwd_w  (per layer)   workgroup per (row chunk, relation): the chunk's g_z = PReLU'(z) g_y and g_comb = g_z W,
//                             then its partial W / bias / slope / eps gradients
//                             (the last and first layers' launches also the readout layers' partial W / bias
//                             gradients, half each);
//   k_sb_bwd_in (layers > 0)  thread per (node type, row, column): the layer input's gradient — every relation's self
//                             term and CSC aggregate of g_comb, in relation order;
//   k_sb_final                every parameter gradient = its partials summed in a fixed order, times d sqrt(loss) /
//                             d sum|u| = 100 / (2 m sqrt(loss_value)) (train.py:40-43; the seed above is linear),
//                             written into one flat gradient buffer whose views are the parameters' .grad;
//                             loss_value = 100 sum|u| / m.
//
// The optimizer: Adam folded into k_sb_final (each gradient entry updates its parameter and moments where it is
// formed: no gradient round trip, no optimizer launches), or torch's optimizer after the step in the same hipGraph.  Every sum runs in a fixed order (deterministic;
// the row chunks of the partials are fixed fractions of the batch's rows).  The aggregates are the GIN path's
// (sequential edge-order fp32 sums: bit-identical); the GEMM-shaped sums and the deferred loss scaling re-associate,
// so the step agrees with the general path within fp32 tolerances (tests/test_gpu_smallbatch.py).  Limits (checked
// by the host, hgin/smallbatch.py): H <= 128, every GEMM K <= 128, readout widths <= 256, at most 3 hidden readout
// layers and 4 GIN layers, fp32.  GLOBAL_FEATS: the first layer's launch also pools each graph's [mean | max]
// (sb_pool), which the readout gathers by row; MLP_BN: the readout runs as the k_sb_bn_* launches (below).
#include "hgin_common.h"

#include <cstddef>
#include <cstring>

namespace hgin {
namespace {

constexpr int kSbThreads = 256;
constexpr int kSbRows = 8;          // path rows per readout tile (hgin/smallbatch.py RO_ROWS)
constexpr int kSbMaxW = 256;        // widest readout layer input / output
constexpr int kSbMaxL = 4;
constexpr int kSbMaxHid = 3;
constexpr int kRel = 4;
// relation r = (src type, dst type), types path 0, link 1, node 2, in models.py:286-298 order
__device__ constexpr int kRelSrc[kRel] = {0, 1, 1, 2};
__device__ constexpr int kRelDst[kRel] = {1, 0, 2, 1};

struct SbConv {
  const float* w;      // [H, K]
  const float* b;      // [H]
  const float* slope;  // [1]
  const float* eps;    // [1]
  int64_t goff;        // offset of this conv's gradients in the flat buffer: W, b, slope, eps
};

// HetroGAT's GATConv of relation r (models.py:413-418, PyG 2.0.2 GATConv(( -1, -1), C, heads, concat=True)): its
// parameters and the offset of their gradients in the flat buffer: att_src [HC], att_dst [HC], bias [HC],
// lin_src.weight [HC][K_src], lin_dst.weight [HC][K_dst] (GATConv's named_parameters order)
struct SbGat {
  const float* ws;     // lin_src.weight [HC][K_src]
  const float* wd;     // lin_dst.weight [HC][K_dst]
  const float* att_s;  // att_src [heads][C]
  const float* att_d;  // att_dst [heads][C]
  const float* b;      // bias [HC]
  int64_t goff;
};

struct SbArgs {
  // batch
  const float* x[3];        // raw features per type (row stride ldx)
  int64_t ldx[3];
  int fdim[3];              // sliced widths
  int cols[3][8];           // sliced column -> raw column
  const int32_t* rowptr[kRel];
  const int32_t* col[kRel];
  const int32_t* cptr[kRel];   // CSC (by source)
  const int32_t* cdst[kRel];
  const int32_t* goff;      // [3][G + 1] per-graph node offsets (type-major)
  int G;
  const float* y;
  const int32_t* m_valid;
  // model
  int L, H;
  SbConv conv[kSbMaxL][kRel];
  int concat_path;
  int pool_w;               // GLOBAL_FEATS (models.py:347-352): 2 x the sliced path columns ([mean | max]), else 0
  int pool_ld;              // row stride of `pooled`
  float* pooled;            // [G][pool_ld]: graph g's [mean | max] of the sliced path columns (k_sb_fwd, layer 0)
  const int64_t* pbatch;    // [cap_path] the path rows' graph ids (PyG's batch vector)
  int nhid;
  int rw[kSbMaxHid];        // hidden widths
  const float* row_w[kSbMaxHid];   // [rw[i], in_i]
  const float* row_b[kSbMaxHid];
  const float* ro_slope;
  const float* head_w;      // [rw[nhid - 1]]
  const float* head_b;      // [1]
  int64_t ro_goff[kSbMaxHid];      // W_i then b_i
  int64_t ro_slope_goff, head_goff;   // head: W then b
  int64_t p_gin, p_ro;      // gradient counts of the GIN convs / the readout (flat buffer = [gin | readout])
  // scratch (capacity-sized; node rows indexed by batch row id)
  float* act;               // [L][3] blocks of cap_t x H
  int64_t act_off[kSbMaxL][3];
  float* comb;              // [L][4] blocks of cap_dst x K
  int64_t comb_off[kSbMaxL][kRel];
  float* zb;                // [L][4] blocks of cap_dst x H
  int64_t zb_off[kSbMaxL][kRel];
  float* gA;                // [3] blocks of cap_t x H  (gradient of the current layer's outputs)
  float* gB;                // same (gradient of its inputs)
  int64_t g_off[3];
  float* gc;                // [4] blocks of cap_dst x Kmax (g_comb per relation)
  int64_t gc_off[kRel];
  int kmax;                 // row stride of the gc blocks (relations differ in K)
  int cap[3];               // row capacity per node type (grid sizes)
  float* part_gin;          // [n_parts][p_gin]
  int n_parts;              // row chunks of the weight-gradient partials
  float* part_ro;           // [n_parts][p_ro] (row chunks of the path rows; the slope entry comes from slope_part)
  float* loss_part;         // [n_tiles]
  float* slope_part;        // [n_tiles] the shared readout slope's gradient
  int n_tiles;              // readout tiles of kSbRows path rows
  int ro_wlds;              // readout: 2 the 32-row MFMA tiles (4: their weights read through the caches), 1 8-row
                            // tiles with the weights in LDS, 0 without, 3 MLP_BN (k_sb_bn_*)
  float* ro_in[kSbMaxHid + 1];   // readout layer i's input rows [cap_path][win_i] (i = nhid: the head)
  float* ro_gz[kSbMaxHid + 1];   // its pre-activation gradient rows [cap_path][rw_i] (the head: [cap_path])
  // outputs
  float* gflat;             // [p_gin + p_ro]
  float* loss_value;        // [1]
  // the optimizer, folded into k_sb_final (adam_step NULL: the host runs torch's optimizer after the step)
  float* pflat;             // [p_gin + p_ro] the parameters (their tensors are views of it), gflat's layout
  float* mflat;             // Adam first moments, same layout
  float* vflat;             // Adam second moments
  float* adam_step;         // [1] Adam's step count (advanced by the step's first launch)
  float lr, beta1, beta2, adam_eps, weight_decay;
  // MLP_BN (models.py:303-313; ro_wlds 3, the k_sb_bn_* launches): hidden readout layer i = Linear -> BatchNorm1d
  // (training mode: statistics over the batch's m valid path rows) -> the shared PReLU
  const float* bn_w[kSbMaxHid];    // gamma [rw_i]
  const float* bn_b[kSbMaxHid];    // beta [rw_i]
  float* bn_rm[kSbMaxHid];         // running_mean / running_var, advanced in place once per step
  float* bn_rv[kSbMaxHid];
  int64_t* bn_nbt[kSbMaxHid];      // num_batches_tracked
  int64_t bn_goff[kSbMaxHid];      // flat offsets of gamma's gradients, then beta's
  float bn_eps, bn_mom;
  float* bn_buf;                   // scratch, per hidden layer the bn_ptr blocks at bn_off[i][0..4]
  int64_t bn_off[kSbMaxHid][5];
  // DROPOUT (models.py:358-359: F.dropout of every node type's output after each layer, training mode)
  int64_t* drop_ctr;               // [1] the step counter: fresh masks per step (advanced by k_sb_final)
  uint64_t drop_seed;
  uint32_t drop_thr;               // an element is dropped when its 32-bit hash is below round(p 2^32); 0: off
  float drop_inv;                  // 1 / (1 - p)
  // evaluation (train.py:70-113 test(), :322-348 evaluate(); hgin/smallbatch.py SmallBatchEval): the forward
  // launches, the readout up to its loss partial, and k_sb_final's loss only
  int eval_only;
  float* out_pred;                 // [cap_path] the head's outputs (eval; may be null)
  float* loss_acc;                 // [2] += loss_value, += loss_value * m (eval: test()'s running sums)
  // bit 4 l + r: conv (l, r) cannot reach the readout, so its parameters get no gradient in the
  // reference (.grad None) and torch's Adam skips them: the folded Adam leaves them (and their moments) untouched
  uint32_t dead_conv;
  // HetroGAT (models.py:380-506, train.py:120-125 MODEL == "GAT"): gat != 0 — the one layer is GATConvs (k_sb_gat_*),
  // H = gat_heads x gat_c; conv[0][r].goff = gatc[r].goff
  int gat;
  int gat_heads, gat_c;
  float gat_slope;                 // the attention logits' leaky ReLU slope (GATConv negative_slope, 0.2)
  SbGat gatc[kRel];
  float* gat_st;                   // per relation [cap_dst][heads][2 + K_src]: max logit, softmax denominator, the
  int64_t gat_st_off[kRel];        // softmax-weighted sum of the raw source rows (the forward's per-head aggregate)
};

// The dropout factor of element q (= row H + column) of layer l's type-t output: 0 (dropped, probability p) or
// 1 / (1 - p), from a splitmix64 hash of (seed, step counter, l, t, q) — the same in the step's forward and backward,
// fresh each step (torch's F.dropout draws from its generator instead: the same distribution, not the same masks)
__device__ __forceinline__ float drop_factor(const SbArgs& a, int l, int t, int64_t q) {
  if (a.drop_thr == 0u) return 1.0f;
  uint64_t x = a.drop_seed + (uint64_t)a.drop_ctr[0] * 0x9E3779B97F4A7C15ull;
  x ^= ((uint64_t)(l * 3 + t) << 56) ^ (uint64_t)q;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32) < a.drop_thr ? 0.0f : a.drop_inv;
}

__device__ __forceinline__ int kdim(const SbArgs& a, int l, int r) {
  return l == 0 ? a.fdim[kRelSrc[r]] + a.fdim[kRelDst[r]] : a.H;
}

// fixed-order block reduction over NT threads (all threads call it; returns the sum to every thread)
template <int NT = kSbThreads>
__device__ float block_sum(float v, float* red) {
  const int t = threadIdx.x;
  __syncthreads();
  red[t] = v;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
    __syncthreads();
  }
  const float s = red[0];
  __syncthreads();
  return s;
}

// two fixed-order block reductions at once (red: 2 NT floats): half the barriers of two block_sum calls, the same
// tree and order for each value
__device__ float2 block_sum2(float v, float w, float* red) {
  constexpr int NT = kSbThreads;
  const int t = threadIdx.x;
  __syncthreads();
  red[t] = v;
  red[NT + t] = w;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (t < off) {
      red[t] = __fadd_rn(red[t], red[t + off]);
      red[NT + t] = __fadd_rn(red[NT + t], red[NT + t + off]);
    }
    __syncthreads();
  }
  const float2 r = make_float2(red[0], red[NT]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ int nrows(const SbArgs& a, int t) { return a.goff[t * (a.G + 1) + a.G]; }

// sum over t < n of x[t sx] y[t sy], in t order (one fma chain onto acc); the operands are loaded 8 pairs at a time so
// that a chain costs a memory round trip per 8 terms, not per term (the small-batch kernels are latency-bound chains)
__device__ __forceinline__ float dot_chain(const float* x, int sx, const float* y, int sy, int n, float acc) {
  int t = 0;
  for (; t + 8 <= n; t += 8) {
    float xv[8], yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xv[j] = x[(t + j) * sx];
      yv[j] = y[(t + j) * sy];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(xv[j], yv[j], acc);
  }
  if (t < n) {   // the tail: clamped loads, the terms past n skipped
    float xv[8], yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int u = t + j < n ? t + j : n - 1;
      xv[j] = x[u * sx];
      yv[j] = y[u * sy];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t + j < n) acc = fmaf(xv[j], yv[j], acc);
  }
  return acc;
}

// acc[j] += sum over t < n of x[j xr + t] y[t sy] for the rows j < nrow (<= 4; the rows past nrow reread row 0),
// in t order: y loaded once per term for all the rows (a readout phase with >= 2 rows per thread: lanes along the
// outputs read y, the rows' x are broadcasts)
__device__ __forceinline__ void dot_rows4(const float* x, int xr, const float* y, int sy, int n, int nrow, float* acc) {
  const int xo[4] = {0, nrow > 1 ? xr : 0, nrow > 2 ? 2 * xr : 0, nrow > 3 ? 3 * xr : 0};
  for (int t = 0; t < n; t += 8) {
    float yv[8], xv[4][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int u = t + j < n ? t + j : n - 1;
      yv[j] = y[u * sy];
#pragma unroll
      for (int r = 0; r < 4; ++r) xv[r][j] = x[xo[r] + u];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t + j < n) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(xv[r][j], yv[j], acc[r]);
      }
  }
}

// threads per output of a readout phase with nout outputs of len-term sums: a power of two <= 16 that keeps the
// phase within one pass of the workgroup and >= 4 terms per thread (thread s of an output sums terms s, s + S, ...;
// the S adjacent lanes then combine in a fixed xor tree, identical on every lane)
template <int NT = kSbThreads>
__device__ __forceinline__ int split_of(int nout, int len) {
  int S = 1;
  while (S < 16 && nout * S * 2 <= NT && len >= 8 * S) S *= 2;
  return S;
}
__device__ __forceinline__ float group_sum(float v, int S) {
  for (int off = 1; off < S; off <<= 1) v = __fadd_rn(v, __shfl_xor(v, off));
  return v;
}

// sum over t < n of x[t sx] onto acc, in t order (one add chain; 8 loads in flight)
__device__ __forceinline__ float sum_chain(const float* x, int64_t sx, int n, float acc) {
  int t = 0;
  for (; t + 8 <= n; t += 8) {
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = x[(t + j) * sx];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __fadd_rn(acc, xv[j]);
  }
  if (t < n) {
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = x[(t + j < n ? t + j : n - 1) * sx];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t + j < n) acc = __fadd_rn(acc, xv[j]);
  }
  return acc;
}

// sum over edges e in [e0, e1) of xs[col[e] ld + c] onto acc, in edge order: 8 column indices, then their 8 values,
// in flight at a time (two dependent round trips per 8 edges instead of per edge)
__device__ __forceinline__ float gather_chain(const int32_t* col, int e0, int e1, const float* xs, int64_t ld, int c,
                                              float acc) {
  for (int e = e0; e < e1; e += 8) {
    int ci[8];
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ci[j] = col[e + j < e1 ? e + j : e1 - 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = xs[(int64_t)ci[j] * ld + c];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (e + j < e1) acc = __fadd_rn(acc, xv[j]);
  }
  return acc;
}

// gather_chain for 4 (row range, column) pairs at once: 8 edges of each in flight per round trip (32 loads), each
// pair's sum in its own edge order (bit-identical to gather_chain per pair); a pair with e0 >= e1 adds nothing
__device__ __forceinline__ void gather_chain4(const int32_t* col, const int (&e0)[4], const int (&e1)[4],
                                              const float* xs, int64_t ld, const int (&c)[4], float (&acc)[4]) {
  int emax = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) emax = e1[j] - e0[j] > emax ? e1[j] - e0[j] : emax;
  for (int o = 0; o < emax; o += 8) {
    int ci[4][8];
    float xv[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 8; ++u) ci[j][u] = e0[j] + o + u < e1[j] ? col[e0[j] + o + u] : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[j][u] = xs[(int64_t)ci[j][u] * ld + c[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0[j] + o + u < e1[j]) acc[j] = __fadd_rn(acc[j], xv[j][u]);
  }
}

// n contiguous floats from global memory into LDS, every load of a thread issued before its first store (one
// memory round trip for up to J x kSbThreads floats)
template <int J = 32>
__device__ __forceinline__ void copy_flat(float* dst, const float* src, int n) {
  for (int b = threadIdx.x; b < n; b += J * kSbThreads) {
    float v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = src[b + j * kSbThreads < n ? b + j * kSbThreads : n - 1];
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (b + j * kSbThreads < n) dst[b + j * kSbThreads] = v[j];
  }
}

// One layer's forward for kSbFwdRows rows of node type t (grid = row blocks x types): per relation into t (relation
// order) comb_r = [aggregate | (1 + eps) x_dst] (concat, first layer) or aggregate + (1 + eps) x_dst (add), the
// aggregate a sequential edge-order sum (models.py:210-215); then per row and output column the sum over those
// relations of prelu(comb_r W_r^T + b_r) (models.py:236-239; HeteroConv's sum, models.py:286-298), z kept per
// relation for the backward.  comb_r also goes to HBM (the weight gradients read it).
constexpr int kSbFwdRows = 32;

typedef float sb_f32x16 __attribute__((ext_vector_type(16)));
template <int NT, int KB = 4, class Epi>
__device__ __forceinline__ void tile_mfma(const float* A, int lda, int nr, const float* Bm, int bsk, int bsn, int N,
                                          int K, float* red, Epi epi);

constexpr int kSbFwdW = 1024;   // k_sb_fwd stages a relation's W [H][K] in LDS when it has at most this many entries

// GLOBAL_FEATS (models.py:347-352, global_mean_pool / global_max_pool of the sliced path features by the batch
// vector): the first layer's fourth grid row, a workgroup per graph; the f sliced columns x 256 / f row lanes (rows
// strided by the lane count), then per column the lanes' (sum, max) in lane order: sum / rows and the max (the first
// maximum; a NaN propagates, as torch's max).  pooled[g] = [mean | max]; the readout gathers it by row (torch.gather,
// models.py:350-351).
__device__ void sb_pool(const SbArgs& a, float* red) {
  const int f = a.pool_w >> 1, tid = threadIdx.x;
  const int lanes = kSbThreads / f, c = tid % f, lane = tid / f;
  for (int g = blockIdx.x; g < a.G; g += gridDim.x) {
    const int lo = a.goff[g], hi = a.goff[g + 1];
    float s = 0.0f, m = -INFINITY;
    if (lane < lanes) {
      const float* xc = a.x[0] + a.cols[0][c];
      for (int r = lo + lane; r < hi; r += lanes) {
        const float v = xc[(int64_t)r * a.ldx[0]];
        s = __fadd_rn(s, v);
        if (v > m || v != v) m = v;
      }
    }
    __syncthreads();
    red[tid] = s;
    red[kSbThreads + tid] = m;
    __syncthreads();
    if (tid < f) {
      float S = 0.0f, M = -INFINITY;
      for (int q = 0; q < lanes; ++q) {
        S = __fadd_rn(S, red[q * f + tid]);
        const float v = red[kSbThreads + q * f + tid];
        if (v > M || v != v) M = v;
      }
      a.pooled[(int64_t)g * a.pool_ld + tid] = __fdiv_rn(S, (float)(hi - lo));
      a.pooled[(int64_t)g * a.pool_ld + f + tid] = M;
    }
  }
}

// kM (hidden >= 64): the Linear of each relation on the matrix cores — tile_mfma over 32-column chunks of W staged in
// LDS, the chunks' partial sums added in chunk order — instead of one dot chain per output (at H = 128 a 128-term
// chain per output made the launch ~120 us); comb rows at an odd stride (the MFMA operand reads a column of rows)
// kM blocks hold 8 rows (round 6): a thread's 4 gather chains of a 128-wide layer are then one gather_chain4 batch
// instead of four after each other, the blocks are 4x as many and 3 fit a CU (hidden 128: 64.8 -> see DESIGN.md §3);
// the MFMA tile's rows past 8 are zeros (tile_mfma's nr), and every output is the same sum in the same order
constexpr int kSbFwdRowsM = 8;
constexpr int kFwdMW = 128 * 17, kFwdMT = kSbFwdRowsM * 129;   // W chunks of 16 columns; the z tile
template <bool kM>
__global__ __launch_bounds__(kSbThreads) void k_sb_fwd(SbArgs a, int l) {
  constexpr int R = kM ? kSbFwdRowsM : kSbFwdRows;   // rows per workgroup
  __shared__ float s_comb[2][kM ? R * 129 : R * 128];   // <= 2 relations into a type, K <= 128
  __shared__ float s_w[2][kM ? 1 : kSbFwdW];           // (kM: H * K > kSbFwdW, W goes through s_m in chunks)
  __shared__ float s_m[kM ? kFwdMW + kFwdMT + (kSbThreads / 64) * 32 * 33 : 1];   // W chunk | z | split partials
  const int t = blockIdx.y;
  if (t == 3) {   // (the first layer with GLOBAL_FEATS)
    sb_pool(a, &s_comb[0][0]);
    return;
  }
  const int tid = threadIdx.x;
  const int H = a.H;
  const int n = nrows(a, t);
  const int r0 = blockIdx.x * R;
  if (a.adam_step && l == 0 && blockIdx.x == 0 && t == 0 && tid == 0) a.adam_step[0] += 1.0f;   // read by k_sb_final
  if (r0 >= n) return;
  const int nr = n - r0 < R ? n - r0 : R;
  // the relations' small weights into LDS first: their loads fly with the aggregate's gathers
  int wl = 0;   // bit sl: relation slot sl's W is in s_w[sl] (the scalar Linear only: kM stages W in chunks)
  if constexpr (!kM) {
    int sl = 0;
    for (int r = 0; r < kRel; ++r) {
      if (kRelDst[r] != t) continue;
      const int HK = H * kdim(a, l, r);
      if (HK <= kSbFwdW) {
        wl |= 1 << sl;
        copy_flat<4>(s_w[sl], a.conv[l][r].w, HK);
      }
      ++sl;
    }
  }
  int slot = 0;
  for (int r = 0; r < kRel; ++r) {
    if (kRelDst[r] != t) continue;
    const int s = kRelSrc[r];
    const int K = kdim(a, l, r);
    const SbConv& cv = a.conv[l][r];
    const float sc = __fadd_rn(1.0f, cv.eps[0]);
    const int32_t* rp = a.rowptr[r];
    const int32_t* cl = a.col[r];
    float* comb = a.comb + a.comb_off[l][r] + (int64_t)r0 * K;
    if (kM && l > 0) {   // (wide rows: 4 elements' gather chains per thread in flight together)
      const float* xs = a.act + a.act_off[l - 1][s];
      const float* xd = a.act + a.act_off[l - 1][t];
      for (int b0 = tid; b0 < nr * K; b0 += 4 * kSbThreads) {
        int e0[4], e1[4], cc[4];
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int idx = b0 + j * kSbThreads;
          const bool ok = idx < nr * K;
          const int i = r0 + (ok ? idx / K : 0);
          cc[j] = ok ? idx % K : 0;
          e0[j] = rp[i];
          e1[j] = ok ? rp[i + 1] : e0[j];
          v[j] = 0.0f;
        }
        gather_chain4(cl, e0, e1, xs, H, cc, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int idx = b0 + j * kSbThreads;
          if (idx < nr * K) {
            const int rr = idx / K;
            const float w = __fadd_rn(v[j], __fmul_rn(sc, xd[(int64_t)(r0 + rr) * H + cc[j]]));
            s_comb[slot][rr * (K | 1) + cc[j]] = w;
            comb[idx] = w;
          }
        }
      }
      ++slot;
      continue;
    }
    for (int idx = tid; idx < nr * K; idx += kSbThreads) {
      const int i = r0 + idx / K, k = idx % K;
      float v = 0.0f;
      if (l == 0) {
        const int fs = a.fdim[s];
        if (k < fs) {
          const float* xs = a.x[s];
          const int64_t ld = a.ldx[s];
          const int c = a.cols[s][k];
          v = gather_chain(cl, rp[i], rp[i + 1], xs, ld, c, v);
        } else {
          v = __fmul_rn(sc, a.x[t][(int64_t)i * a.ldx[t] + a.cols[t][k - fs]]);
        }
      } else {
        const float* xs = a.act + a.act_off[l - 1][s];
        v = gather_chain(cl, rp[i], rp[i + 1], xs, H, k, v);
        v = __fadd_rn(v, __fmul_rn(sc, a.act[a.act_off[l - 1][t] + (int64_t)i * H + k]));
      }
      s_comb[slot][kM ? (idx / K) * (K | 1) + idx % K : idx] = v;
      comb[idx] = v;
    }
    ++slot;
  }
  __syncthreads();
  if constexpr (kM) {
    float* s_wc = s_m;               // [H][17]: W[:, kc : kc + 16]
    float* s_z = s_m + kFwdMW;       // [R][H | 1]
    float* red = s_z + kFwdMT;
    const int ly = H | 1;
    int nrel = 0;
    for (int r = 0; r < kRel; ++r) nrel += kRelDst[r] == t;
    float* act = a.act + a.act_off[l][t] + (int64_t)r0 * H;
    int sl = 0;
    for (int r = 0; r < kRel; ++r) {
      if (kRelDst[r] != t) continue;
      const int K = kdim(a, l, r), lc = K | 1;
      const SbConv& cv = a.conv[l][r];
      for (int kc = 0; kc < K; kc += 16) {
        const int kn = K - kc < 16 ? K - kc : 16;
        __syncthreads();   // the previous chunk's / relation's readers of s_wc, s_z
        for (int idx = tid; idx < H * 16; idx += kSbThreads) {
          const int n = idx >> 4, kk = idx & 15;
          if (kk < kn) s_wc[n * 17 + kk] = cv.w[(int64_t)n * K + kc + kk];
        }
        __syncthreads();
        tile_mfma<kSbThreads>(s_comb[sl] + kc, lc, nr, s_wc, 1, 17, H, kn, red, [&](int rr, int n, float v) {
          s_z[rr * ly + n] = kc == 0 ? v : __fadd_rn(s_z[rr * ly + n], v);
        });
      }
      __syncthreads();
      float* zb = a.zb + a.zb_off[l][r] + (int64_t)r0 * H;
      const float slope = cv.slope[0];
      // the relations' PReLU outputs summed in relation order in the output rows themselves (each element by the
      // same thread), the dropout with the last
      for (int idx = tid; idx < nr * H; idx += kSbThreads) {
        const int ii = idx / H, h = idx - ii * H;
        const float z = __fadd_rn(s_z[ii * ly + h], cv.b[h]);
        zb[idx] = z;
        const float yv = z > 0.0f ? z : __fmul_rn(slope, z);
        float y = sl == 0 ? yv : __fadd_rn(act[idx], yv);
        if (sl == nrel - 1 && a.drop_thr) y = __fmul_rn(y, drop_factor(a, l, t, (int64_t)r0 * H + idx));
        act[idx] = y;
      }
      ++sl;
    }
    return;
  }
  for (int idx = tid; idx < nr * H; idx += kSbThreads) {
    const int ii = idx / H, h = idx % H;
    float y = 0.0f;
    bool first = true;
    int sl = 0;
    for (int r = 0; r < kRel; ++r) {
      if (kRelDst[r] != t) continue;
      const int K = kdim(a, l, r);
      const SbConv& cv = a.conv[l][r];
      const float* cr = s_comb[sl] + ii * K;
      float z = (wl >> sl) & 1 ? dot_chain(cr, 1, s_w[sl] + h * K, 1, K, 0.0f) : dot_chain(cr, 1, cv.w + (int64_t)h * K, 1, K, 0.0f);
      ++sl;
      z = __fadd_rn(z, cv.b[h]);
      a.zb[a.zb_off[l][r] + (int64_t)(r0 + ii) * H + h] = z;
      const float yv = z > 0.0f ? z : __fmul_rn(cv.slope[0], z);
      y = first ? yv : __fadd_rn(y, yv);
      first = false;
    }
    const int64_t q = (int64_t)(r0 + ii) * H + h;
    a.act[a.act_off[l][t] + q] = a.drop_thr ? __fmul_rn(y, drop_factor(a, l, t, q)) : y;
  }
}

// n / d for 0 <= n < 2^16, 1 <= d < 2^16 by one multiply-high: m = floor(2^32 / d) + 1 over-estimates 1 / d by less
// than 2^-32, which moves n / d by less than 2^-16 < 1 / d, so the floor is exact
struct FastDiv {
  unsigned m;
  int d;
};
__device__ __forceinline__ FastDiv fast_div(int d) { return {d > 1 ? 0xFFFFFFFFu / (unsigned)d + 1u : 0u, d}; }
__device__ __forceinline__ int fdq(const FastDiv& f, int n) { return f.d > 1 ? (int)__umulhi((unsigned)n, f.m) : n; }

// column k of path row `row`'s readout input (models.py:362-371): the final path embedding (H columns), then the
// sliced raw path features when concat_path (fp columns), then GLOBAL_FEATS' [mean | max] of the sliced columns
// over the row's graph (pool_w = 2 fp columns, read from the pooled rows of every raw column)
__device__ __forceinline__ float readout_input(const SbArgs& a, const float* xp, int64_t row, int k, int H, int fp) {
  if (k < H) return xp[row * H + k];
  if (k < H + fp) return a.x[0][row * a.ldx[0] + a.cols[0][k - H]];
  return a.pooled[a.pbatch[row] * a.pool_ld + (k - H - fp)];
}

// The readout's parameters into LDS (kWL; otherwise only the offsets / strides of the global rows): per hidden layer
// W_i [rw_i][win_i | 1] (rows padded to an odd stride: lanes reading different W rows and lanes reading along one
// are both conflict-free) and b_i [rw_i], then the head's W [KL]; every load of a thread in flight at once (up to
// kStageW slots of each W), then the padded stores.  Returns the first float past them.
template <bool kWL, int NT = kSbThreads>
__device__ __forceinline__ int stage_ro_params(const SbArgs& a, float* sm, int nh, const int (&win)[kSbMaxHid + 1],
                                               int KL, int (&oW)[kSbMaxHid], int (&ldw)[kSbMaxHid]) {
  const int tid = threadIdx.x;
  int off = 0;
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    oW[i] = off;
    ldw[i] = kWL ? (win[i] | 1) : win[i];
    if (kWL && i < nh) off += a.rw[i] * (ldw[i] + 1);
  }
  if (kWL) {
    const int oH = off;
    off += KL;
    // every parameter load of a thread in flight at once (up to kStageW slots of each W), then the padded stores
    constexpr int kStageW = 16;
    float vw[kSbMaxHid][kStageW], vb[kSbMaxHid];
#pragma unroll
    for (int i = 0; i < kSbMaxHid; ++i) {
      if (i < nh) {
        const int n = win[i] * a.rw[i], N = a.rw[i];
#pragma unroll
        for (int j = 0; j < kStageW; ++j) vw[i][j] = a.row_w[i][tid + j * NT < n ? tid + j * NT : n - 1];
        vb[i] = a.row_b[i][tid < N ? tid : N - 1];
      }
    }
    const float vh = a.head_w[tid < KL ? tid : KL - 1];
#pragma unroll
    for (int i = 0; i < kSbMaxHid; ++i) {
      if (i < nh) {
        const int K = win[i], N = a.rw[i], n = K * N;
        const FastDiv fk = fast_div(K);
#pragma unroll
        for (int j = 0; j < kStageW; ++j) {
          const int idx = tid + j * NT;
          const int q = fdq(fk, idx);
          if (idx < n) sm[oW[i] + q * ldw[i] + idx - q * K] = vw[i][j];
        }
        for (int idx = tid + kStageW * NT; idx < n; idx += NT) {   // (wider layers than cfg1's)
          const int q = idx / K;
          sm[oW[i] + q * ldw[i] + idx - q * K] = a.row_w[i][idx];
        }
        for (int o = tid; o < N; o += NT) sm[oW[i] + N * ldw[i] + o] = o == tid ? vb[i] : a.row_b[i][o];
      }
    }
    for (int k = tid; k < KL; k += NT) sm[oH + k] = k == tid ? vh : a.head_w[k];
  }
  return off;
}

// Tiles of kSbRows path rows (a grid-stride loop over the batch's tiles): readout forward, loss partial, readout
// backward (unscaled) down to the path embeddings' gradient.  Each layer's input rows and pre-activation gradient rows
// go to ro_in / ro_gz, from which the readout blocks of k_sb_bwd_w form the weight-gradient partials over the same
// row chunks as the GIN's (a tile that also reduced its own rows' weight gradients spent most of its time there and
// left n_tiles partials to sum).  kWL: the readout's parameters are staged in LDS in the flat gradient layout (rows
// unpadded: the backward's lanes read along a W row, and the forward's, which read different W rows, start at rotated
// columns when the row stride is even, so both are free of bank conflicts).  The layer loops are unrolled over kSbMaxHid so that every buffer pointer is a
// known LDS (or global) address, and each phase splits its sums over split_of() lanes: a tile is a chain of short
// dependent phases, and its time is their LDS round trips (profiles/r05: 34 us per batch when every term was one).
// HGIN_SB_STAMPS (a diagnostic build only, tools/sb_stamps.py): thread 0 of each readout workgroup writes the
// wall clock at its phase boundaries, each bwd_w block at its start and end (read back by hgin_sb_stamps_read)
#ifdef HGIN_SB_STAMPS
constexpr int kStampRo = 1024 * 16, kStampW = 2 * 2048 * 2;
__device__ unsigned long long g_sb_stamps[kStampRo + kStampW];
#define SB_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < 1024) g_sb_stamps[blockIdx.x * 16 + (k)] = wall_clock64()
#define SB_STAMP_W(l, k)                                                                      \
  if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < 2048)                         \
  g_sb_stamps[kStampRo + ((l) * 2048 + blockIdx.y * gridDim.x + blockIdx.x) * 2 + (k)] = wall_clock64()
#else
#define SB_STAMP(k)
#define SB_STAMP_W(l, k)
#endif

// MLP_BN in evaluation (SmallBatchEval): hidden layer i's BatchNorm1d with its running statistics, an affine map per
// column — (z - running_mean) / sqrt(running_var + eps) gamma + beta, torch's eval-mode order of operations
__device__ __forceinline__ float bn_eval(const SbArgs& a, int i, int n, float z) {
  if (!a.eval_only || !a.bn_w[i]) return z;
  const float xh = __fdiv_rn(__fsub_rn(z, a.bn_rm[i][n]), sqrtf(__fadd_rn(a.bn_rv[i][n], a.bn_eps)));
  return __fadd_rn(__fmul_rn(xh, a.bn_w[i][n]), a.bn_b[i][n]);
}

template <bool kWL>
__global__ __launch_bounds__(kSbThreads) void k_sb_readout(SbArgs a) {
  extern __shared__ float sm[];
  __shared__ float red[kSbThreads];
  const int tid = threadIdx.x;
  const int H = a.H;
  const int m = a.m_valid[0];
  constexpr int R = kSbRows;
  const int ntile = (m + R - 1) / R;
  if ((int)blockIdx.x >= ntile) return;   // (the grid is sized for the capacity; uniform per workgroup)
  SB_STAMP(0);
  const int nh = a.nhid;
  const int fp = a.concat_path ? a.fdim[0] : 0;
  const int w0 = H + fp + a.pool_w;
  int win[kSbMaxHid + 1];   // input width of layer i (i = nhid: the head)
  win[0] = w0;
  int maxw = w0;
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    win[i + 1] = i < nh ? a.rw[i] : 0;
    maxw = i < nh && a.rw[i] > maxw ? a.rw[i] : maxw;
  }
  const int KL = a.rw[nh - 1];
  // LDS: [kWL: per hidden layer W_i [rw_i][win_i | 1] (rows padded to an odd stride: the forward's lanes read
  // different W rows, the backward's read along one; both conflict-free) and b_i [rw_i], then the head's W [KL]] in0
  // [R][w0] | z_i, y_i [R][rw_i] per hidden layer | gbuf x2 [R][maxw] | outv [R].  (Float offsets, not pointer arrays:
  // the pointers formed from them at each use are plain LDS addresses, where arrays of pointers became generic ones.)
  int oW[kSbMaxHid], ldw[kSbMaxHid];
  int off = stage_ro_params<kWL>(a, sm, nh, win, KL, oW, ldw);
  const int oH = off - (kWL ? KL : 0);
  const float* hw = kWL ? (const float*)(sm + oH) : a.head_w;
  int oZ[kSbMaxHid], oY[kSbMaxHid];
  float* in0 = sm + off;
  off += R * w0;
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    oZ[i] = oY[i] = off;
    if (i < nh) {
      oY[i] = off + R * a.rw[i];
      off += 2 * R * a.rw[i];
    }
  }
  float* gb0 = sm + off;
  float* gb1 = gb0 + R * maxw;
  float* outv = gb1 + R * maxw;   // [R]
#define RO_W(i) (kWL ? (const float*)(sm + oW[i]) : a.row_w[i])
#define RO_B(i) (kWL ? (const float*)(sm + oW[i] + a.rw[i] * ldw[i]) : a.row_b[i])
  const float* xp = a.act + a.act_off[a.L - 1][0];
  const float slope = a.ro_slope[0];
  const float head_b = a.head_b[0];
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int r0 = tile * R;
    const int nr = m - r0 < R ? m - r0 : R;
    __syncthreads();   // the staged weights / the previous tile's LDS reads
    SB_STAMP(1);
    for (int idx = tid; idx < nr * w0; idx += kSbThreads) {
      const int rr = idx / w0, k = idx % w0;
      const int64_t row = r0 + rr;
      const float v = readout_input(a, xp, row, k, H, fp);
      in0[rr * w0 + k] = v;
      a.ro_in[0][(int64_t)r0 * w0 + idx] = v;
    }
    __syncthreads();
    SB_STAMP(2);
#pragma unroll
    for (int i = 0; i < kSbMaxHid; ++i) {
      if (i < nh) {
        const float* in = i == 0 ? in0 : sm + oY[i > 0 ? i - 1 : 0];
        const int K = win[i], N = a.rw[i];
        auto epi = [&](int q, int o, float z) {
          z = bn_eval(a, i, o, __fadd_rn(z, RO_B(i)[o]));
          sm[oZ[i] + q] = z;
          const float yv = z > 0.0f ? z : __fmul_rn(slope, z);
          sm[oY[i] + q] = yv;
          a.ro_in[i + 1][(int64_t)r0 * N + q] = yv;
        };
        if (nr * N >= 2 * kSbThreads) {   // >= 2 rows per thread: up to 4 rows share each W load
          const int CT = N < kSbThreads ? N : kSbThreads, RG = kSbThreads / CT;
          for (int c0 = 0; c0 < N; c0 += CT) {
            const int o = c0 + tid % CT;
            if (tid < RG * CT && o < N) {
              for (int rb = tid / CT; rb < nr; rb += 4 * RG) {
                const int nrow = (nr - rb + RG - 1) / RG < 4 ? (nr - rb + RG - 1) / RG : 4;
                float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                dot_rows4(in + rb * K, RG * K, RO_W(i) + o * ldw[i], 1, K, nrow, acc);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (j < nrow) epi((rb + j * RG) * N + o, o, acc[j]);
              }
            }
          }
        } else {
          const int S = split_of(nr * N, K);
          for (int idx = tid; idx < nr * N * S; idx += kSbThreads) {
            const int q = idx / S, s = idx % S;
            const int rr = q / N, o = q % N;
            float z = dot_chain(in + rr * K + s, S, RO_W(i) + o * ldw[i] + s, S, (K - s + S - 1) / S, 0.0f);
            z = group_sum(z, S);
            if (s == 0) epi(q, o, z);
          }
        }
        __syncthreads();
        SB_STAMP(3 + i);
      }
    }
    const float* yl = sm + (nh == 1 ? oY[0] : (nh == 2 ? oY[1] : oY[2]));
    // head + loss numerator + seed, split_of() lanes per row
    {
      const int S = split_of(nr, KL);
      for (int idx = tid; idx < nr * S; idx += kSbThreads) {
        const int rr = idx / S, s = idx % S;
        float o = dot_chain(yl + rr * KL + s, S, hw + s, S, (KL - s + S - 1) / S, 0.0f);
        o = group_sum(o, S);
        if (s == 0) {
          o = __fadd_rn(o, head_b);
          if (a.out_pred) a.out_pred[r0 + rr] = o;
          const float yv = a.y[r0 + rr];
          const float u = __fdiv_rn(__fsub_rn(o, yv), yv);
          red[rr] = fabsf(u);
          const float sg = u > 0.0f ? 1.0f : (u < 0.0f ? -1.0f : 0.0f);
          const float go = __fdiv_rn(sg, yv);   // d |u| / d out
          outv[rr] = go;
          a.ro_gz[nh][r0 + rr] = go;
        }
      }
    }
    __syncthreads();
    SB_STAMP(6);
    // fixed-order tile sum of |u| (rows in order)
    if (tid == 0) {
      float s = 0.0f;
      for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, red[rr]);
      a.loss_part[tile] = s;
    }
    if (a.eval_only) continue;   // (uniform; the next tile's loop head syncs)
    for (int idx = tid; idx < nr * KL; idx += kSbThreads) {
      const int rr = idx / KL, k = idx % KL;
      gb0[rr * KL + k] = __fmul_rn(outv[rr], hw[k]);
    }
    __syncthreads();
    SB_STAMP(7);
    float slope_part = 0.0f;   // this thread's share of the shared slope's gradient (fixed assignment)
    float* g_y = gb0;
    float* g_next = gb1;
#pragma unroll
    for (int i = kSbMaxHid - 1; i >= 0; --i) {
      if (i < nh) {
        const int K = win[i], N = a.rw[i];
        // g_z (in place over g_y) and the slope partial
        for (int idx = tid; idx < nr * N; idx += kSbThreads) {
          const float z = sm[oZ[i] + idx];
          const float g = g_y[idx];
          if (z <= 0.0f) slope_part = fmaf(g, z, slope_part);
          const float gz = z > 0.0f ? g : __fmul_rn(slope, g);
          g_y[idx] = gz;
          a.ro_gz[i][(int64_t)r0 * N + idx] = gz;
        }
        __syncthreads();
        SB_STAMP(8 + 2 * i);
        // g_in[k] = sum_o g_z[o] W[o][k] (the first layer: only the path embeddings' H columns have a gradient)
        const int KG = i == 0 ? H : K;
        if (nr * KG >= 2 * kSbThreads) {   // >= 2 rows per thread: up to 4 rows share each W load
          const int CT = KG < kSbThreads ? KG : kSbThreads, RG = kSbThreads / CT;
          for (int c0 = 0; c0 < KG; c0 += CT) {
            const int k = c0 + tid % CT;
            if (tid < RG * CT && k < KG) {
              for (int rb = tid / CT; rb < nr; rb += 4 * RG) {
                const int nrow = (nr - rb + RG - 1) / RG < 4 ? (nr - rb + RG - 1) / RG : 4;
                float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                dot_rows4(g_y + rb * N, RG * N, RO_W(i) + k, ldw[i], N, nrow, acc);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (j < nrow) g_next[(rb + j * RG) * KG + k] = acc[j];
              }
            }
          }
        } else {
          const int S = split_of(nr * KG, N);
          for (int idx = tid; idx < nr * KG * S; idx += kSbThreads) {
            const int q = idx / S, s = idx % S;
            const int rr = q / KG, k = q % KG;
            float v = dot_chain(g_y + rr * N + s, S, RO_W(i) + s * ldw[i] + k, S * ldw[i], (N - s + S - 1) / S, 0.0f);
            v = group_sum(v, S);
            if (s == 0) g_next[q] = v;
          }
        }
        __syncthreads();
        SB_STAMP(9 + 2 * i);
        float* t = g_y;
        g_y = g_next;
        g_next = t;
      }
    }
    const float sp = block_sum(slope_part, red);
    SB_STAMP(12);
    if (tid == 0) a.slope_part[tile] = sp;
    // the path embeddings' gradient for the GIN backward
    float* gpath = a.gA + a.g_off[0];
    for (int idx = tid; idx < nr * H; idx += kSbThreads) gpath[(int64_t)r0 * H + idx] = g_y[idx];
    SB_STAMP(13);
  }
}
#undef RO_W
#undef RO_B

// ---------------------------------------------------------------------------------------------------------------
// The readout on the matrix cores (hgin_sb_readout_lds_bytes mode 2, the default where it fits): tiles of 32 path
// rows, each readout GEMM of the tile — the hidden layers' forward, their input gradients — as 32 x 32 blocks of
// v_mfma_f32_32x32x2_f32 (fp32 products, fp32 accumulation) over LDS operands.  A quarter as many workgroups stage the
// parameters, and a phase is a few dozen MFMAs per wave instead of a chain of dependent LDS round trips per output
// (profiles/r05/sb/stamps_after.txt: 12 such phases made the 8-row scalar tile's ~20 us).
constexpr int kSbRowsM = 32;
constexpr int kRoThreadsM = 512;   // 8 waves: 2 per SIMD, so one wave's LDS / MFMA latency overlaps the other's

// C[32 x N] = A[32 x K] B[K x N] for one tile: A(r, k) = A[r asr + k ask] (rows >= nr read as zero), B(k, n) =
// Bm[k bsk + n bsn].  The ceil(N / 32) column blocks go to the NT / 64 waves; with fewer blocks than waves a block's
// k-steps are split over the idle ones (a fixed power-of-two split) and the partials, parked in red [NT / 64][32][33],
// are added in split order.
// epi(r, n, v) receives every output of rows < nr and columns < N (v = 0 + the products in k order within a split).
// KB k-steps' operands are loaded together before their MFMAs: 4 for LDS operands; 16 where an operand comes through
// the caches (a weight matrix too large to stage), so a 128-deep product is 4 dependent L2 round trips instead of 16
// (round 6: hidden 128 / the GAT readout — the same products in the same order)
template <int NT, int KB = 4, class Epi>
__device__ __forceinline__ void tile_mfma_s(const float* A, int asr, int ask, int nr, const float* Bm, int bsk, int bsn,
                                            int N, int K, float* red, Epi epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int nb = (N + 31) >> 5;
  constexpr int W = NT / 64;
  // k-splits per block (a power of two) only for one or two column blocks: from three up, the partials' extra
  // barrier and pass cost more than the idle waves would save (profiles/r05/sb/stamps_mfma512.txt)
  int ks = 1;
  while (nb <= 2 && nb * ks * 2 <= W) ks *= 2;
  const int steps = (K + 1) >> 1;
  const int sc = (steps + ks - 1) / ks;
  const bool rok = li < nr;
  const int rc = rok ? li : 0;
  for (int task = w; task < nb * ks; task += W) {
    const int cb = task % nb, sp = task / nb;
    const int n = cb * 32 + li;
    const bool nok = n < N;
    const int nc = nok ? n : N - 1;
    const int s0 = sp * sc, s1 = s0 + sc < steps ? s0 + sc : steps;
    sb_f32x16 acc;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    for (int st = s0; st < s1; st += KB) {   // KB k-steps' operands loaded together, then their MFMAs
      float av[KB], bv[KB];
#pragma unroll
      for (int q = 0; q < KB; ++q) {
        const int k = 2 * (st + q) + lh;
        const bool kok = st + q < s1 && k < K;
        const int kc = k < K ? k : K - 1;
        const float x = A[rc * asr + kc * ask], y = Bm[kc * bsk + nc * bsn];
        av[q] = rok && kok ? x : 0.0f;
        bv[q] = nok && kok ? y : 0.0f;
      }
#pragma unroll
      for (int q = 0; q < KB; ++q)
        if (st + q < s1) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc, 0, 0, 0);
    }
    if (ks == 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int r = (j & 3) + 8 * (j >> 2) + 4 * lh;   // the 32 x 32 accumulator layout: column li, row r
        if (r < nr && nok) epi(r, n, acc[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) red[(task * 32 + (j & 3) + 8 * (j >> 2) + 4 * lh) * 33 + li] = acc[j];
    }
  }
  if (ks > 1) {
    __syncthreads();
    for (int idx = threadIdx.x; idx < nr * N; idx += NT) {
      const int r = idx / N, n = idx % N, cb = n >> 5;
      float v = 0.0f;
      for (int sp = 0; sp < ks; ++sp) v = __fadd_rn(v, red[((sp * nb + cb) * 32 + r) * 33 + (n & 31)]);
      epi(r, n, v);
    }
  }
}

// A(r, k) = A[r lda + k] (row-major A)
template <int NT, int KB, class Epi>
__device__ __forceinline__ void tile_mfma(const float* A, int lda, int nr, const float* Bm, int bsk, int bsn, int N,
                                          int K, float* red, Epi epi) {
  tile_mfma_s<NT, KB>(A, lda, 1, nr, Bm, bsk, bsn, N, K, red, epi);
}

// kWL false (hgin_sb_readout_lds_bytes mode 4: the staged weights would not fit, e.g. hidden 128): the MFMA operands'
// W rows and the head's W are read through the caches instead
template <bool kWL>
__global__ __launch_bounds__(kRoThreadsM) void k_sb_readout_mfma(SbArgs a) {
  extern __shared__ float sm[];
  constexpr int NT = kRoThreadsM;
  __shared__ float red1[NT];
  const int tid = threadIdx.x;
  const int H = a.H;
  const int m = a.m_valid[0];
  constexpr int R = kSbRowsM;
  const int ntile = (m + R - 1) / R;
  const int tile = blockIdx.x;
  if (tile >= ntile) return;   // (the grid is sized for the capacity; uniform per workgroup)
  SB_STAMP(0);
  const int nh = a.nhid;
  const int fp = a.concat_path ? a.fdim[0] : 0;
  const int w0 = H + fp + a.pool_w;
  int win[kSbMaxHid + 1];
  win[0] = w0;
  int maxw = w0;
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    win[i + 1] = i < nh ? a.rw[i] : 0;
    maxw = i < nh && a.rw[i] > maxw ? a.rw[i] : maxw;
  }
  const int KL = a.rw[nh - 1];
  // LDS: the parameters (stage_ro_params) | in0 [R][w0 | 1] | z_i, y_i [R][rw_i | 1] per hidden layer | gbuf x2
  // [R][maxw | 1] | outv [R] | red [4][32][33] (odd row strides everywhere: an MFMA operand read is 32 rows of one
  // column)
  int oW[kSbMaxHid], ldw[kSbMaxHid];
  int off = stage_ro_params<kWL, NT>(a, sm, nh, win, KL, oW, ldw);
  const float* hw = kWL ? (const float*)(sm + off - KL) : a.head_w;
#define RO_WM(i) (kWL ? (const float*)(sm + oW[i]) : a.row_w[i])
  const int l0 = w0 | 1;
  float* in0 = sm + off;
  off += R * l0;
  int oZ[kSbMaxHid], oY[kSbMaxHid], lz[kSbMaxHid];
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    oZ[i] = oY[i] = off;
    lz[i] = 1;
    if (i < nh) {
      lz[i] = a.rw[i] | 1;
      oY[i] = off + R * lz[i];
      off += 2 * R * lz[i];
    }
  }
  const int lg = maxw | 1;
  float* gb0 = sm + off;
  float* gb1 = gb0 + R * lg;
  float* outv = gb1 + R * lg;
  float* red = outv + R;
  const float* xp = a.act + a.act_off[a.L - 1][0];
  const float slope = a.ro_slope[0];
  const float head_b = a.head_b[0];
  const int r0 = tile * R;
  const int nr = m - r0 < R ? m - r0 : R;
  for (int idx = tid; idx < nr * w0; idx += NT) {
    const int rr = idx / w0, k = idx % w0;
    const int64_t row = r0 + rr;
    const float v = readout_input(a, xp, row, k, H, fp);
    in0[rr * l0 + k] = v;
    a.ro_in[0][(int64_t)r0 * w0 + idx] = v;
  }
  __syncthreads();   // the parameters and in0
  SB_STAMP(2);
#pragma unroll
  for (int i = 0; i < kSbMaxHid; ++i) {
    if (i < nh) {
      const float* in = i == 0 ? in0 : sm + oY[i > 0 ? i - 1 : 0];
      const int lin = i == 0 ? l0 : lz[i > 0 ? i - 1 : 0];
      const int N = a.rw[i];
      const float* b = kWL ? (const float*)(sm + oW[i] + N * ldw[i]) : a.row_b[i];
      tile_mfma<NT, kWL ? 4 : 16>(in, lin, nr, RO_WM(i), 1, ldw[i], N, win[i], red, [&](int r, int n, float v) {
        const float z = bn_eval(a, i, n, __fadd_rn(v, b[n]));
        sm[oZ[i] + r * lz[i] + n] = z;
        const float yv = z > 0.0f ? z : __fmul_rn(slope, z);
        sm[oY[i] + r * lz[i] + n] = yv;
        a.ro_in[i + 1][(int64_t)(r0 + r) * N + n] = yv;
      });
      __syncthreads();
      SB_STAMP(3 + i);
    }
  }
  const int lyl = nh == 1 ? lz[0] : (nh == 2 ? lz[1] : lz[2]);
  const float* yl = sm + (nh == 1 ? oY[0] : (nh == 2 ? oY[1] : oY[2]));
  {   // head + loss numerator + seed, split_of() lanes per row
    const int S = split_of<NT>(nr, KL);
    for (int idx = tid; idx < nr * S; idx += NT) {
      const int rr = idx / S, s = idx % S;
      float o = dot_chain(yl + rr * lyl + s, S, hw + s, S, (KL - s + S - 1) / S, 0.0f);
      o = group_sum(o, S);
      if (s == 0) {
        o = __fadd_rn(o, head_b);
        if (a.out_pred) a.out_pred[r0 + rr] = o;
        const float yv = a.y[r0 + rr];
        const float u = __fdiv_rn(__fsub_rn(o, yv), yv);
        red1[rr] = fabsf(u);
        const float sg = u > 0.0f ? 1.0f : (u < 0.0f ? -1.0f : 0.0f);
        const float go = __fdiv_rn(sg, yv);   // d |u| / d out
        outv[rr] = go;
        a.ro_gz[nh][r0 + rr] = go;
      }
    }
  }
  __syncthreads();
  SB_STAMP(6);
  if (tid == 0) {   // fixed-order tile sum of |u| (rows in order)
    float s = 0.0f;
    for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, red1[rr]);
    a.loss_part[tile] = s;
  }
  if (a.eval_only) return;   // (uniform)
  for (int idx = tid; idx < nr * KL; idx += NT) {
    const int rr = idx / KL, k = idx % KL;
    gb0[rr * (KL | 1) + k] = __fmul_rn(outv[rr], hw[k]);
  }
  __syncthreads();
  SB_STAMP(7);
  float slope_part = 0.0f;   // this thread's share of the shared slope's gradient (fixed assignment)
  float* g_y = gb0;
  float* g_next = gb1;
#pragma unroll
  for (int i = kSbMaxHid - 1; i >= 0; --i) {
    if (i < nh) {
      const int K = win[i], N = a.rw[i], ly = N | 1;
      // g_z (in place over g_y) and the slope partial, 4 elements' loads in flight per thread
      for (int i0 = tid; i0 < nr * N; i0 += 4 * NT) {
        float zv[4], gv[4];
        int q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = i0 + u * NT < nr * N ? i0 + u * NT : i0;
          const int rr = idx / N, o = idx - rr * N;
          q[u] = rr * ly + o;
          zv[u] = sm[oZ[i] + rr * lz[i] + o];
          gv[u] = g_y[q[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = i0 + u * NT;
          if (idx < nr * N) {
            if (zv[u] <= 0.0f) slope_part = fmaf(gv[u], zv[u], slope_part);
            const float gz = zv[u] > 0.0f ? gv[u] : __fmul_rn(slope, gv[u]);
            g_y[q[u]] = gz;
            a.ro_gz[i][(int64_t)r0 * N + idx] = gz;
          }
        }
      }
      __syncthreads();
      SB_STAMP(8 + 2 * i);
      // g_in = g_z W (the first layer: only the path embeddings' H columns have a gradient)
      const int KG = i == 0 ? H : K, lgn = KG | 1;
      float* gn = g_next;
      tile_mfma<NT, kWL ? 4 : 16>(g_y, ly, nr, RO_WM(i), ldw[i], 1, KG, N, red,
                [&](int r, int n, float v) { gn[r * lgn + n] = v; });
      __syncthreads();
      SB_STAMP(9 + 2 * i);
      float* t = g_y;
      g_y = g_next;
      g_next = t;
    }
  }
  const float sp = block_sum<NT>(slope_part, red1);
  SB_STAMP(12);
  if (tid == 0) a.slope_part[tile] = sp;
  float* gpath = a.gA + a.g_off[0];
  for (int idx = tid; idx < nr * H; idx += NT) {
    const int rr = idx / H, k = idx % H;
    gpath[(int64_t)r0 * H + idx] = g_y[rr * (H | 1) + k];
  }
  SB_STAMP(13);
}
#undef RO_WM

// ---------------------------------------------------------------------------------------------------------------
// MLP_BN (models.py:303-313, ro_wlds 3): each hidden readout layer is Linear -> BatchNorm1d -> the shared PReLU, and
// the BatchNorm's training-mode statistics span the batch's m valid path rows — a reduction over every tile between
// each layer's GEMM and its activation, forward and backward.  So the readout becomes 2 nhid + 1 launches over the
// same 32-row tiles (tile_mfma for the GEMMs), each closing a layer at the reduction its successor needs:
//   k_sb_bn_fwd(i)  layer i's input (i = 0: the readout input; else PReLU(BN(z_{i-1})) with the statistics merged
//                   from the tiles' partials) -> z_i = W_i in + b_i, and the tile's (mean, M2) partials of z_i;
//   k_sb_bn_head    the last hidden layer's BN + PReLU, the head, the MAPE numerator and seed (as the unfused
//                   readout), g_y = PReLU'(y) (go w_head) and the tile's (sum g_y, sum g_y xhat) partials;
//   k_sb_bn_bwd(i)  g_z = gamma invstd / m (m g_y - sum g_y - xhat sum g_y xhat) (the BatchNorm backward over the
//                   batch), g_in = g_z W_i, then (i > 0) layer i - 1's g_y and partials, or (i = 0) the path
//                   embeddings' gradient.
// Statistics merge in a fixed order (Chan's pairwise (n, mean, M2) update, bn_merge_fwd), every block redoing the
// merge it needs (a few hundred partials: cheaper than a launch); the first block of each records them and
// advances running_mean / running_var (unbiased, the layer's momentum) and num_batches_tracked once per step.  gamma's
// and beta's gradients (sum g_y xhat, sum g_y) go to part_ro's first row chunk (the other chunks stay zero), so
// k_sb_final scales them and folds Adam like every other entry.  Rows past m are never touched.
constexpr int kBnWMax = 20480;   // a layer's W [N][K | 1] (+ b) is staged in LDS up to this many floats, else read via L2
constexpr int kBnRed = (kRoThreadsM / 64) * 32 * 33;   // tile_mfma's k-split partials

// bn_buf blocks of hidden layer i: 0 z [cap_path][N], 1 g_y [cap_path][N], 2 forward partials [tiles][2][N] (mean,
// M2), 3 backward partials [tiles][2][N] (sum g_y, sum g_y xhat), 4 merged statistics [2][N] (mean, invstd)
__device__ __forceinline__ float* bn_ptr(const SbArgs& a, int i, int k) { return a.bn_buf + a.bn_off[i][k]; }

__host__ __device__ __forceinline__ bool bn_wl(int N, int K) { return N * ((K | 1) + 1) <= kBnWMax; }

// layer i's batch mean / invstd into s_mean / s_inv (N floats each) from the tiles' (mean, M2) partials: the
// NT / N thread groups each merge every (NT / N)-th tile in order, then the groups' results merge in group order
// (Chan et al.'s pairwise update: n = na + nb, d = mb - ma, mean = ma + d nb / n, M2 = M2a + M2b + d^2 na nb / n) —
// a handful of loads in flight per thread instead of a few hundred dependent ones per column.  The first block
// records the statistics and advances the running statistics.  red: 3 NT floats.
__device__ __forceinline__ void chan_merge(float& n, float& mu, float& M2, float nb, float mb, float M2b) {
  const float nn = __fadd_rn(n, nb);
  const float d = __fsub_rn(mb, mu);
  const float r = __fdiv_rn(nb, nn);
  mu = __fadd_rn(mu, __fmul_rn(d, r));
  M2 = __fadd_rn(__fadd_rn(M2, M2b), __fmul_rn(__fmul_rn(__fmul_rn(d, d), n), r));
  n = nn;
}
__device__ void bn_merge_fwd(const SbArgs& a, int i, int m, int ntile, float* s_mean, float* s_inv, bool first,
                             float* red) {
  const int N = a.rw[i], NT = blockDim.x, tid = threadIdx.x;
  const int P = NT / N, c = tid % N, p = tid / N;
  const float* pf = bn_ptr(a, i, 2);
  float n = 0.0f, mu = 0.0f, M2 = 0.0f;
  if (p < P) {
#pragma unroll 4
    for (int t = p; t < ntile; t += P) {
      const float nt = (float)(m - t * kSbRowsM < kSbRowsM ? m - t * kSbRowsM : kSbRowsM);
      chan_merge(n, mu, M2, nt, pf[(int64_t)t * 2 * N + c], pf[(int64_t)t * 2 * N + N + c]);
    }
  }
  __syncthreads();
  red[tid] = n;
  red[NT + tid] = mu;
  red[2 * NT + tid] = M2;
  __syncthreads();
  if (tid < N) {
    float gn = 0.0f, gm = 0.0f, g2 = 0.0f;
    for (int q = 0; q < P; ++q)
      if (red[q * N + tid] > 0.0f) chan_merge(gn, gm, g2, red[q * N + tid], red[NT + q * N + tid], red[2 * NT + q * N + tid]);
    const float var = __fdiv_rn(g2, (float)m);
    const float inv = __fdiv_rn(1.0f, sqrtf(__fadd_rn(var, a.bn_eps)));
    s_mean[tid] = gm;
    s_inv[tid] = inv;
    if (first) {
      float* st = bn_ptr(a, i, 4);
      st[tid] = gm;
      st[N + tid] = inv;
    }
    if (first && m > 1) {   // (torch raises on a one-row training batch; here the running statistics stay as they are)
      const float mo = a.bn_mom, keep = __fsub_rn(1.0f, mo);
      const float unb = __fdiv_rn(g2, (float)(m - 1));
      a.bn_rm[i][tid] = __fadd_rn(__fmul_rn(keep, a.bn_rm[i][tid]), __fmul_rn(mo, gm));
      a.bn_rv[i][tid] = __fadd_rn(__fmul_rn(keep, a.bn_rv[i][tid]), __fmul_rn(mo, unb));
    }
  }
  if (first && m > 1 && tid == 0) a.bn_nbt[i][0] += 1;
  __syncthreads();
}

// W_i [N][K] (+ b_i [N] after the rows) into LDS rows of stride K | 1
__device__ void bn_stage_w(const SbArgs& a, int i, int N, int K, float* s_w, bool with_b) {
  const int ld = K | 1;
  for (int idx = threadIdx.x; idx < N * K; idx += blockDim.x) {
    const int o = idx / K;
    s_w[o * ld + idx - o * K] = a.row_w[i][idx];
  }
  if (with_b)
    for (int o = threadIdx.x; o < N; o += blockDim.x) s_w[N * ld + o] = a.row_b[i][o];
}

// LDS floats of each launch (the kernels lay their arrays out in the same order)
__host__ __device__ __forceinline__ int bn_fwd_floats(int N, int K, int Kp) {
  return kSbRowsM * (K | 1) + (bn_wl(N, K) ? N * ((K | 1) + 1) : 0) + kSbRowsM * (N | 1) + kBnRed + 2 * Kp;
}
__host__ __device__ __forceinline__ int bn_head_floats(int N) { return 2 * N + kSbRowsM * (N | 1) + kSbRowsM + 3 * kRoThreadsM; }
__host__ __device__ __forceinline__ int bn_bwd_floats(int N, int K, int KG) {
  return 4 * N + kSbRowsM * (N | 1) + (bn_wl(N, K) ? N * (K | 1) : 0) + kSbRowsM * (KG | 1) + kBnRed + kRoThreadsM;
}

__global__ __launch_bounds__(kRoThreadsM) void k_sb_bn_fwd(SbArgs a, int i) {
  extern __shared__ float sm[];
  constexpr int NT = kRoThreadsM, R = kSbRowsM;
  const int tid = threadIdx.x;
  const int m = a.m_valid[0];
  const int ntile = (m + R - 1) / R;
  const int tile = blockIdx.x;
  if (tile >= ntile) return;
  const int r0 = tile * R, nr = m - r0 < R ? m - r0 : R;
  const int H = a.H, fp = a.concat_path ? a.fdim[0] : 0;
  const int K = i == 0 ? H + fp + a.pool_w : a.rw[i - 1];
  const int N = a.rw[i], lk = K | 1, ln = N | 1;
  const bool wl = bn_wl(N, K);
  float* s_in = sm;                                    // [R][lk]
  float* s_w = s_in + R * lk;                          // [N][lk] + b [N] (wl)
  float* s_z = s_w + (wl ? N * (lk + 1) : 0);          // [R][ln]
  float* red = s_z + R * ln;                           // kBnRed
  float* s_mean = red + kBnRed;                        // [K] (i > 0: layer i - 1's statistics)
  float* s_inv = s_mean + K;
  if (i > 0) bn_merge_fwd(a, i - 1, m, ntile, s_mean, s_inv, tile == 0, red);
  if (wl) bn_stage_w(a, i, N, K, s_w, true);
  __syncthreads();
  float* gin = a.ro_in[i];
  if (i == 0) {
    const float* xp = a.act + a.act_off[a.L - 1][0];
    for (int idx = tid; idx < nr * K; idx += NT) {
      const int rr = idx / K, k = idx - rr * K;
      const float v = readout_input(a, xp, r0 + rr, k, H, fp);
      s_in[rr * lk + k] = v;
      gin[(int64_t)r0 * K + idx] = v;
    }
  } else {
    const float* zp = bn_ptr(a, i - 1, 0);
    const float* ga = a.bn_w[i - 1];
    const float* be = a.bn_b[i - 1];
    const float slope = a.ro_slope[0];
    for (int idx = tid; idx < nr * K; idx += NT) {
      const int rr = idx / K, k = idx - rr * K;
      const float xh = __fmul_rn(__fsub_rn(zp[(int64_t)r0 * K + idx], s_mean[k]), s_inv[k]);
      const float y = __fadd_rn(__fmul_rn(xh, ga[k]), be[k]);
      const float v = y > 0.0f ? y : __fmul_rn(slope, y);
      s_in[rr * lk + k] = v;
      gin[(int64_t)r0 * K + idx] = v;
    }
  }
  __syncthreads();
  const float* Wp = wl ? s_w : a.row_w[i];
  const float* bp = wl ? s_w + N * lk : a.row_b[i];
  float* zg = bn_ptr(a, i, 0);
  tile_mfma<NT>(s_in, lk, nr, Wp, 1, wl ? lk : K, N, K, red, [&](int r, int n, float v) {
    const float z = __fadd_rn(v, bp[n]);
    s_z[r * ln + n] = z;
    zg[(int64_t)(r0 + r) * N + n] = z;
  });
  __syncthreads();
  float* pf = bn_ptr(a, i, 2) + (int64_t)tile * 2 * N;
  for (int c = tid; c < N; c += NT) {   // the tile's (sum, M2) per column, rows in order
    float S = 0.0f;
    for (int r = 0; r < nr; ++r) S = __fadd_rn(S, s_z[r * ln + c]);
    const float mu = __fdiv_rn(S, (float)nr);
    float M2 = 0.0f;
    for (int r = 0; r < nr; ++r) {
      const float d = __fsub_rn(s_z[r * ln + c], mu);
      M2 = fmaf(d, d, M2);
    }
    pf[c] = mu;
    pf[N + c] = M2;
  }
}

// layer i's backward seed from g_a (the gradient of its PReLU output, LDS [nr][lga]): g_y = PReLU'(y) g_a with
// y = gamma xhat + beta recomputed from z_i and the layer's statistics (st: mean [N], invstd [N]), written to bn_g;
// the tile's (sum g_y, sum g_y xhat) partials (the NT / N thread groups take every (NT / N)-th row, then the groups
// add in order; red: 2 NT floats); returns this thread's share of the shared slope's gradient (sum over y <= 0 of
// g_a y)
__device__ float bn_seed_bwd(const SbArgs& a, int i, int tile, int r0, int nr, const float* g_a, int lga,
                             const float* st, float* red) {
  const int N = a.rw[i], NT = blockDim.x, tid = threadIdx.x;
  const int P = NT / N, c = tid % N, p = tid / N;
  const float* zp = bn_ptr(a, i, 0);
  float* gy = bn_ptr(a, i, 1);
  float* pb = bn_ptr(a, i, 3) + (int64_t)tile * 2 * N;
  const float slope = a.ro_slope[0];
  float sp = 0.0f, Sg = 0.0f, Sgx = 0.0f;
  if (p < P) {
    const float mean = st[c], inv = st[N + c], ga = a.bn_w[i][c], be = a.bn_b[i][c];
#pragma unroll 4
    for (int r = p; r < nr; r += P) {
      const int64_t q = (int64_t)(r0 + r) * N + c;
      const float xh = __fmul_rn(__fsub_rn(zp[q], mean), inv);
      const float y = __fadd_rn(__fmul_rn(xh, ga), be);
      const float g = g_a[r * lga + c];
      if (y <= 0.0f) sp = fmaf(g, y, sp);
      const float gyv = y > 0.0f ? g : __fmul_rn(slope, g);
      gy[q] = gyv;
      Sg = __fadd_rn(Sg, gyv);
      Sgx = fmaf(gyv, xh, Sgx);
    }
  }
  __syncthreads();
  red[tid] = Sg;
  red[NT + tid] = Sgx;
  __syncthreads();
  if (tid < N) {
    float g = 0.0f, gx = 0.0f;
    for (int q = 0; q < P; ++q) {
      g = __fadd_rn(g, red[q * N + tid]);
      gx = __fadd_rn(gx, red[NT + q * N + tid]);
    }
    pb[tid] = g;
    pb[N + tid] = gx;
  }
  return sp;
}

__global__ __launch_bounds__(kRoThreadsM) void k_sb_bn_head(SbArgs a) {
  extern __shared__ float sm[];
  constexpr int NT = kRoThreadsM, R = kSbRowsM;
  const int tid = threadIdx.x;
  const int m = a.m_valid[0];
  const int ntile = (m + R - 1) / R;
  const int tile = blockIdx.x;
  if (tile >= ntile) return;
  const int r0 = tile * R, nr = m - r0 < R ? m - r0 : R;
  const int nh = a.nhid, N = a.rw[nh - 1], ln = N | 1;
  float* s_mean = sm;                 // [N]
  float* s_inv = s_mean + N;          // [N]
  float* s_a = s_inv + N;             // [R][ln] the activations, then g_a
  float* s_go = s_a + R * ln;         // [R]
  float* red1 = s_go + R;             // [3 NT] (the merge's, then block_sum's)
  bn_merge_fwd(a, nh - 1, m, ntile, s_mean, s_inv, tile == 0, red1);
  __syncthreads();
  const float* zp = bn_ptr(a, nh - 1, 0);
  const float* ga = a.bn_w[nh - 1];
  const float* be = a.bn_b[nh - 1];
  const float slope = a.ro_slope[0];
  float* gin = a.ro_in[nh];
  for (int idx = tid; idx < nr * N; idx += NT) {
    const int rr = idx / N, k = idx - rr * N;
    const float xh = __fmul_rn(__fsub_rn(zp[(int64_t)r0 * N + idx], s_mean[k]), s_inv[k]);
    const float y = __fadd_rn(__fmul_rn(xh, ga[k]), be[k]);
    const float v = y > 0.0f ? y : __fmul_rn(slope, y);
    s_a[rr * ln + k] = v;
    gin[(int64_t)r0 * N + idx] = v;
  }
  __syncthreads();
  const float* hw = a.head_w;
  const float head_b = a.head_b[0];
  {   // head + loss numerator + seed (as k_sb_readout_mfma)
    const int S = split_of<NT>(nr, N);
    for (int idx = tid; idx < nr * S; idx += NT) {
      const int rr = idx / S, s = idx % S;
      float o = dot_chain(s_a + rr * ln + s, S, hw + s, S, (N - s + S - 1) / S, 0.0f);
      o = group_sum(o, S);
      if (s == 0) {
        o = __fadd_rn(o, head_b);
        const float yv = a.y[r0 + rr];
        const float u = __fdiv_rn(__fsub_rn(o, yv), yv);
        red1[rr] = fabsf(u);
        const float sg = u > 0.0f ? 1.0f : (u < 0.0f ? -1.0f : 0.0f);
        const float go = __fdiv_rn(sg, yv);   // d |u| / d out
        s_go[rr] = go;
        a.ro_gz[nh][r0 + rr] = go;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.0f;
    for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, red1[rr]);
    a.loss_part[tile] = s;
  }
  for (int idx = tid; idx < nr * N; idx += NT) {
    const int rr = idx / N, k = idx - rr * N;
    s_a[rr * ln + k] = __fmul_rn(s_go[rr], hw[k]);
  }
  __syncthreads();
  // (the statistics from LDS: the global record is this launch's first block's)
  const float sp = block_sum<NT>(bn_seed_bwd(a, nh - 1, tile, r0, nr, s_a, ln, s_mean, red1), red1);
  if (tid == 0) a.slope_part[tile] = sp;
}

__global__ __launch_bounds__(kRoThreadsM) void k_sb_bn_bwd(SbArgs a, int i) {
  extern __shared__ float sm[];
  constexpr int NT = kRoThreadsM, R = kSbRowsM;
  const int tid = threadIdx.x;
  const int m = a.m_valid[0];
  const int ntile = (m + R - 1) / R;
  const int tile = blockIdx.x;
  if (tile >= ntile) return;
  const int r0 = tile * R, nr = m - r0 < R ? m - r0 : R;
  const int H = a.H, fp = a.concat_path ? a.fdim[0] : 0;
  const int K = i == 0 ? H + fp + a.pool_w : a.rw[i - 1];
  const int KG = i == 0 ? H : K;   // (the first layer: only the path embeddings' columns have a gradient)
  const int N = a.rw[i], ln = N | 1, lk = K | 1, lg = KG | 1;
  const bool wl = bn_wl(N, K);
  float* s_c = sm;                    // [4][N]: mean, invstd, sum g_y, sum g_y xhat
  float* s_gz = s_c + 4 * N;          // [R][ln]
  float* s_w = s_gz + R * ln;         // [N][lk] (wl)
  float* s_gi = s_w + (wl ? N * lk : 0);   // [R][lg]
  float* red = s_gi + R * lg;         // kBnRed
  float* red1 = red + kBnRed;         // [NT]
  const float* pb = bn_ptr(a, i, 3);
  const float* st = bn_ptr(a, i, 4);
  float* part = a.part_ro - a.p_gin + a.bn_goff[i];   // the first row chunk's gamma, beta entries
  {   // the tiles' (sum g_y, sum g_y xhat): NT / N thread groups over every (NT / N)-th tile, then the groups in order
    const int P = NT / N, c = tid % N, p = tid / N;
    float Sg = 0.0f, Sgx = 0.0f;
    if (p < P) {
#pragma unroll 4
      for (int t = p; t < ntile; t += P) {
        Sg = __fadd_rn(Sg, pb[(int64_t)t * 2 * N + c]);
        Sgx = __fadd_rn(Sgx, pb[(int64_t)t * 2 * N + N + c]);
      }
    }
    red[tid] = Sg;
    red[NT + tid] = Sgx;
    __syncthreads();
    if (tid < N) {
      float g = 0.0f, gx = 0.0f;
      for (int q = 0; q < P; ++q) {
        g = __fadd_rn(g, red[q * N + tid]);
        gx = __fadd_rn(gx, red[NT + q * N + tid]);
      }
      s_c[tid] = st[tid];
      s_c[N + tid] = st[N + tid];
      s_c[2 * N + tid] = g;
      s_c[3 * N + tid] = gx;
      if (tile == 0) {
        part[tid] = gx;      // d gamma
        part[N + tid] = g;   // d beta
      }
    }
  }
  if (wl) bn_stage_w(a, i, N, K, s_w, false);
  __syncthreads();
  const float* zp = bn_ptr(a, i, 0);
  const float* gy = bn_ptr(a, i, 1);
  const float fm = (float)m;
  for (int idx = tid; idx < nr * N; idx += NT) {
    const int rr = idx / N, c = idx - rr * N;
    const int64_t q = (int64_t)r0 * N + idx;
    const float xh = __fmul_rn(__fsub_rn(zp[q], s_c[c]), s_c[N + c]);
    const float coef = __fdiv_rn(__fmul_rn(a.bn_w[i][c], s_c[N + c]), fm);
    const float t = __fsub_rn(__fsub_rn(__fmul_rn(fm, gy[q]), s_c[2 * N + c]), __fmul_rn(xh, s_c[3 * N + c]));
    const float gz = __fmul_rn(coef, t);
    s_gz[rr * ln + c] = gz;
    a.ro_gz[i][q] = gz;
  }
  __syncthreads();
  const float* Wp = wl ? s_w : a.row_w[i];
  tile_mfma<NT>(s_gz, ln, nr, Wp, wl ? lk : K, 1, KG, N, red,
                [&](int r, int n, float v) { s_gi[r * lg + n] = v; });
  __syncthreads();
  if (i == 0) {
    float* gpath = a.gA + a.g_off[0];
    for (int idx = tid; idx < nr * H; idx += NT) {
      const int rr = idx / H, k = idx - rr * H;
      gpath[(int64_t)r0 * H + idx] = s_gi[rr * lg + k];
    }
    return;
  }
  const float sp = block_sum<NT>(bn_seed_bwd(a, i - 1, tile, r0, nr, s_gi, lg, bn_ptr(a, i - 1, 4), red), red1);
  if (tid == 0) a.slope_part[tile] = __fadd_rn(a.slope_part[tile], sp);
}

// the readout blocks of k_sb_bwd_w: over row chunk p of the m valid path rows, one group of layer i's (i = nhid: the
// head's) partial weight / bias gradients, g_W[o][k] = sum_rows g_z[o] in[k], g_b[o] = sum_rows g_z[o] (the bias as
// an input column of ones: fmaf(g, 1, v) is the add), the chunk's rows in order (staged as many rows at a time as
// the staging array holds: the whole chunk at cfg1 sizes).  A group is ro_to(N) x (kSbThreads / ro_to(N)) threads,
// each an MO x MK register tile of (o, k) entries strided by the thread grid (lanes read consecutive o: conflict-free;
// 6 LDS reads per 8 products, not 16).  Block y-index u (after the relations' kRel) -> (layer, group): the layers'
// groups in order.
constexpr int kRoMO = 4, kRoMK = 2;
constexpr int kSbStage = 8192;   // k_sb_bwd_w's staging floats (32 KiB: 16 rows of the widest readout layer)

__host__ __device__ __forceinline__ int ro_to(int N) {
  int t = 1;
  while (t < kSbThreads && kRoMO * t < N) t *= 2;
  return t;
}
__host__ __device__ __forceinline__ int ro_groups_nk(int N, int K) {
  const int tk = kSbThreads / ro_to(N);
  return (K + 1 + kRoMK * tk - 1) / (kRoMK * tk);
}
__device__ __forceinline__ int ro_in_width(const SbArgs& a, int i) {
  return i == 0 ? a.H + (a.concat_path ? a.fdim[0] : 0) + a.pool_w : a.rw[i - 1];
}
__device__ __forceinline__ int ro_groups(const SbArgs& a, int i) {
  return ro_groups_nk(i < a.nhid ? a.rw[i] : 1, ro_in_width(a, i));
}

// one thread's register tile of a weight-gradient group: entries (oj[j], kj[jk]) of g_W's [N][K + 1] (column K: the
// bias), strided by the group's TO x TK thread grid; the indices are clamped (read, never stored) past N / K + 1
struct WgTile {
  int to, tk, TO, TK, kc0;
  int oj[kRoMO], kj[kRoMK];
  float acc[kRoMO][kRoMK];
};
__device__ __forceinline__ void wg_setup(WgTile& t, int N, int K1, int u) {
  t.TO = ro_to(N);
  t.TK = kSbThreads / t.TO;
  t.to = threadIdx.x % t.TO;
  t.tk = threadIdx.x / t.TO;
  t.kc0 = u * kRoMK * t.TK;
#pragma unroll
  for (int j = 0; j < kRoMO; ++j) t.oj[j] = t.to + t.TO * j < N ? t.to + t.TO * j : N - 1;
#pragma unroll
  for (int j = 0; j < kRoMK; ++j) t.kj[j] = t.kc0 + t.tk + t.TK * j < K1 ? t.kc0 + t.tk + t.TK * j : K1 - 1;
#pragma unroll
  for (int j = 0; j < kRoMO; ++j)
#pragma unroll
    for (int jk = 0; jk < kRoMK; ++jk) t.acc[j][jk] = 0.0f;
}
// acc += sum over the nr staged rows (in order) of s_g[rr][o] s_in[rr][k] (s_g [nr][N], s_in [nr][K] as copied from
// HBM; column K, the bias's, reads as ones: fmaf(g, 1, v) is the add)
__device__ __forceinline__ void wg_accum(WgTile& t, const float* s_g, const float* s_in, int nr, int N, int K) {
#pragma unroll 4
  for (int rr = 0; rr < nr; ++rr) {
    float g[kRoMO], x[kRoMK];
#pragma unroll
    for (int j = 0; j < kRoMO; ++j) g[j] = s_g[rr * N + t.oj[j]];
#pragma unroll
    for (int j = 0; j < kRoMK; ++j) {
      const float v = s_in[rr * K + (t.kj[j] < K ? t.kj[j] : 0)];
      x[j] = t.kj[j] < K ? v : 1.0f;
    }
#pragma unroll
    for (int j = 0; j < kRoMO; ++j)
#pragma unroll
      for (int jk = 0; jk < kRoMK; ++jk) t.acc[j][jk] = fmaf(g[j], x[jk], t.acc[j][jk]);
  }
}
// the tile's entries into part (W [N][K] row-major, then b [N])
__device__ __forceinline__ void wg_store(const WgTile& t, float* part, int N, int K) {
#pragma unroll
  for (int j = 0; j < kRoMO; ++j) {
#pragma unroll
    for (int jk = 0; jk < kRoMK; ++jk) {
      const int o = t.to + t.TO * j, k = t.kc0 + t.tk + t.TK * jk;
      if (o < N && k <= K) part[k < K ? (int64_t)o * K + k : (int64_t)N * K + o] = t.acc[j][jk];
    }
  }
}

__device__ void ro_weight_part(const SbArgs& a, int p, int u, float* stage) {
  int i = 0;
  while (i < a.nhid && u >= ro_groups(a, i)) u -= ro_groups(a, i++);
  const int tid = threadIdx.x;
  const int m = a.m_valid[0];
  const int ch = (m + a.n_parts - 1) / a.n_parts;
  const int i0 = p * ch < m ? p * ch : m, i1 = (p + 1) * ch < m ? (p + 1) * ch : m;
  const int K = ro_in_width(a, i), K1 = K + 1;
  const int N = i < a.nhid ? a.rw[i] : 1;
  const float* in = a.ro_in[i];
  const float* gz = a.ro_gz[i];
  // indexed by the flat readout offsets
  float* part = a.part_ro + (int64_t)p * a.p_ro - a.p_gin + (i < a.nhid ? a.ro_goff[i] : a.head_goff);
  WgTile t;
  wg_setup(t, N, K1, u);
  // the chunk's rows RS at a time (all of them at cfg1 sizes: one memory round trip), both images contiguous copies
  const int rcap = kSbStage / (N + K);
  const int RS = (i1 - i0) < rcap ? (i1 - i0 > 0 ? i1 - i0 : 1) : rcap;
  float* s_g = stage;
  float* s_in = stage + RS * N;
  for (int rb = i0; rb < i1; rb += RS) {
    const int nr = i1 - rb < RS ? i1 - rb : RS;
    __syncthreads();
    copy_flat<16>(s_in, in + (int64_t)rb * K, nr * K);
    copy_flat<8>(s_g, gz + (int64_t)rb * N, nr * N);
    __syncthreads();
    wg_accum(t, s_g, s_in, nr, N, K);
  }
  wg_store(t, part, N, K);
}

// layer l's output gradient of type d (gcur: written by the readout for path rows, by k_sb_bwd_in of layer l + 1
// otherwise); the last layer's link / node outputs feed nothing (models.py:362-376 reads path only)
__device__ __forceinline__ float gout(const SbArgs& a, const float* gcur, int l, int d, int64_t q) {
  if (l == a.L - 1 && d != 0) return 0.0f;
  const float g = gcur[a.g_off[d] + q];
  return a.drop_thr ? __fmul_rn(g, drop_factor(a, l, d, q)) : g;   // (through the dropout of the layer's output)
}

// one row chunk's partial W / bias / slope / eps gradients of one relation (grid = n_parts x relations, plus half
// the readout layers' blocks in the last layer's launch and half in the first's); rows of chunk p: [p c, (p + 1) c),
// c = ceil(rows / n_parts)
// kM (hidden >= 64): g_comb = g_z W and the W partial g_z^T comb on the matrix cores (tile_mfma over the staged rows;
// the scalar register tiles at H = 128 re-staged the rows for 8 groups), the chunk's rows staged at once
constexpr int kSbStageM = 16384, kSbRedM = (kSbThreads / 64) * 32 * 33;
template <bool kM>
__global__ __launch_bounds__(kSbThreads, kM ? 1 : 4) void k_sb_bwd_w(SbArgs a, int l, const float* gcur,
                                                                     int ro_first) {
  __shared__ float red[2 * kSbThreads];   // (block_sum2)
  __shared__ float stage[kM ? kSbStageM : kSbStage];
  const int p = blockIdx.x, r = blockIdx.y;
  SB_STAMP_W(l & 1, 0);
  if (r >= kRel) {   // the readout's blocks: groups ro_first, ... (grid.y = kRel + their count)
    ro_weight_part(a, p, r - kRel + ro_first, stage);
    SB_STAMP_W(l & 1, 1);
    return;
  }
  const int s = kRelSrc[r], d = kRelDst[r];
  const int H = a.H, K = kdim(a, l, r);
  const int tid = threadIdx.x;
  const int rows = nrows(a, d);
  const int ch = (rows + a.n_parts - 1) / a.n_parts;
  const int i0 = p * ch < rows ? p * ch : rows, i1 = (p + 1) * ch < rows ? (p + 1) * ch : rows;
  const SbConv& cv = a.conv[l][r];
  float* part = a.part_gin + (int64_t)p * a.p_gin + cv.goff;
  const float* comb = a.comb + a.comb_off[l][r];
  const float* zb = a.zb + a.zb_off[l][r];
  float* gc = a.gc + a.gc_off[r];
  const float slope = cv.slope[0];
  const int fs = l == 0 ? a.fdim[s] : 0;
  const int K1 = K + 1;
  if constexpr (kM) {
    const int lg = H | 1, lk = K | 1;
    const int rcap = (kSbStageM - kSbRedM) / (lg + lk);
    const int RS = (i1 - i0) < rcap ? (i1 - i0 > 0 ? i1 - i0 : 1) : rcap;
    float* s_g = stage;               // [RS][lg] g_z
    float* s_in = s_g + RS * lg;      // [RS][lk] comb
    float* redm = s_in + RS * lk;     // tile_mfma's split partials
    float sp = 0.0f, epv = 0.0f, bsum = 0.0f;
    for (int rb = i0; rb < i1; rb += RS) {
      const int nr = i1 - rb < RS ? i1 - rb : RS;
      __syncthreads();
      for (int idx = tid; idx < nr * K; idx += kSbThreads) {
        const int rr = idx / K;
        s_in[rr * lk + idx - rr * K] = comb[(int64_t)rb * K + idx];
      }
#pragma unroll 4
      for (int idx = tid; idx < nr * H; idx += kSbThreads) {
        const int64_t qq = (int64_t)rb * H + idx;
        const float z = zb[qq], g = gout(a, gcur, l, d, qq);
        const int rr = idx / H;
        s_g[rr * lg + idx - rr * H] = z > 0.0f ? g : __fmul_rn(slope, g);
        if (z <= 0.0f) sp = fmaf(g, z, sp);
      }
      __syncthreads();
      if (tid < H)   // the bias partial: the rows in order
        for (int rr = 0; rr < nr; ++rr) bsum = __fadd_rn(bsum, s_g[rr * lg + tid]);
      for (int sb = 0; sb < nr; sb += 32) {   // g_comb rows (row-local: k_sb_bwd_in reads them after this launch)
        const int ns = nr - sb < 32 ? nr - sb : 32;
        tile_mfma<kSbThreads, 16>(s_g + sb * lg, lg, ns, cv.w, K, 1, K, H, redm, [&](int r, int k, float v) {
          const int i = rb + sb + r;
          gc[(int64_t)i * a.kmax + k] = v;
          if (k >= fs) {
            const float xv = l == 0 ? a.x[d][(int64_t)i * a.ldx[d] + a.cols[d][k - fs]]
                                    : a.act[a.act_off[l - 1][d] + (int64_t)i * H + k];
            epv = fmaf(v, xv, epv);
          }
        });
      }
      for (int h0 = 0; h0 < H; h0 += 32) {   // W partial [h][k] += sum over the staged rows of g_z[h] comb[k]
        const int nh = H - h0 < 32 ? H - h0 : 32;
        tile_mfma_s<kSbThreads>(s_g + h0, 1, lg, nh, s_in, lk, 1, K, nr, redm, [&](int r, int k, float v) {
          float* e = part + (int64_t)(h0 + r) * K + k;
          *e = rb == i0 ? v : __fadd_rn(*e, v);
        });
      }
    }
    if (i1 <= i0) {   // an empty chunk: zero partials
      for (int e = tid; e < H * K; e += kSbThreads) part[e] = 0.0f;
    }
    if (tid < H) part[(int64_t)H * K + tid] = bsum;
    const float2 se = block_sum2(sp, epv, red);
    if (tid == 0) {
      part[(int64_t)H * K + H] = se.x;
      part[(int64_t)H * K + H + 1] = se.y;
    }
    return;
  }
  // the chunk's rows RS at a time in LDS (all of them at cfg1 sizes): g_z = PReLU'(z) g_y into s_g, comb with a
  // column of ones into s_in; then g_comb = g_z W (row-local; k_sb_bwd_in reads every row's g_comb after this launch)
  // with the eps partial (g_comb over the self columns times x_dst), and the register-tiled W / bias partials
  // (wg_accum, the rows in order).  The slope partial: sum over z <= 0 of g_y z.  A group beyond the first (H (K + 1)
  // above kRoMO x kRoMK x kSbThreads entries) stages the rows again.
  // W [H][K] in LDS too when small (the g_comb dots read a column of it per output)
  const int wsz = H * K <= 2048 ? H * K : 0;
  const int rcap = (kSbStage - wsz) / (H + K);
  const int RS = (i1 - i0) < rcap ? (i1 - i0 > 0 ? i1 - i0 : 1) : rcap;
  float* s_w = stage;
  float* s_g = stage + wsz;
  float* s_in = s_g + RS * H;
  if (wsz) copy_flat<8>(s_w, cv.w, wsz);   // (visible after the first row block's barrier)
  float sp = 0.0f, epv = 0.0f;
  const int ng = ro_groups_nk(H, K);
  for (int u = 0; u < ng; ++u) {
    WgTile t;
    wg_setup(t, H, K1, u);
    for (int rb = i0; rb < i1; rb += RS) {
      const int nr = i1 - rb < RS ? i1 - rb : RS;
      __syncthreads();
      copy_flat<16>(s_in, comb + (int64_t)rb * K, nr * K);
#pragma unroll 4
      for (int idx = tid; idx < nr * H; idx += kSbThreads) {
        const int64_t qq = (int64_t)rb * H + idx;
        const float z = zb[qq], g = gout(a, gcur, l, d, qq);
        s_g[idx] = z > 0.0f ? g : __fmul_rn(slope, g);
        if (u == 0 && z <= 0.0f) sp = fmaf(g, z, sp);
      }
      __syncthreads();
      if (u == 0) {
        for (int idx = tid; idx < nr * K; idx += kSbThreads) {
          const int rr = idx / K, k = idx % K;
          const int i = rb + rr;
          const float v = wsz ? dot_chain(s_g + rr * H, 1, s_w + k, K, H, 0.0f)
                              : dot_chain(s_g + rr * H, 1, cv.w + k, K, H, 0.0f);
          gc[(int64_t)i * a.kmax + k] = v;
          if (k >= fs) {
            const float xv = l == 0 ? a.x[d][(int64_t)i * a.ldx[d] + a.cols[d][k - fs]]
                                    : a.act[a.act_off[l - 1][d] + (int64_t)i * H + k];
            epv = fmaf(v, xv, epv);
          }
        }
      }
      wg_accum(t, s_g, s_in, nr, H, K);
    }
    wg_store(t, part, H, K);
  }
  const float2 se = block_sum2(sp, epv, red);
  const float ssum = se.x, esum = se.y;
  if (tid == 0) {
    part[(int64_t)H * K + H] = ssum;
    part[(int64_t)H * K + H + 1] = esum;
  }
  SB_STAMP_W(l & 1, 1);
}

// the gradient of layer l's input of type t (l > 0: layer l - 1's output): per relation in order, the self term
// (1 + eps) g_comb where t is the destination (add mode: every column) and the CSC aggregate of g_comb where t is
// the source (edge order).  grid.y = node type
__global__ __launch_bounds__(kSbThreads) void k_sb_bwd_in(SbArgs a, int l, float* gnxt) {
  const int t = blockIdx.y;
  const int H = a.H;
  const int64_t idx = (int64_t)blockIdx.x * kSbThreads + threadIdx.x;
  if (idx >= (int64_t)nrows(a, t) * H) return;
  const int u = (int)(idx / H), k = (int)(idx % H);
  float v = 0.0f;
  for (int r = 0; r < kRel; ++r) {
    const float* gc = a.gc + a.gc_off[r];
    if (kRelDst[r] == t)
      v = __fadd_rn(v, __fmul_rn(__fadd_rn(1.0f, a.conv[l][r].eps[0]), gc[(int64_t)u * a.kmax + k]));
    if (kRelSrc[r] == t) {
      const int32_t* cp = a.cptr[r];
      const int32_t* cd = a.cdst[r];
      v = gather_chain(cd, cp[u], cp[u + 1], gc, a.kmax, k, v);
    }
  }
  gnxt[a.g_off[t] + (int64_t)u * H + k] = v;
}

// every gradient entry = its n_parts partials in a fixed order (thread (j, g) of a 32-entry group sums parts g, g + 8,
// ...; then the 8 group sums in order), times the sqrt-MAPE scale; the loss and the shared readout slope from the
// per-tile partials (thread t sums tiles t, t + 256, ..., then a tree); every block recomputes the scale
// Adam (torch.optim.Adam's rule, amsgrad / maximize off; L2 weight decay folded into the gradient) on entry e, in
// fp32: m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
struct AdamCoef {
  float step_size, bc2_sqrt;
};
__device__ __forceinline__ void adam_update(const SbArgs& a, int64_t e, float gv, const AdamCoef& c) {
  float p = a.pflat[e];
  const float gd = a.weight_decay != 0.0f ? __fadd_rn(gv, __fmul_rn(a.weight_decay, p)) : gv;
  const float m = __fadd_rn(__fmul_rn(a.beta1, a.mflat[e]), __fmul_rn(__fsub_rn(1.0f, a.beta1), gd));
  const float v = __fadd_rn(__fmul_rn(a.beta2, a.vflat[e]), __fmul_rn(__fmul_rn(__fsub_rn(1.0f, a.beta2), gd), gd));
  const float den = __fadd_rn(__fdiv_rn(sqrtf(v), c.bc2_sqrt), a.adam_eps);
  p = __fsub_rn(p, __fmul_rn(c.step_size, __fdiv_rn(m, den)));
  a.mflat[e] = m;
  a.vflat[e] = v;
  a.pflat[e] = p;
}

// entry e (< p_gin) belongs to a conv that cannot reach the readout (its parameter block [goff, goff + size))
// (the convs' gradient blocks are contiguous in (layer, relation) order: the owner is the last conv starting at or
// before e)
__device__ __forceinline__ bool entry_dead(const SbArgs& a, int64_t e) {
  for (int l = a.L - 1; l >= 0; --l)
    for (int r = kRel - 1; r >= 0; --r)
      if (e >= a.conv[l][r].goff) return (a.dead_conv >> (4 * l + r)) & 1u;
  return false;
}

__global__ __launch_bounds__(kSbThreads) void k_sb_final(SbArgs a) {
  __shared__ float red[2 * kSbThreads];   // (block_sum2)
  const int tid = threadIdx.x;
  AdamCoef ad{0.0f, 1.0f};
  if (a.adam_step) {
    const float st = a.adam_step[0];
    ad.step_size = __fdiv_rn(a.lr, __fsub_rn(1.0f, powf(a.beta1, st)));
    ad.bc2_sqrt = sqrtf(__fsub_rn(1.0f, powf(a.beta2, st)));
  }
  const int m = a.m_valid[0];
  const int rows = a.ro_wlds >= 2 ? kSbRowsM : kSbRows;   // the readout tiles' rows (one loss / slope partial each)
  const int ntile = (m + rows - 1) / rows;
  float lp = 0.0f, sp = 0.0f;
  for (int t = tid; t < ntile; t += kSbThreads) {
    lp = __fadd_rn(lp, a.loss_part[t]);
    sp = __fadd_rn(sp, a.slope_part[t]);
  }
  const float2 ls = block_sum2(lp, sp, red);
  const float s = ls.x, slope_sum = ls.y;
  const float lv = __fdiv_rn(__fmul_rn(100.0f, s), (float)m);       // 100 * mean |u| (train.py:12-13)
  const float scale = __fdiv_rn(__fdiv_rn(100.0f, (float)m), __fmul_rn(2.0f, sqrtf(lv)));
  if (blockIdx.x == 0 && tid == 0) {
    a.loss_value[0] = lv;
    if (a.drop_thr) a.drop_ctr[0] += 1;   // (no kernel of this step reads it after this one starts)
    if (a.eval_only) {
      a.loss_acc[0] = __fadd_rn(a.loss_acc[0], lv);
      a.loss_acc[1] = __fadd_rn(a.loss_acc[1], __fmul_rn(lv, (float)m));
    }
  }
  if (a.eval_only) return;
  const int64_t P = a.p_gin + a.p_ro;
  const int j = tid & 31, g = tid >> 5;
  for (int64_t e0 = (int64_t)blockIdx.x * 32; e0 < P; e0 += (int64_t)gridDim.x * 32) {
    const int64_t e = e0 + j;
    float v = 0.0f;
    const int np = (a.n_parts - g + 7) / 8;   // parts g, g + 8, ...
    if (e < a.p_gin) {
      v = sum_chain(a.part_gin + (int64_t)g * a.p_gin + e, 8 * a.p_gin, np, v);
    } else if (e < P && e != a.ro_slope_goff) {
      v = sum_chain(a.part_ro + (int64_t)g * a.p_ro + (e - a.p_gin), 8 * a.p_ro, np, v);
    }
    red[tid] = v;
    __syncthreads();
    if (g == 0 && e < P) {
      float t = 0.0f;
      for (int q = 0; q < 8; ++q) t = __fadd_rn(t, red[q * 32 + j]);
      const float gv = __fmul_rn(e == a.ro_slope_goff ? slope_sum : t, scale);
      a.gflat[e] = gv;
      if (a.adam_step && !(a.dead_conv && e < a.p_gin && entry_dead(a, e))) adam_update(a, e, gv, ad);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
// HetroGAT in the fused step (models.py:380-506; config.json MODEL "GAT": HEADS 16, NODE_EMBEDDING_SIZE 8, MP_LAYERS 1
// — the reference's HetroGAT runs one layer when heads > 1).  A GATConv (PyG 2.0.2) of relation (s -> d) on the raw
// (sliced) features x: x_s' = x_s W_s^T, x_d' = x_d W_d^T [HC = heads x C]; per head h the logits
// e_ji = leaky_relu(a_s[j] + a_d[i]) with a_s[j] = x_s'[j, h, :] . att_s[h], a_d[i] = x_d'[i, h, :] . att_d[h], over the
// edges into i after GATConv's self-loop handling (edges with src id == dst id removed, (i, i) appended for
// i < min(N_s, N_d), bipartite relations included), softmax over them, out_i = sum_j alpha_ji x_s'[j] + bias; the
// relations into a type summed in relation order (HeteroConv aggr 'sum').
// The projections are linear, so they are folded: a_s[j] = x_s[j] . v_s[h] with v_s[h] = W_s[h]^T att_s[h] (K_src
// values), and out_i[h] = W_s[h] u_i[h] + bias[h] with u_i[h] = sum_j alpha_ji x_s[j] (the softmax-weighted sum of the
// K_src-wide raw rows): per edge and head K_src multiply-adds instead of C, no x_s' table.  The same sums in another
// association than the reference's (fp32 tolerance, tests/test_gpu_smallbatch.py).
// Backward (a linear chain in the seed g = d sum|u| / d out_i, which the readout leaves in gA):
//   q_i[h] = W_s[h]^T g_i[h];  per edge g_alpha = x_s[j] . q_i[h];  S_i = sum_j alpha g_alpha;
//   g_pre = alpha (g_alpha - S_i) leaky'(pre);  r[h] += g_pre x_s[j];  t[h] += (sum_j g_pre) x_d[i];
//   g_W_s[h] = sum_i g_i[h] u_i[h]^T + att_s[h] r[h]^T,  g_att_s[h] = W_s[h] r[h],  g_bias = sum_i g_i,
//   g_W_d[h] = att_d[h] t[h]^T,  g_att_d[h] = W_d[h] t[h]
// — row-local sums, so no source-side (CSC) pass: the sources are the raw features, which need no gradient.
constexpr int kGatK = 8;   // raw (sliced) feature columns per type (the host checks)

// thread (row slot, head): rows of type t handled per workgroup pass
__device__ __forceinline__ int gat_rows_per_pass(const SbArgs& a) { return kSbThreads / a.gat_heads; }

__device__ __forceinline__ void gat_row(const SbArgs& a, int t, int64_t i, float (&x)[kGatK]) {
  const int K = a.fdim[t];
#pragma unroll
  for (int k = 0; k < kGatK; ++k) x[k] = k < K ? a.x[t][i * a.ldx[t] + a.cols[t][k]] : 0.0f;
}

// One relation's folded attention vectors and source projection staged in LDS by the whole block (round 6: every
// thread used to form its head's v_s / v_d from C x K global loads of W and att, and read W_s again for its output —
// ~300 dependent-latency loads per thread; now each thread makes at most a few of the NH x K folds, in the
// per-thread fold's c order, so the values are the same bits).  sws [HC][fs] (W_s rows), svs [NH][kGatK], svd [NH][kGatK], sb [HC] (or
// NULL: the bias is not needed).
template <int C>
__device__ __forceinline__ void gat_stage(const SbArgs& a, const SbGat& g, int fs, int fd, float* sws, float* svs,
                                          float* svd, float* sb) {
  const int NH = a.gat_heads, HC = NH * C;
  for (int idx = threadIdx.x; idx < HC * fs; idx += kSbThreads) sws[idx] = g.ws[idx];
  if (sb)
    for (int idx = threadIdx.x; idx < HC; idx += kSbThreads) sb[idx] = g.b[idx];
  for (int idx = threadIdx.x; idx < 2 * NH * kGatK; idx += kSbThreads) {
    const bool dst = idx >= NH * kGatK;
    const int j = dst ? idx - NH * kGatK : idx, h = j / kGatK, k = j - h * kGatK;
    const int K = dst ? fd : fs;
    const float* w = dst ? g.wd : g.ws;
    const float* att = dst ? g.att_d : g.att_s;
    float v = 0.0f;
    if (k < K) {
#pragma unroll
      for (int c = 0; c < C; ++c) v = fmaf(att[h * C + c], w[(int64_t)(h * C + c) * K + k], v);
    }
    (dst ? svd : svs)[j] = v;
  }
}

// the edges into row i of relation r after GATConv's self-loop handling, in the adjusted list's order (CSR edge order
// without the j == i edges, then the appended loop)
template <class F>
__device__ __forceinline__ void gat_edges(const SbArgs& a, int r, int i, int n_src, int n_dst, F f) {
  const int32_t* cl = a.col[r];
  const int e1 = a.rowptr[r][i + 1];
  for (int e = a.rowptr[r][i]; e < e1; ++e) {
    const int j = cl[e];
    if (j != i) f(j);
  }
  if (i < (n_src < n_dst ? n_src : n_dst)) f(i);
}

template <int C>
__global__ __launch_bounds__(kSbThreads) void k_sb_gat_fwd(SbArgs a) {
  __shared__ float red[2 * kSbThreads];
  __shared__ float sws[128 * kGatK], svs[32 * kGatK], svd[32 * kGatK], sb[128];
  const int t = blockIdx.y;
  if (t == 3) {   // GLOBAL_FEATS
    sb_pool(a, red);
    return;
  }
  const int tid = threadIdx.x;
  if (a.adam_step && blockIdx.x == 0 && t == 0 && tid == 0) a.adam_step[0] += 1.0f;   // read by k_sb_final
  const int NH = a.gat_heads, HC = NH * C, RS = gat_rows_per_pass(a);
  const int slot = tid / NH, h = tid - slot * NH;
  const int n = nrows(a, t);
  const int i = blockIdx.x * RS + slot;
  if (blockIdx.x * RS >= n) return;                 // (block-uniform: the staging below needs every thread)
  const bool act = slot < RS && i < n;
  const int fd = a.fdim[t];
  float xi[kGatK];
  if (act) gat_row(a, t, i, xi);
  float y[C];
  bool first = true;
  for (int r = 0; r < kRel; ++r) {
    if (kRelDst[r] != t) continue;
    const int s = kRelSrc[r], fs = a.fdim[s];
    const SbGat& g = a.gatc[r];
    __syncthreads();                                // (the previous relation's reads of the staged values)
    gat_stage<C>(a, g, fs, fd, sws, svs, svd, sb);
    __syncthreads();
    if (!act) continue;
    float vs[kGatK], vd[kGatK];
#pragma unroll
    for (int k = 0; k < kGatK; ++k) {
      vs[k] = svs[h * kGatK + k];
      vd[k] = svd[h * kGatK + k];
    }
    float ad = 0.0f;
#pragma unroll
    for (int k = 0; k < kGatK; ++k) ad = fmaf(vd[k], xi[k], ad);
    float m = -INFINITY, ssum = 0.0f, u[kGatK];
#pragma unroll
    for (int k = 0; k < kGatK; ++k) u[k] = 0.0f;
    gat_edges(a, r, i, nrows(a, s), n, [&](int j) {
      float xj[kGatK];
      gat_row(a, s, j, xj);
      float as = 0.0f;
#pragma unroll
      for (int k = 0; k < kGatK; ++k) as = fmaf(vs[k], xj[k], as);
      float ev = __fadd_rn(as, ad);
      ev = ev > 0.0f ? ev : __fmul_rn(a.gat_slope, ev);
      if (ev > m) {   // online softmax: rescale the running sums to the new maximum
        const float sc = expf(m - ev);
        ssum = fmaf(ssum, sc, 1.0f);
#pragma unroll
        for (int k = 0; k < kGatK; ++k) u[k] = fmaf(u[k], sc, xj[k]);
        m = ev;
      } else {
        const float w = expf(ev - m);
        ssum = __fadd_rn(ssum, w);
#pragma unroll
        for (int k = 0; k < kGatK; ++k) u[k] = fmaf(w, xj[k], u[k]);
      }
    });
    const float den = __fadd_rn(ssum, 1e-16f);   // PyG softmax: / (sum + 1e-16)
    float* st = a.gat_st + a.gat_st_off[r] + ((int64_t)i * NH + h) * (2 + fs);
    st[0] = m;
    st[1] = den;
#pragma unroll
    for (int k = 0; k < kGatK; ++k) {
      u[k] = ssum > 0.0f ? __fdiv_rn(u[k], den) : 0.0f;
      if (k < fs) st[2 + k] = u[k];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* wr = sws + (h * C + c) * fs;
      float o = 0.0f;
#pragma unroll
      for (int k = 0; k < kGatK; ++k)
        if (k < fs) o = fmaf(wr[k], u[k], o);
      o = __fadd_rn(o, sb[h * C + c]);
      y[c] = first ? o : __fadd_rn(y[c], o);
    }
    first = false;
  }
  if (!act) return;
  float* out = a.act + a.act_off[0][t] + (int64_t)i * HC + h * C;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int64_t q = (int64_t)i * HC + h * C + c;
    out[c] = a.drop_thr ? __fmul_rn(first ? 0.0f : y[c], drop_factor(a, 0, t, q)) : (first ? 0.0f : y[c]);
  }
}

// one row chunk's partial gradients of one live relation's GATConv (grid = n_parts x (relations + the readout's weight
// groups)); per thread (row slot, head) sums over its rows, then over the slots in a fixed order (xor tree within the
// wave, then the waves in order)
template <int C>
__global__ __launch_bounds__(kSbThreads) void k_sb_gat_bwd(SbArgs a, const float* gcur) {
  __shared__ float stage[kSbStage];
  const int p = blockIdx.x, r = blockIdx.y;
  if (r >= kRel) {
    ro_weight_part(a, p, r - kRel, stage);
    return;
  }
  if ((a.dead_conv >> r) & 1u) return;   // (its partials stay zero; its parameters are not stepped)
  const int s = kRelSrc[r], d = kRelDst[r];
  const int fs = a.fdim[s], fd = a.fdim[d];
  const int NH = a.gat_heads, HC = NH * C, RS = gat_rows_per_pass(a);
  const int tid = threadIdx.x, slot = tid / NH, h = tid - slot * NH;
  const int rows = nrows(a, d), n_src = nrows(a, s);
  const int ch = (rows + a.n_parts - 1) / a.n_parts;
  const int i0 = p * ch < rows ? p * ch : rows, i1 = (p + 1) * ch < rows ? (p + 1) * ch : rows;
  const SbGat& g = a.gatc[r];
  // staged W_s / folds after the wave-reduction area (at most 4 waves x 32 heads x 52 values, C = 4: 6656 floats)
  constexpr int kGatStg = kSbStage - (128 * kGatK + 2 * 32 * kGatK);
  float* sws = stage + kGatStg;
  float* svs = sws + 128 * kGatK;
  float* svd = svs + 32 * kGatK;
  gat_stage<C>(a, g, fs, fd, sws, svs, svd, nullptr);
  __syncthreads();
  float vs[kGatK], vd[kGatK];
#pragma unroll
  for (int k = 0; k < kGatK; ++k) {
    vs[k] = svs[h * kGatK + k];
    vd[k] = svd[h * kGatK + k];
  }
  float G[C][kGatK], bsum[C], rsum[kGatK], tsum[kGatK];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    bsum[c] = 0.0f;
#pragma unroll
    for (int k = 0; k < kGatK; ++k) G[c][k] = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < kGatK; ++k) rsum[k] = tsum[k] = 0.0f;
  const float sl = a.gat_slope;
  for (int rb = i0; rb < i1; rb += RS) {
    const int i = rb + slot;
    if (slot >= RS || i >= i1) continue;
    float gy[C];
#pragma unroll
    for (int c = 0; c < C; ++c) gy[c] = gout(a, gcur, 0, d, (int64_t)i * HC + h * C + c);
    float q[kGatK];
#pragma unroll
    for (int k = 0; k < kGatK; ++k) q[k] = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      bsum[c] = __fadd_rn(bsum[c], gy[c]);
#pragma unroll
      for (int k = 0; k < kGatK; ++k)
        if (k < fs) q[k] = fmaf(sws[(h * C + c) * fs + k], gy[c], q[k]);
    }
    const float* st = a.gat_st + a.gat_st_off[r] + ((int64_t)i * NH + h) * (2 + fs);
    const float m = st[0], den = st[1];
#pragma unroll
    for (int k = 0; k < kGatK; ++k) {
      const float uk = k < fs ? st[2 + k] : 0.0f;
#pragma unroll
      for (int c = 0; c < C; ++c) G[c][k] = fmaf(gy[c], uk, G[c][k]);
    }
    float xi[kGatK];
    gat_row(a, d, i, xi);
    float ad = 0.0f;
#pragma unroll
    for (int k = 0; k < kGatK; ++k) ad = fmaf(vd[k], xi[k], ad);
    // alpha and g_alpha of edge j (the forward's logit arithmetic)
    auto edge = [&](int j, float (&xj)[kGatK], float& pre, float& al, float& ga) {
      gat_row(a, s, j, xj);
      float as = 0.0f;
      ga = 0.0f;
#pragma unroll
      for (int k = 0; k < kGatK; ++k) {
        as = fmaf(vs[k], xj[k], as);
        ga = fmaf(xj[k], q[k], ga);
      }
      pre = __fadd_rn(as, ad);
      const float ev = pre > 0.0f ? pre : __fmul_rn(sl, pre);
      al = __fdiv_rn(expf(ev - m), den);
    };
    float gad = 0.0f;
    if constexpr (C <= 8) {
      // one walk (round 6): g_pre = lr' alpha (g_alpha - S) is linear in S = sum alpha g_alpha, so its sums split into
      // sum lr' alpha g_alpha [x_s] - S sum lr' alpha [x_s], all four gathered in the walk that forms S — half the
      // dependent memory round trips of the two-walk form below (the same sums in another association: fp32 tolerance)
      float S = 0.0f, D = 0.0f, E = 0.0f, A[kGatK], B[kGatK];
#pragma unroll
      for (int k = 0; k < kGatK; ++k) A[k] = B[k] = 0.0f;
      gat_edges(a, r, i, n_src, rows, [&](int j) {
        float xj[kGatK], pre, al, ga;
        edge(j, xj, pre, al, ga);
        S = fmaf(al, ga, S);
        const float w1 = pre > 0.0f ? al : __fmul_rn(sl, al);
        const float w2 = __fmul_rn(w1, ga);
        D = __fadd_rn(D, w1);
        E = __fadd_rn(E, w2);
#pragma unroll
        for (int k = 0; k < kGatK; ++k) {
          A[k] = fmaf(w2, xj[k], A[k]);
          B[k] = fmaf(w1, xj[k], B[k]);
        }
      });
      gad = fmaf(-S, D, E);
#pragma unroll
      for (int k = 0; k < kGatK; ++k) rsum[k] = __fadd_rn(rsum[k], fmaf(-S, B[k], A[k]));
    } else {   // (C = 16: G alone holds 128 registers, the one-walk sums would spill)
      float S = 0.0f;
      gat_edges(a, r, i, n_src, rows, [&](int j) {
        float xj[kGatK], pre, al, ga;
        edge(j, xj, pre, al, ga);
        S = fmaf(al, ga, S);
      });
      gat_edges(a, r, i, n_src, rows, [&](int j) {
        float xj[kGatK], pre, al, ga;
        edge(j, xj, pre, al, ga);
        const float ge = __fmul_rn(al, __fsub_rn(ga, S));
        const float gp = pre > 0.0f ? ge : __fmul_rn(sl, ge);
        gad = __fadd_rn(gad, gp);
#pragma unroll
        for (int k = 0; k < kGatK; ++k) rsum[k] = fmaf(gp, xj[k], rsum[k]);
      });
    }
#pragma unroll
    for (int k = 0; k < kGatK; ++k) tsum[k] = fmaf(gad, xi[k], tsum[k]);
  }
  // the slots' sums per head: xor tree over the wave's slots (lanes h, h + NH, ...), then the waves in order
  constexpr int V = C * kGatK + C + 2 * kGatK;
  float* wred = stage;   // [waves][NH][V]
  const int lane = tid & 63, w = tid >> 6;
  auto put = [&](int v, float x) {
    for (int off = NH; off < 64; off <<= 1) x = __fadd_rn(x, __shfl_xor(x, off));
    if (lane < NH) wred[(w * NH + lane) * V + v] = x;
  };
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int k = 0; k < kGatK; ++k) put(c * kGatK + k, G[c][k]);
    put(C * kGatK + c, bsum[c]);
  }
#pragma unroll
  for (int k = 0; k < kGatK; ++k) {
    put(C * kGatK + C + k, rsum[k]);
    put(C * kGatK + C + kGatK + k, tsum[k]);
  }
  __syncthreads();
  const int nw = kSbThreads / 64;
  auto tot = [&](int hh, int v) {
    float x = 0.0f;
    for (int q = 0; q < nw; ++q) x = __fadd_rn(x, wred[(q * NH + hh) * V + v]);
    return x;
  };
  float* part = a.part_gin + (int64_t)p * a.p_gin + g.goff;
  for (int idx = tid; idx < HC; idx += kSbThreads) {   // att_src, att_dst, bias
    const int hh = idx / C, c = idx - hh * C;
    float as = 0.0f, adv = 0.0f;
    for (int k = 0; k < fs; ++k) as = fmaf(g.ws[(int64_t)idx * fs + k], tot(hh, C * kGatK + C + k), as);
    for (int k = 0; k < fd; ++k) adv = fmaf(g.wd[(int64_t)idx * fd + k], tot(hh, C * kGatK + C + kGatK + k), adv);
    part[idx] = as;
    part[HC + idx] = adv;
    part[2 * HC + idx] = tot(hh, C * kGatK + c);
  }
  for (int idx = tid; idx < HC * fs; idx += kSbThreads) {   // lin_src.weight
    const int o = idx / fs, k = idx - o * fs, hh = o / C, c = o - hh * C;
    part[3 * HC + idx] = fmaf(g.att_s[o], tot(hh, C * kGatK + C + k), tot(hh, c * kGatK + k));
  }
  for (int idx = tid; idx < HC * fd; idx += kSbThreads) {   // lin_dst.weight
    const int o = idx / fd, k = idx - o * fd, hh = o / C;
    part[3 * HC + HC * fs + idx] = __fmul_rn(g.att_d[o], tot(hh, C * kGatK + C + kGatK + k));
  }
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_sb_readout_lds_bytes(int64_t H, int64_t f_path, int concat_path, int nhid, const int32_t* widths,
                                         int with_weights, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && widths && nhid >= 1 && nhid <= kSbMaxHid && H >= 1, "hgin_sb_readout_lds_bytes: bad args");
  const int64_t w0 = H + (concat_path ? f_path : 0);
  int64_t maxw = w0, tot = w0;
  int64_t wts = widths[nhid - 1], win = w0;   // the head's weights, then per layer W (odd row stride) and b
  for (int i = 0; i < nhid; ++i) {
    HGIN_ARG_CHECK(widths[i] >= 1 && widths[i] <= kSbMaxW, "hgin_sb_readout_lds_bytes: width %d", (int)widths[i]);
    tot += 2 * widths[i];
    maxw = widths[i] > maxw ? widths[i] : maxw;
    wts += widths[i] * ((win | 1) + 1);
    win = widths[i];
  }
  HGIN_ARG_CHECK(w0 <= kSbMaxW, "hgin_sb_readout_lds_bytes: input width %lld", (long long)w0);
  if (with_weights == 3) {   // MLP_BN: the largest of the k_sb_bn_* launches
    int f = 0;
    for (int i = 0; i < nhid; ++i) {
      const int K = i == 0 ? (int)w0 : widths[i - 1], N = widths[i];
      const int fw = bn_fwd_floats(N, K, i > 0 ? K : 0), fb = bn_bwd_floats(N, K, i == 0 ? (int)H : K);
      f = fw > f ? fw : f;
      f = fb > f ? fb : f;
    }
    const int fh = bn_head_floats(widths[nhid - 1]);
    *bytes = sizeof(float) * (size_t)(fh > f ? fh : f);
    return HGIN_OK;
  }
  if (with_weights == 2 || with_weights == 4) {   // k_sb_readout_mfma: 32-row tiles, odd row strides, the split
    int64_t act = w0 | 1;                            // partials (4: the weights through the caches)
    for (int i = 0; i < nhid; ++i) act += 2 * (widths[i] | 1);
    *bytes = sizeof(float) * (size_t)((with_weights == 2 ? wts : 0) + kSbRowsM * (act + 2 * (maxw | 1)) + kSbRowsM +
                                      (kRoThreadsM / 64) * 32 * 33);
    return HGIN_OK;
  }
  *bytes = sizeof(float) * (size_t)(kSbRows * (tot + 2 * maxw) + kSbRows + (with_weights ? wts : 0));
  return HGIN_OK;
}

// args: a host pointer to the filled SbArgs struct (layout in hgin/smallbatch.py); n_tiles = ceil(cap_path / 16);
// readout_lds = hgin_sb_readout_lds_bytes(..., with_weights = ro_wlds, ...).
extern "C" int hgin_sb_step(const void* args, size_t args_bytes, size_t readout_lds, void* stream) {
  HGIN_ARG_CHECK(args && args_bytes == sizeof(SbArgs), "hgin_sb_step: args %zu bytes, expected %zu", args_bytes,
                 sizeof(SbArgs));
  SbArgs a;
  std::memcpy(&a, args, sizeof(SbArgs));
  HGIN_ARG_CHECK(a.G >= 1 && a.L >= 1 && a.L <= kSbMaxL && a.H >= 1 && a.H <= 128 && a.nhid >= 1 && a.kmax <= 128 &&
                     a.nhid <= kSbMaxHid && a.n_tiles >= 1 && readout_lds <= 160 * 1024,
                 "hgin_sb_step: unsupported shape");
  HGIN_ARG_CHECK(a.drop_thr == 0u || a.drop_ctr, "hgin_sb_step: dropout step counter");
  HGIN_ARG_CHECK(a.pool_w == 0 || (a.pooled && a.pbatch && a.pool_w == 2 * a.fdim[0] && a.pool_ld >= a.pool_w),
                 "hgin_sb_step: pooled features (pool_w %d, pool_ld %d)", a.pool_w, a.pool_ld);
  hipStream_t s = as_stream(stream);
  HGIN_TRACE("k_sb_step");
  // the readout kernel's dynamic LDS may use what its static reduction array leaves of the CU's 160 KiB; the limit
  // is a per-device attribute, so it is raised once per device this process launches on (idempotent if two threads
  // race on it)
  int dev = 0;
  HGIN_ARG_CHECK(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "hgin_sb_step: device id");
  static int dyn_max_dev[64];   // 0: not raised yet on that device; -1: failed
  if (dyn_max_dev[dev] == 0) {
    int m = 160 * 1024;   // the smaller of the two variants' limits (-1 if either failed)
    for (const void* fn : {reinterpret_cast<const void*>(k_sb_readout<true>),
                           reinterpret_cast<const void*>(k_sb_readout<false>),
                           reinterpret_cast<const void*>(k_sb_readout_mfma<true>),
                           reinterpret_cast<const void*>(k_sb_readout_mfma<false>),
                           reinterpret_cast<const void*>(k_sb_bn_fwd), reinterpret_cast<const void*>(k_sb_bn_head),
                           reinterpret_cast<const void*>(k_sb_bn_bwd)}) {
      hipFuncAttributes fa;
      int mf = -1;
      if (hipFuncGetAttributes(&fa, fn) == hipSuccess) {
        mf = 160 * 1024 - (int)fa.sharedSizeBytes;
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, mf) != hipSuccess) mf = -1;
      }
      m = mf < m ? mf : m;
    }
    dyn_max_dev[dev] = m;
  }
  const int dyn_max = dyn_max_dev[dev];
  if (dyn_max < 0) {
    set_error("hgin_sb_step: could not raise the readout kernel's dynamic LDS limit");
    return (int)hipErrorInvalidValue;
  }
  HGIN_ARG_CHECK((int64_t)readout_lds <= dyn_max, "hgin_sb_step: readout LDS %zu above %d", readout_lds, dyn_max);
  auto blocks = [](int64_t n) { return (unsigned)(n > 0 ? ceil_div(n, (int64_t)kSbThreads) : 1); };
  int capt_max = 0, kmx = 0;
  for (int t = 0; t < 3; ++t) capt_max = a.cap[t] > capt_max ? a.cap[t] : capt_max;
  for (int r = 0; r < kRel; ++r) {
    const int K0 = a.fdim[kRelSrc[r]] + a.fdim[kRelDst[r]];
    kmx = K0 > kmx ? K0 : kmx;
  }
  HGIN_ARG_CHECK(kmx <= a.kmax && a.H <= a.kmax && a.n_parts >= 1 && capt_max >= 1, "hgin_sb_step: kmax / n_parts");
  HGIN_ARG_CHECK((int64_t)a.n_tiles * kSbRows >= a.cap[0], "hgin_sb_step: %d readout tiles of %d rows < %d path rows",
                 a.n_tiles, kSbRows, a.cap[0]);
  int ro_blocks = 0;   // the readout weight-gradient blocks' groups (ro_groups, on the host)
  for (int i = 0, win = a.H + (a.concat_path ? a.fdim[0] : 0) + a.pool_w; i <= a.nhid; ++i) {
    const int N = i < a.nhid ? a.rw[i] : 1;
    ro_blocks += ro_groups_nk(N, win);
    if (i < a.nhid) win = a.rw[i];
  }
  if (a.gat) {   // HetroGAT: one GATConv layer (k_sb_gat_fwd / k_sb_gat_bwd)
    const int nh = a.gat_heads, c = a.gat_c;
    HGIN_ARG_CHECK(a.L == 1 && nh >= 1 && nh <= 32 && (nh & (nh - 1)) == 0 && (c == 4 || c == 8 || c == 16) &&
                       a.H == nh * c && a.gat_st && a.fdim[0] <= kGatK && a.fdim[1] <= kGatK && a.fdim[2] <= kGatK,
                   "hgin_sb_step: GAT shape (heads %d, C %d, H %d)", nh, c, a.H);
    const dim3 g((unsigned)ceil_div((int64_t)capt_max, (int64_t)(kSbThreads / nh)), a.pool_w ? 4 : 3);
    if (c == 4) k_sb_gat_fwd<4><<<g, kSbThreads, 0, s>>>(a);
    else if (c == 8) k_sb_gat_fwd<8><<<g, kSbThreads, 0, s>>>(a);
    else k_sb_gat_fwd<16><<<g, kSbThreads, 0, s>>>(a);
  } else {
    const unsigned fwd_blocks = (unsigned)ceil_div((int64_t)capt_max, (int64_t)(a.H >= 64 ? kSbFwdRowsM : kSbFwdRows));
    for (int l = 0; l < a.L; ++l) {
      const dim3 g(fwd_blocks, l == 0 && a.pool_w ? 4 : 3);
      if (a.H >= 64)
        k_sb_fwd<true><<<g, kSbThreads, 0, s>>>(a, l);
      else
        k_sb_fwd<false><<<g, kSbThreads, 0, s>>>(a, l);
    }
  }
  // one tile per workgroup (a grid of 512 looping over the tiles, staging the weights once each: 52.9 vs 35 us per
  // batch, profiles/r04/gpu_r — the tiles' serial layer chains want the parallelism, not fewer weight stagings)
  if (a.ro_wlds == 3) {   // MLP_BN: 2 nhid + 1 launches over 32-row tiles (k_sb_bn_*)
    HGIN_ARG_CHECK(a.bn_buf && a.m_valid, "hgin_sb_step: MLP_BN scratch");
    const unsigned nt = (unsigned)ceil_div((int64_t)a.cap[0], (int64_t)kSbRowsM);
    const int w0 = a.H + (a.concat_path ? a.fdim[0] : 0) + a.pool_w;
    for (int i = 0; i < a.nhid; ++i) {
      const int K = i == 0 ? w0 : a.rw[i - 1];
      const size_t lb = sizeof(float) * (size_t)bn_fwd_floats(a.rw[i], K, i > 0 ? K : 0);
      HGIN_ARG_CHECK((int64_t)lb <= dyn_max, "hgin_sb_step: MLP_BN LDS %zu above %d", lb, dyn_max);
      k_sb_bn_fwd<<<nt, kRoThreadsM, lb, s>>>(a, i);
    }
    const size_t lh = sizeof(float) * (size_t)bn_head_floats(a.rw[a.nhid - 1]);
    HGIN_ARG_CHECK((int64_t)lh <= dyn_max, "hgin_sb_step: MLP_BN LDS %zu above %d", lh, dyn_max);
    k_sb_bn_head<<<nt, kRoThreadsM, lh, s>>>(a);
    for (int i = a.nhid - 1; i >= 0; --i) {
      const int K = i == 0 ? w0 : a.rw[i - 1];
      const size_t lb = sizeof(float) * (size_t)bn_bwd_floats(a.rw[i], K, i == 0 ? a.H : K);
      HGIN_ARG_CHECK((int64_t)lb <= dyn_max, "hgin_sb_step: MLP_BN LDS %zu above %d", lb, dyn_max);
      k_sb_bn_bwd<<<nt, kRoThreadsM, lb, s>>>(a, i);
    }
  } else if (a.ro_wlds == 2 || a.ro_wlds == 4) {
    const unsigned g = (unsigned)ceil_div((int64_t)a.n_tiles * kSbRows, (int64_t)kSbRowsM);
    if (a.ro_wlds == 2)
      k_sb_readout_mfma<true><<<g, kRoThreadsM, readout_lds, s>>>(a);
    else
      k_sb_readout_mfma<false><<<g, kRoThreadsM, readout_lds, s>>>(a);
  }
  else if (a.ro_wlds)
    k_sb_readout<true><<<a.n_tiles, kSbThreads, readout_lds, s>>>(a);
  else
    k_sb_readout<false><<<a.n_tiles, kSbThreads, readout_lds, s>>>(a);
  if (a.eval_only) {   // the loss only (and the running sums)
    HGIN_ARG_CHECK(a.loss_acc && a.ro_wlds != 3 && !a.drop_thr, "hgin_sb_step: eval (needs loss_acc, no dropout)");
    k_sb_final<<<1, kSbThreads, 0, s>>>(a);
    return check_launch("hgin_sb_step");
  }
  float* gcur = a.gA;
  float* gnxt = a.gB;
  if (a.gat) {   // the GATConv partials and every readout weight group in one launch
    const dim3 gw(a.n_parts, kRel + ro_blocks);
    if (a.gat_c == 4) k_sb_gat_bwd<4><<<gw, kSbThreads, 0, s>>>(a, gcur);
    else if (a.gat_c == 8) k_sb_gat_bwd<8><<<gw, kSbThreads, 0, s>>>(a, gcur);
    else k_sb_gat_bwd<16><<<gw, kSbThreads, 0, s>>>(a, gcur);
    const int64_t P = a.p_gin + a.p_ro;
    const int64_t fb = ceil_div(P, (int64_t)32);
    k_sb_final<<<(unsigned)(fb < 1024 ? fb : 1024), kSbThreads, 0, s>>>(a);
    return check_launch("hgin_sb_step");
  }
  // the readout's weight-gradient groups ride in the last layer's launch and (L > 1) the first layer's, half each,
  // so that each launch's blocks are resident at once (4 per CU)
  const int ro_hi = a.L > 1 ? (ro_blocks + 1) / 2 : ro_blocks;
  for (int l = a.L - 1; l >= 0; --l) {
    const int ro_n = l == a.L - 1 ? ro_hi : (l == 0 ? ro_blocks - ro_hi : 0);
    const dim3 gw(a.n_parts, kRel + ro_n);
    if (a.H >= 64)
      k_sb_bwd_w<true><<<gw, kSbThreads, 0, s>>>(a, l, gcur, l == a.L - 1 ? 0 : ro_hi);
    else
      k_sb_bwd_w<false><<<gw, kSbThreads, 0, s>>>(a, l, gcur, l == a.L - 1 ? 0 : ro_hi);
    if (l > 0) {
      k_sb_bwd_in<<<dim3(blocks((int64_t)capt_max * a.H), 3), kSbThreads, 0, s>>>(a, l, gnxt);
      float* tt = gcur;
      gcur = gnxt;
      gnxt = tt;
    }
  }
  const int64_t P = a.p_gin + a.p_ro;
  const int64_t fb = ceil_div(P, (int64_t)32);
  k_sb_final<<<(unsigned)(fb < 1024 ? fb : 1024), kSbThreads, 0, s>>>(a);
  return check_launch("hgin_sb_step");
}

extern "C" size_t hgin_sb_args_size(void) { return sizeof(SbArgs); }

#ifdef HGIN_SB_STAMPS
extern "C" int hgin_sb_stamps_read(unsigned long long* out, int64_t n) {
  HGIN_ARG_CHECK(out && n >= kStampRo + kStampW, "hgin_sb_stamps_read: need %d slots", kStampRo + kStampW);
  void* dev = nullptr;   // read, then cleared for the next step
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sb_stamps), sizeof(g_sb_stamps)) != hipSuccess ||
      hipGetSymbolAddress(&dev, HIP_SYMBOL(g_sb_stamps)) != hipSuccess || hipMemset(dev, 0, sizeof(g_sb_stamps)) != hipSuccess)
    return -1;
  return HGIN_OK;
}
#endif

// offsets of the SbArgs fields the host mirror is checked against (hgin/smallbatch.py): one per field group
extern "C" int hgin_sb_args_offsets(int64_t* out, int64_t n) {
  const int64_t offs[] = {(int64_t)offsetof(SbArgs, goff),     (int64_t)offsetof(SbArgs, m_valid),
                          (int64_t)offsetof(SbArgs, conv),     (int64_t)offsetof(SbArgs, rw),
                          (int64_t)offsetof(SbArgs, ro_goff),  (int64_t)offsetof(SbArgs, p_ro),
                          (int64_t)offsetof(SbArgs, act_off),  (int64_t)offsetof(SbArgs, zb_off),
                          (int64_t)offsetof(SbArgs, gc_off),   (int64_t)offsetof(SbArgs, n_tiles),
                          (int64_t)offsetof(SbArgs, loss_value), (int64_t)offsetof(SbArgs, adam_step),
                          (int64_t)offsetof(SbArgs, weight_decay), (int64_t)offsetof(SbArgs, bn_off),
                          (int64_t)offsetof(SbArgs, drop_inv), (int64_t)offsetof(SbArgs, loss_acc),
                          (int64_t)offsetof(SbArgs, dead_conv), (int64_t)offsetof(SbArgs, gatc),
                          (int64_t)offsetof(SbArgs, gat_st_off)};
  const int64_t k = (int64_t)(sizeof(offs) / sizeof(offs[0]));
  HGIN_ARG_CHECK(out && n >= k, "hgin_sb_args_offsets: need %lld slots", (long long)k);
  for (int64_t i = 0; i < k; ++i) out[i] = offs[i];
  return HGIN_OK;
}

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
//                             (the last layer's launch also the readout layers' partial W / bias gradients);
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
// by the host, hgin/smallbatch.py): H <= 64, every GEMM K <= 128, readout widths <= 256, at most 3 hidden readout
// layers and 4 GIN layers, fp32.
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
  float* gz;                // [4] blocks of cap_dst x H     (per relation)
  float* gc;                // [4] blocks of cap_dst x Kmax
  int64_t gz_off[kRel], gc_off[kRel];
  int kmax;                 // row stride of the gc blocks (relations differ in K)
  int cap[3];               // row capacity per node type (grid sizes)
  float* part_gin;          // [n_parts][p_gin]
  int n_parts;              // row chunks of the weight-gradient partials
  float* part_ro;           // [n_parts][p_ro] (row chunks of the path rows; the slope entry comes from slope_part)
  float* loss_part;         // [n_tiles]
  float* slope_part;        // [n_tiles] the shared readout slope's gradient
  int n_tiles;              // readout tiles of kSbRows path rows
  int ro_wlds;              // 1: the readout tiles stage the hidden weights in LDS
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
};

__device__ __forceinline__ int kdim(const SbArgs& a, int l, int r) {
  return l == 0 ? a.fdim[kRelSrc[r]] + a.fdim[kRelDst[r]] : a.H;
}

// fixed-order block reduction (all threads call it; returns the sum to every thread)
__device__ float block_sum(float v, float* red) {
  const int t = threadIdx.x;
  __syncthreads();
  red[t] = v;
  __syncthreads();
  for (int off = kSbThreads / 2; off > 0; off >>= 1) {
    if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
    __syncthreads();
  }
  const float s = red[0];
  __syncthreads();
  return s;
}

__device__ __forceinline__ int nrows(const SbArgs& a, int t) { return a.goff[t * (a.G + 1) + a.G]; }

// One layer's forward for kSbFwdRows rows of node type t (grid = row blocks x types): per relation into t (relation
// order) comb_r = [aggregate | (1 + eps) x_dst] (concat, first layer) or aggregate + (1 + eps) x_dst (add), the
// aggregate a sequential edge-order sum (models.py:210-215); then per row and output column the sum over those
// relations of prelu(comb_r W_r^T + b_r) (models.py:236-239; HeteroConv's sum, models.py:286-298), z kept per
// relation for the backward.  comb_r also goes to HBM (the weight gradients read it).
constexpr int kSbFwdRows = 32;

__global__ __launch_bounds__(kSbThreads) void k_sb_fwd(SbArgs a, int l) {
  __shared__ float s_comb[2][kSbFwdRows * 128];   // <= 2 relations into a type, K <= kmax <= 128
  const int t = blockIdx.y;
  const int tid = threadIdx.x;
  const int H = a.H;
  const int n = nrows(a, t);
  const int r0 = blockIdx.x * kSbFwdRows;
  if (a.adam_step && l == 0 && blockIdx.x == 0 && t == 0 && tid == 0) a.adam_step[0] += 1.0f;   // read by k_sb_final
  if (r0 >= n) return;
  const int nr = n - r0 < kSbFwdRows ? n - r0 : kSbFwdRows;
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
    for (int idx = tid; idx < nr * K; idx += kSbThreads) {
      const int i = r0 + idx / K, k = idx % K;
      float v = 0.0f;
      if (l == 0) {
        const int fs = a.fdim[s];
        if (k < fs) {
          const float* xs = a.x[s];
          const int64_t ld = a.ldx[s];
          const int c = a.cols[s][k];
          for (int e = rp[i]; e < rp[i + 1]; ++e) v = __fadd_rn(v, xs[(int64_t)cl[e] * ld + c]);
        } else {
          v = __fmul_rn(sc, a.x[t][(int64_t)i * a.ldx[t] + a.cols[t][k - fs]]);
        }
      } else {
        const float* xs = a.act + a.act_off[l - 1][s];
        for (int e = rp[i]; e < rp[i + 1]; ++e) v = __fadd_rn(v, xs[(int64_t)cl[e] * H + k]);
        v = __fadd_rn(v, __fmul_rn(sc, a.act[a.act_off[l - 1][t] + (int64_t)i * H + k]));
      }
      s_comb[slot][idx] = v;
      comb[idx] = v;
    }
    ++slot;
  }
  __syncthreads();
  for (int idx = tid; idx < nr * H; idx += kSbThreads) {
    const int ii = idx / H, h = idx % H;
    float y = 0.0f;
    bool first = true;
    int sl = 0;
    for (int r = 0; r < kRel; ++r) {
      if (kRelDst[r] != t) continue;
      const int K = kdim(a, l, r);
      const SbConv& cv = a.conv[l][r];
      const float* cr = s_comb[sl++] + ii * K;
      const float* wr = cv.w + (int64_t)h * K;
      float z = 0.0f;
      for (int k = 0; k < K; ++k) z = fmaf(cr[k], wr[k], z);
      z = __fadd_rn(z, cv.b[h]);
      a.zb[a.zb_off[l][r] + (int64_t)(r0 + ii) * H + h] = z;
      const float yv = z > 0.0f ? z : __fmul_rn(cv.slope[0], z);
      y = first ? yv : __fadd_rn(y, yv);
      first = false;
    }
    a.act[a.act_off[l][t] + (int64_t)(r0 + ii) * H + h] = y;
  }
}

// Tiles of kSbRows path rows (a grid-stride loop over the batch's tiles): readout forward, loss partial, readout
// backward (unscaled) down to the path embeddings' gradient.  Each layer's input rows and pre-activation gradient rows go to ro_in / ro_gz, from which
// the readout blocks of k_sb_bwd_w form the weight-gradient partials over the same row chunks as the GIN's (a tile
// that also reduced its own rows' weight gradients spent most of its time there and left n_tiles partials to sum).
// The hidden weights are staged in LDS when they fit (row stride K | 1: odd, so the forward's column-per-thread reads
// and the backward's row-per-thread reads are both free of bank conflicts).
__global__ __launch_bounds__(kSbThreads) void k_sb_readout(SbArgs a) {
  extern __shared__ float sm[];
  __shared__ float red[kSbThreads];
  const int tid = threadIdx.x;
  const int H = a.H;
  const int m = a.m_valid[0];
  constexpr int R = kSbRows;
  const int fp = a.concat_path ? a.fdim[0] : 0;
  const int w0 = H + fp;
  int win[kSbMaxHid + 1];   // input width of layer i (i = nhid: the head)
  win[0] = w0;
  for (int i = 0; i < a.nhid; ++i) win[i + 1] = a.rw[i];
  int maxw = w0;
  for (int i = 0; i < a.nhid; ++i) maxw = a.rw[i] > maxw ? a.rw[i] : maxw;
  // LDS: [W_i [rw_i][win_i | 1] when ro_wlds] in0 [R][w0] | per hidden layer z_i, y_i [R][rw_i] | gbuf x2 [R][maxw]
  float* p = sm;
  const float* W[kSbMaxHid];
  int ldw[kSbMaxHid];
  for (int i = 0; i < a.nhid; ++i) {
    const int K = win[i], N = a.rw[i];
    if (a.ro_wlds) {
      const int ks = K | 1;
      for (int idx = tid; idx < N * K; idx += kSbThreads) p[(idx / K) * ks + idx % K] = a.row_w[i][idx];
      W[i] = p;
      ldw[i] = ks;
      p += N * ks;
    } else {
      W[i] = a.row_w[i];
      ldw[i] = K;
    }
  }
  float* in0 = p;
  float* zs[kSbMaxHid];
  float* ys[kSbMaxHid];
  p = in0 + R * w0;
  for (int i = 0; i < a.nhid; ++i) {
    zs[i] = p;
    ys[i] = p + R * a.rw[i];
    p += 2 * R * a.rw[i];
  }
  float* gb0 = p;
  float* gb1 = p + R * maxw;
  float* outv = gb1 + R * maxw;   // [R]
  const float* xp = a.act + a.act_off[a.L - 1][0];
  // tiles in a grid-stride loop: the weights are staged once per workgroup
  const int ntile = (m + R - 1) / R;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int r0 = tile * R;
    const int nr = m - r0 < R ? m - r0 : R;
    __syncthreads();   // the staged weights / the previous tile's LDS reads
    for (int idx = tid; idx < nr * w0; idx += kSbThreads) {
      const int rr = idx / w0, k = idx % w0;
      const int64_t row = r0 + rr;
      const float v = k < H ? xp[row * H + k] : a.x[0][row * a.ldx[0] + a.cols[0][k - H]];
      in0[rr * w0 + k] = v;
      a.ro_in[0][(int64_t)r0 * w0 + idx] = v;
    }
    __syncthreads();
    const float slope = a.ro_slope[0];
    for (int i = 0; i < a.nhid; ++i) {
      const float* in = i == 0 ? in0 : ys[i - 1];
      const int K = win[i], N = a.rw[i], lw = ldw[i];
      for (int idx = tid; idx < nr * N; idx += kSbThreads) {
        const int rr = idx / N, o = idx % N;
        const float* wr = W[i] + (int64_t)o * lw;
        float z = 0.0f;
        for (int k = 0; k < K; ++k) z = fmaf(in[rr * K + k], wr[k], z);
        z = __fadd_rn(z, a.row_b[i][o]);
        zs[i][rr * N + o] = z;
        const float yv = z > 0.0f ? z : __fmul_rn(slope, z);
        ys[i][rr * N + o] = yv;
        a.ro_in[i + 1][(int64_t)r0 * N + idx] = yv;
      }
      __syncthreads();
    }
    const int KL = win[a.nhid];
    const float* yl = ys[a.nhid - 1];
    // head + loss numerator + seed, one thread per row
    float lp = 0.0f;
    if (tid < nr) {
      float o = 0.0f;
      for (int k = 0; k < KL; ++k) o = fmaf(yl[tid * KL + k], a.head_w[k], o);
      o = __fadd_rn(o, a.head_b[0]);
      const float yv = a.y[r0 + tid];
      const float u = __fdiv_rn(__fsub_rn(o, yv), yv);
      lp = fabsf(u);
      const float sg = u > 0.0f ? 1.0f : (u < 0.0f ? -1.0f : 0.0f);
      const float go = __fdiv_rn(sg, yv);   // d |u| / d out
      outv[tid] = go;
      a.ro_gz[a.nhid][r0 + tid] = go;
    }
    // fixed-order tile sum of |u| (rows in order)
    red[tid] = tid < nr ? lp : 0.0f;
    __syncthreads();
    if (tid == 0) {
      float s = 0.0f;
      for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, red[rr]);
      a.loss_part[tile] = s;
    }
    for (int idx = tid; idx < nr * KL; idx += kSbThreads) {
      const int rr = idx / KL, k = idx % KL;
      gb0[rr * KL + k] = __fmul_rn(outv[rr], a.head_w[k]);
    }
    __syncthreads();
    float slope_part = 0.0f;   // this thread's share of the shared slope's gradient (fixed assignment)
    float* g_y = gb0;
    float* g_next = gb1;
    for (int i = a.nhid - 1; i >= 0; --i) {
      const int K = win[i], N = a.rw[i], lw = ldw[i];
      // g_z (in place over g_y) and the slope partial
      for (int idx = tid; idx < nr * N; idx += kSbThreads) {
        const float z = zs[i][idx];
        const float g = g_y[idx];
        if (z <= 0.0f) slope_part = fmaf(g, z, slope_part);
        const float gz = z > 0.0f ? g : __fmul_rn(slope, g);
        g_y[idx] = gz;
        a.ro_gz[i][(int64_t)r0 * N + idx] = gz;
      }
      __syncthreads();
      // g_in[k] = sum_o g_z[o] W[o][k] (the first layer: only the path embeddings' H columns have a gradient)
      const int KG = i == 0 ? H : K;
      for (int idx = tid; idx < nr * KG; idx += kSbThreads) {
        const int rr = idx / KG, k = idx % KG;
        float s = 0.0f;
        for (int o = 0; o < N; ++o) s = fmaf(g_y[rr * N + o], W[i][(int64_t)o * lw + k], s);
        g_next[rr * KG + k] = s;
      }
      __syncthreads();
      float* t = g_y;
      g_y = g_next;
      g_next = t;
    }
    const float sp = block_sum(slope_part, red);
    if (tid == 0) a.slope_part[tile] = sp;
    // the path embeddings' gradient for the GIN backward
    float* gpath = a.gA + a.g_off[0];
    for (int idx = tid; idx < nr * H; idx += kSbThreads) gpath[(int64_t)r0 * H + idx] = g_y[idx];
  }
}

// the readout blocks of k_sb_bwd_w: over row chunk p of the m valid path rows, one group of kRoJ x kSbThreads of
// layer i's (i = nhid: the head's) partial weight / bias gradients, g_W[o][k] = sum_rows g_z[o] in[k],
// g_b[o] = sum_rows g_z[o], the chunk's rows in order (staged kRoSub rows at a time).  Block y-index u (after the
// relations' kRel) -> (layer, group): the layers' groups in order.
constexpr int kRoSub = 16;
constexpr int kRoJ = 8;

__device__ __forceinline__ int ro_in_width(const SbArgs& a, int i) {
  return i == 0 ? a.H + (a.concat_path ? a.fdim[0] : 0) : a.rw[i - 1];
}
__device__ __forceinline__ int ro_groups(const SbArgs& a, int i) {
  const int N = i < a.nhid ? a.rw[i] : 1;
  return (N * (ro_in_width(a, i) + 1) + kRoJ * kSbThreads - 1) / (kRoJ * kSbThreads);
}

__device__ void ro_weight_part(const SbArgs& a, int p, int u, float* s_in, float* s_g) {
  int i = 0;
  while (i < a.nhid && u >= ro_groups(a, i)) u -= ro_groups(a, i++);
  const int tid = threadIdx.x;
  const int m = a.m_valid[0];
  const int ch = (m + a.n_parts - 1) / a.n_parts;
  const int i0 = p * ch < m ? p * ch : m, i1 = (p + 1) * ch < m ? (p + 1) * ch : m;
  const int K = ro_in_width(a, i);
  const int N = i < a.nhid ? a.rw[i] : 1;
  const int E = N * (K + 1);
  const float* in = a.ro_in[i];
  const float* gz = a.ro_gz[i];
  float* part = a.part_ro + (int64_t)p * a.p_ro - a.p_gin;   // indexed by the flat readout offsets
  const int64_t wo = i < a.nhid ? a.ro_goff[i] : a.head_goff;
  constexpr int J = kRoJ;
  {
    const int q0 = u * J * kSbThreads;
    float acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.0f;
    for (int rb = i0; rb < i1; rb += kRoSub) {
      const int nr = i1 - rb < kRoSub ? i1 - rb : kRoSub;
      __syncthreads();
      for (int idx = tid; idx < nr * K; idx += kSbThreads) s_in[idx] = in[(int64_t)rb * K + idx];
      for (int idx = tid; idx < nr * N; idx += kSbThreads) s_g[idx] = gz[(int64_t)rb * N + idx];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int q = q0 + j * kSbThreads + tid;
        if (q < E) {
          const int o = q / (K + 1), k = q % (K + 1);
          float v = acc[j];
          if (k < K) {
            for (int rr = 0; rr < nr; ++rr) v = fmaf(s_g[rr * N + o], s_in[rr * K + k], v);
          } else {
            for (int rr = 0; rr < nr; ++rr) v = __fadd_rn(v, s_g[rr * N + o]);
          }
          acc[j] = v;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = q0 + j * kSbThreads + tid;
      if (q < E) {
        const int o = q / (K + 1), k = q % (K + 1);
        part[wo + (k < K ? (int64_t)o * K + k : (int64_t)N * K + o)] = acc[j];
      }
    }
  }
}

// layer l's output gradient of type d (gcur: written by the readout for path rows, by k_sb_bwd_in of layer l + 1
// otherwise); the last layer's link / node outputs feed nothing (models.py:362-376 reads path only)
__device__ __forceinline__ float gout(const SbArgs& a, const float* gcur, int l, int d, int64_t q) {
  return (l == a.L - 1 && d != 0) ? 0.0f : gcur[a.g_off[d] + q];
}

// one row chunk's partial W / bias / slope / eps gradients of one relation (grid = n_parts x relations, plus the
// readout layers' blocks in the last layer's launch); rows of chunk p: [p c, (p + 1) c), c = ceil(rows / n_parts)
__global__ __launch_bounds__(kSbThreads) void k_sb_bwd_w(SbArgs a, int l, const float* gcur) {
  __shared__ float red[kSbThreads];
  __shared__ float stage[2 * kRoSub * kSbMaxW];
  const int p = blockIdx.x, r = blockIdx.y;
  if (r >= kRel) {   // the last layer's launch carries the readout's blocks (grid.y = kRel + their groups)
    ro_weight_part(a, p, r - kRel, stage, stage + kRoSub * kSbMaxW);
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
  float* gz = a.gz + a.gz_off[r];
  const float* comb = a.comb + a.comb_off[l][r];
  const float* zb = a.zb + a.zb_off[l][r];
  float* gc = a.gc + a.gc_off[r];
  // the chunk's rows first: g_z = PReLU'(z) g_y, then g_comb = g_z W (row-local; k_sb_bwd_in reads every row's
  // g_comb after this launch)
  {
    const float slope = cv.slope[0];
    for (int q = tid; q < (i1 - i0) * H; q += kSbThreads) {
      const int64_t qq = (int64_t)i0 * H + q;
      const float z = zb[qq], g = gout(a, gcur, l, d, qq);
      gz[qq] = z > 0.0f ? g : __fmul_rn(slope, g);
    }
    __syncthreads();
    for (int q = tid; q < (i1 - i0) * K; q += kSbThreads) {
      const int i = i0 + q / K, k = q % K;
      const float* gzr = gz + (int64_t)i * H;
      float v = 0.0f;
      for (int h = 0; h < H; ++h) v = fmaf(gzr[h], cv.w[(int64_t)h * K + k], v);
      gc[(int64_t)i * a.kmax + k] = v;
    }
    __syncthreads();
  }
  // g_W[h][k] = sum_i g_z[i][h] comb[i][k]; g_b[h] = sum_i g_z[i][h] (the chunk's rows in order)
  for (int q = tid; q < H * (K + 1); q += kSbThreads) {
    const int h = q / (K + 1), k = q % (K + 1);
    float v = 0.0f;
    for (int i = i0; i < i1; ++i) {
      const float g = gz[(int64_t)i * H + h];
      v = k < K ? fmaf(g, comb[(int64_t)i * K + k], v) : __fadd_rn(v, g);
    }
    part[k < K ? (int64_t)h * K + k : (int64_t)H * K + h] = v;
  }
  // the slope (sum over z <= 0 of g_y z) and eps (g_comb over the self columns times x_dst) partials
  const int fs = l == 0 ? a.fdim[s] : 0;
  float sp = 0.0f, epv = 0.0f;
  for (int q = tid; q < (i1 - i0) * H; q += kSbThreads) {
    const int64_t qq = (int64_t)i0 * H + q;
    const float z = zb[qq];
    if (z <= 0.0f) sp = fmaf(gout(a, gcur, l, d, qq), z, sp);
  }
  const int KS = K - fs;
  for (int q = tid; q < (i1 - i0) * KS; q += kSbThreads) {
    const int i = i0 + q / KS, k = fs + q % KS;
    const float xv = l == 0 ? a.x[d][(int64_t)i * a.ldx[d] + a.cols[d][k - fs]]
                            : a.act[a.act_off[l - 1][d] + (int64_t)i * H + k];
    epv = fmaf(gc[(int64_t)i * a.kmax + k], xv, epv);
  }
  const float ssum = block_sum(sp, red);
  const float esum = block_sum(epv, red);
  if (tid == 0) {
    part[(int64_t)H * K + H] = ssum;
    part[(int64_t)H * K + H + 1] = esum;
  }
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
      for (int e = cp[u]; e < cp[u + 1]; ++e) v = __fadd_rn(v, gc[(int64_t)cd[e] * a.kmax + k]);
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

__global__ __launch_bounds__(kSbThreads) void k_sb_final(SbArgs a) {
  __shared__ float red[kSbThreads];
  const int tid = threadIdx.x;
  AdamCoef ad{0.0f, 1.0f};
  if (a.adam_step) {
    const float st = a.adam_step[0];
    ad.step_size = __fdiv_rn(a.lr, __fsub_rn(1.0f, powf(a.beta1, st)));
    ad.bc2_sqrt = sqrtf(__fsub_rn(1.0f, powf(a.beta2, st)));
  }
  const int m = a.m_valid[0];
  const int ntile = (m + kSbRows - 1) / kSbRows;
  float lp = 0.0f, sp = 0.0f;
  for (int t = tid; t < ntile; t += kSbThreads) {
    lp = __fadd_rn(lp, a.loss_part[t]);
    sp = __fadd_rn(sp, a.slope_part[t]);
  }
  const float s = block_sum(lp, red);
  const float slope_sum = block_sum(sp, red);
  const float lv = __fdiv_rn(__fmul_rn(100.0f, s), (float)m);       // 100 * mean |u| (train.py:12-13)
  const float scale = __fdiv_rn(__fdiv_rn(100.0f, (float)m), __fmul_rn(2.0f, sqrtf(lv)));
  if (blockIdx.x == 0 && tid == 0) a.loss_value[0] = lv;
  const int64_t P = a.p_gin + a.p_ro;
  const int j = tid & 31, g = tid >> 5;
  for (int64_t e0 = (int64_t)blockIdx.x * 32; e0 < P; e0 += (int64_t)gridDim.x * 32) {
    const int64_t e = e0 + j;
    float v = 0.0f;
    if (e < a.p_gin) {
      for (int pp = g; pp < a.n_parts; pp += 8) v = __fadd_rn(v, a.part_gin[(int64_t)pp * a.p_gin + e]);
    } else if (e < P && e != a.ro_slope_goff) {
      for (int pp = g; pp < a.n_parts; pp += 8) v = __fadd_rn(v, a.part_ro[(int64_t)pp * a.p_ro + (e - a.p_gin)]);
    }
    red[tid] = v;
    __syncthreads();
    if (g == 0 && e < P) {
      float t = 0.0f;
      for (int q = 0; q < 8; ++q) t = __fadd_rn(t, red[q * 32 + j]);
      const float gv = __fmul_rn(e == a.ro_slope_goff ? slope_sum : t, scale);
      a.gflat[e] = gv;
      if (a.adam_step) adam_update(a, e, gv, ad);
    }
    __syncthreads();
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
  int64_t wts = 0, win = w0;
  for (int i = 0; i < nhid; ++i) {
    HGIN_ARG_CHECK(widths[i] >= 1 && widths[i] <= kSbMaxW, "hgin_sb_readout_lds_bytes: width %d", (int)widths[i]);
    tot += 2 * widths[i];
    maxw = widths[i] > maxw ? widths[i] : maxw;
    wts += widths[i] * (win | 1);
    win = widths[i];
  }
  HGIN_ARG_CHECK(w0 <= kSbMaxW, "hgin_sb_readout_lds_bytes: input width %lld", (long long)w0);
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
  HGIN_ARG_CHECK(a.G >= 1 && a.L >= 1 && a.L <= kSbMaxL && a.H >= 1 && a.H <= 64 && a.nhid >= 1 && a.kmax <= 128 &&
                     a.nhid <= kSbMaxHid && a.n_tiles >= 1 && readout_lds <= 160 * 1024,
                 "hgin_sb_step: unsupported shape");
  hipStream_t s = as_stream(stream);
  HGIN_TRACE("k_sb_step");
  // the readout kernel's dynamic LDS may use what its static reduction array leaves of the CU's 160 KiB; the limit
  // is a per-device attribute, so it is raised once per device this process launches on (idempotent if two threads
  // race on it)
  int dev = 0;
  HGIN_ARG_CHECK(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "hgin_sb_step: device id");
  static int dyn_max_dev[64];   // 0: not raised yet on that device; -1: failed
  if (dyn_max_dev[dev] == 0) {
    hipFuncAttributes fa;
    int m = -1;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_sb_readout)) == hipSuccess) {
      m = 160 * 1024 - (int)fa.sharedSizeBytes;
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_sb_readout), hipFuncAttributeMaxDynamicSharedMemorySize,
                              m) != hipSuccess)
        m = -1;
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
  for (int i = 0, win = a.H + (a.concat_path ? a.fdim[0] : 0); i <= a.nhid; ++i) {
    const int N = i < a.nhid ? a.rw[i] : 1;
    ro_blocks += (N * (win + 1) + kRoJ * kSbThreads - 1) / (kRoJ * kSbThreads);
    if (i < a.nhid) win = a.rw[i];
  }
  const unsigned fwd_blocks = (unsigned)ceil_div((int64_t)capt_max, (int64_t)kSbFwdRows);
  for (int l = 0; l < a.L; ++l) k_sb_fwd<<<dim3(fwd_blocks, 3), kSbThreads, 0, s>>>(a, l);
  // one tile per workgroup (a grid of 512 looping over the tiles, staging the weights once each: 52.9 vs 35 us per
  // batch, profiles/r04/gpu_r — the tiles' serial layer chains want the parallelism, not fewer weight stagings)
  k_sb_readout<<<a.n_tiles, kSbThreads, readout_lds, s>>>(a);
  float* gcur = a.gA;
  float* gnxt = a.gB;
  for (int l = a.L - 1; l >= 0; --l) {
    k_sb_bwd_w<<<dim3(a.n_parts, l == a.L - 1 ? kRel + ro_blocks : kRel), kSbThreads, 0, s>>>(a, l, gcur);
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

// offsets of the SbArgs fields the host mirror is checked against (hgin/smallbatch.py): one per field group
extern "C" int hgin_sb_args_offsets(int64_t* out, int64_t n) {
  const int64_t offs[] = {(int64_t)offsetof(SbArgs, goff),     (int64_t)offsetof(SbArgs, m_valid),
                          (int64_t)offsetof(SbArgs, conv),     (int64_t)offsetof(SbArgs, rw),
                          (int64_t)offsetof(SbArgs, ro_goff),  (int64_t)offsetof(SbArgs, p_ro),
                          (int64_t)offsetof(SbArgs, act_off),  (int64_t)offsetof(SbArgs, zb_off),
                          (int64_t)offsetof(SbArgs, gc_off),   (int64_t)offsetof(SbArgs, n_tiles),
                          (int64_t)offsetof(SbArgs, loss_value), (int64_t)offsetof(SbArgs, adam_step),
                          (int64_t)offsetof(SbArgs, weight_decay)};
  const int64_t k = (int64_t)(sizeof(offs) / sizeof(offs[0]));
  HGIN_ARG_CHECK(out && n >= k, "hgin_sb_args_offsets: need %lld slots", (long long)k);
  for (int64_t i = 0; i < k; ++i) out[i] = offs[i];
  return HGIN_OK;
}

// F1 — the reference's real training loop (dataset.py:26, :239-244; train.py:25-44): shuffled batches of a few small
// network graphs.  A batch of 8 RouteNet-sized graphs is a few thousand vertices, so the general path (one launch per
// relation, layer and GEMM family, ~100 per step even as one hipGraph replay) is bound by kernel boundaries, not work.
// Here the whole train step of a HetroGIN over a padded batch (hgin/store.py PaddedBatch) is four launches:
//
//   k_sb_gin_fwd   one workgroup per graph of the batch (graphs are disjoint: no cross-workgroup dependency): every
//                  layer, every relation — the CSR aggregate in edge order, the (1 + eps) x_dst self term (concat in the
//                  first layer, add above it: models.py:210-215), Linear + PReLU (models.py:236-239), the per-
//                  destination relation sum (HeteroConv, models.py:286-298) — with workgroup barriers between phases;
//   k_sb_readout   16-row tiles of path rows: the readout MLP (models.py:300-330, :362-376: hidden Linear + the ONE
//                  shared PReLU, Linear head), the MAPE numerator sum_rows |(out - y) / y| (train.py:12-13) and the
//                  readout backward seeded with d sum|u| / d out = sgn(u) / y, per-tile weight-gradient partials;
//   k_sb_gin_bwd   one workgroup per graph: the GIN backward, layers in reverse (PReLU, bias, weight, eps gradients as
//                  per-graph partials; the input gradients through the self term and the CSC aggregate);
//   k_sb_final     every parameter gradient = its partials summed in a fixed order, times d sqrt(loss) / d sum|u| =
//                  100 / (2 m sqrt(loss_value)) (train.py:40-43; the seed above is linear), written into one flat
//                  gradient buffer whose views are the parameters' .grad; loss_value = 100 sum|u| / m.
//
// The optimizer (torch Adam, fused) follows in the same hipGraph.  Every sum runs in a fixed order (deterministic).
// The aggregates are the GIN path's (sequential edge-order fp32 sums: bit-identical); the GEMM-shaped sums and the
// deferred loss scaling re-associate, so the step agrees with the general path within fp32 tolerances
// (tests/test_gpu_smallbatch.py).  Limits (checked by the host, hgin/smallbatch.py): H <= 64, every GEMM K <= 128,
// readout widths <= 256, at most 3 hidden readout layers and 4 GIN layers, fp32.
#include "hgin_common.h"

#include <cstddef>
#include <cstring>

namespace hgin {
namespace {

constexpr int kSbThreads = 256;
constexpr int kSbRows = 16;         // readout rows per workgroup
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
  float* gz;                // [3] blocks of cap_t x H     (per destination type: graphs are row-disjoint)
  float* gc;                // [3] blocks of cap_t x Kmax
  int64_t gz_off[3], gc_off[3];
  int kmax;                 // row stride of the gc blocks (relations into one type may differ in K)
  float* part_gin;          // [G][p_gin]
  float* part_ro;           // [n_tiles][p_ro]
  float* loss_part;         // [n_tiles]
  int n_tiles;
  // outputs
  float* gflat;             // [p_gin + p_ro]
  float* loss_value;        // [1]
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

__global__ __launch_bounds__(kSbThreads) void k_sb_gin_fwd(SbArgs a) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  const int H = a.H;
  int n0[3], n1[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    n0[t] = a.goff[t * (a.G + 1) + j];
    n1[t] = a.goff[t * (a.G + 1) + j + 1];
  }
  for (int l = 0; l < a.L; ++l) {
    for (int r = 0; r < kRel; ++r) {
      const int s = kRelSrc[r], d = kRelDst[r];
      const int K = kdim(a, l, r);
      const SbConv& cv = a.conv[l][r];
      const float sc = __fadd_rn(1.0f, cv.eps[0]);
      const int rows = n1[d] - n0[d];
      float* comb = a.comb + a.comb_off[l][r];
      const int32_t* rp = a.rowptr[r];
      const int32_t* cl = a.col[r];
      // comb = [aggregate | (1 + eps) x_dst] (concat, first layer) or aggregate + (1 + eps) x_dst (add)
      for (int idx = tid; idx < rows * K; idx += kSbThreads) {
        const int i = n0[d] + idx / K;
        const int k = idx % K;
        float v = 0.0f;
        if (l == 0) {
          const int fs = a.fdim[s];
          if (k < fs) {
            const float* xs = a.x[s];
            const int64_t ld = a.ldx[s];
            const int c = a.cols[s][k];
            for (int e = rp[i]; e < rp[i + 1]; ++e) v = __fadd_rn(v, xs[(int64_t)cl[e] * ld + c]);
          } else {
            v = __fmul_rn(sc, a.x[d][(int64_t)i * a.ldx[d] + a.cols[d][k - fs]]);
          }
        } else {
          const float* xs = a.act + a.act_off[l - 1][s];
          for (int e = rp[i]; e < rp[i + 1]; ++e) v = __fadd_rn(v, xs[(int64_t)cl[e] * H + k]);
          v = __fadd_rn(v, __fmul_rn(sc, a.act[a.act_off[l - 1][d] + (int64_t)i * H + k]));
        }
        comb[(int64_t)i * K + k] = v;
      }
      __syncthreads();
      // z = comb W^T + b; y = prelu(z); the layer output of d = the sum over its relations (first one stores)
      const bool first = (r == 0 || r == 1 || r == 2);   // r = 3 (node -> link) adds onto path -> link's output
      float* zb = a.zb + a.zb_off[l][r];
      float* act = a.act + a.act_off[l][d];
      const float slope = cv.slope[0];
      for (int idx = tid; idx < rows * H; idx += kSbThreads) {
        const int i = n0[d] + idx / H;
        const int h = idx % H;
        const float* cr = comb + (int64_t)i * K;
        const float* wr = cv.w + (int64_t)h * K;
        float z = 0.0f;
        for (int k = 0; k < K; ++k) z = fmaf(cr[k], wr[k], z);
        z = __fadd_rn(z, cv.b[h]);
        zb[(int64_t)i * H + h] = z;
        const float yv = z > 0.0f ? z : __fmul_rn(slope, z);
        float* o = act + (int64_t)i * H + h;
        *o = first ? yv : __fadd_rn(*o, yv);
      }
      __syncthreads();
    }
  }
}

// One 16-row tile of path rows: readout forward, loss partial, readout backward (unscaled), weight-gradient partials.
__global__ __launch_bounds__(kSbThreads) void k_sb_readout(SbArgs a) {
  extern __shared__ float sm[];
  __shared__ float red[kSbThreads];
  const int tid = threadIdx.x;
  const int H = a.H;
  const int m = a.m_valid[0];
  const int r0 = blockIdx.x * kSbRows;
  if (r0 >= m) return;
  const int nr = m - r0 < kSbRows ? m - r0 : kSbRows;
  const int fp = a.concat_path ? a.fdim[0] : 0;
  const int w0 = H + fp;
  int win[kSbMaxHid + 1];   // input width of layer i (i = nhid: the head)
  win[0] = w0;
  for (int i = 0; i < a.nhid; ++i) win[i + 1] = a.rw[i];
  // LDS: in0 [16][w0] | per hidden layer z_i, y_i [16][rw_i] | gbuf x2 [16][maxw]
  int maxw = w0;
  for (int i = 0; i < a.nhid; ++i) maxw = a.rw[i] > maxw ? a.rw[i] : maxw;
  float* in0 = sm;
  float* zs[kSbMaxHid];
  float* ys[kSbMaxHid];
  float* p = in0 + kSbRows * w0;
  for (int i = 0; i < a.nhid; ++i) {
    zs[i] = p;
    ys[i] = p + kSbRows * a.rw[i];
    p += 2 * kSbRows * a.rw[i];
  }
  float* gb0 = p;
  float* gb1 = p + kSbRows * maxw;
  float* outv = gb1 + kSbRows * maxw;   // [16]
  const float* xp = a.act + a.act_off[a.L - 1][0];
  for (int idx = tid; idx < nr * w0; idx += kSbThreads) {
    const int rr = idx / w0, k = idx % w0;
    const int64_t row = r0 + rr;
    in0[rr * w0 + k] = k < H ? xp[row * H + k] : a.x[0][row * a.ldx[0] + a.cols[0][k - H]];
  }
  __syncthreads();
  const float slope = a.ro_slope[0];
  for (int i = 0; i < a.nhid; ++i) {
    const float* in = i == 0 ? in0 : ys[i - 1];
    const int K = win[i], N = a.rw[i];
    for (int idx = tid; idx < nr * N; idx += kSbThreads) {
      const int rr = idx / N, o = idx % N;
      const float* wr = a.row_w[i] + (int64_t)o * K;
      float z = 0.0f;
      for (int k = 0; k < K; ++k) z = fmaf(in[rr * K + k], wr[k], z);
      z = __fadd_rn(z, a.row_b[i][o]);
      zs[i][rr * N + o] = z;
      ys[i][rr * N + o] = z > 0.0f ? z : __fmul_rn(slope, z);
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
    outv[tid] = __fdiv_rn(sg, yv);   // d |u| / d out
  }
  // fixed-order tile sum of |u| (rows in order)
  red[tid] = tid < nr ? lp : 0.0f;
  __syncthreads();
  if (tid == 0) {
    float s = 0.0f;
    for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, red[rr]);
    a.loss_part[blockIdx.x] = s;
  }
  __syncthreads();
  float* part = a.part_ro + (int64_t)blockIdx.x * a.p_ro - a.p_gin;   // indexed by the flat readout offsets
  // head gradients: g_w[k] = sum_rows g_out y_last[k]; g_b = sum_rows g_out; g_y_last = g_out w
  for (int k = tid; k < KL; k += kSbThreads) {
    float s = 0.0f;
    for (int rr = 0; rr < nr; ++rr) s = fmaf(outv[rr], yl[rr * KL + k], s);
    part[a.head_goff + k] = s;
  }
  if (tid == 0) {
    float s = 0.0f;
    for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, outv[rr]);
    part[a.head_goff + KL] = s;
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
    const int K = win[i], N = a.rw[i];
    const float* in = i == 0 ? in0 : ys[i - 1];
    // g_z (in place over g_y) and the slope partial
    for (int idx = tid; idx < nr * N; idx += kSbThreads) {
      const float z = zs[i][idx];
      const float g = g_y[idx];
      if (z <= 0.0f) slope_part = fmaf(g, z, slope_part);
      g_y[idx] = z > 0.0f ? g : __fmul_rn(slope, g);
    }
    __syncthreads();
    // g_W[o][k] = sum_rows g_z[o] in[k]; g_b[o] = sum_rows g_z[o]
    const int64_t wo = a.ro_goff[i];
    for (int idx = tid; idx < N * K; idx += kSbThreads) {
      const int o = idx / K, k = idx % K;
      float s = 0.0f;
      for (int rr = 0; rr < nr; ++rr) s = fmaf(g_y[rr * N + o], in[rr * K + k], s);
      part[wo + idx] = s;
    }
    for (int o = tid; o < N; o += kSbThreads) {
      float s = 0.0f;
      for (int rr = 0; rr < nr; ++rr) s = __fadd_rn(s, g_y[rr * N + o]);
      part[wo + (int64_t)N * K + o] = s;
    }
    // g_in[k] = sum_o g_z[o] W[o][k]
    for (int idx = tid; idx < nr * K; idx += kSbThreads) {
      const int rr = idx / K, k = idx % K;
      float s = 0.0f;
      for (int o = 0; o < N; ++o) s = fmaf(g_y[rr * N + o], a.row_w[i][(int64_t)o * K + k], s);
      g_next[rr * K + k] = s;
    }
    __syncthreads();
    float* t = g_y;
    g_y = g_next;
    g_next = t;
  }
  const float sp = block_sum(slope_part, red);
  if (tid == 0) part[a.ro_slope_goff] = sp;
  // the path embeddings' gradient (first H columns of the readout input) for the GIN backward
  float* gpath = a.gA + a.g_off[0];
  for (int idx = tid; idx < nr * H; idx += kSbThreads) {
    const int rr = idx / H, k = idx % H;
    gpath[(int64_t)(r0 + rr) * H + k] = g_y[rr * w0 + k];
  }
}

__global__ __launch_bounds__(kSbThreads) void k_sb_gin_bwd(SbArgs a) {
  __shared__ float red[kSbThreads];
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  const int H = a.H;
  int n0[3], n1[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    n0[t] = a.goff[t * (a.G + 1) + j];
    n1[t] = a.goff[t * (a.G + 1) + j + 1];
  }
  float* part = a.part_gin + (int64_t)j * a.p_gin;
  float* gcur = a.gA;
  float* gnxt = a.gB;
  // the last layer's link / node outputs feed nothing (models.py:362-376 reads path only): zero gradient
  for (int t = 1; t < 3; ++t)
    for (int idx = tid; idx < (n1[t] - n0[t]) * H; idx += kSbThreads) gcur[a.g_off[t] + (int64_t)n0[t] * H + idx] = 0.0f;
  // padding-free: path rows of this graph were written by k_sb_readout (rows < m_valid)
  __syncthreads();
  for (int l = a.L - 1; l >= 0; --l) {
    if (l > 0) {
      for (int t = 0; t < 3; ++t)
        for (int idx = tid; idx < (n1[t] - n0[t]) * H; idx += kSbThreads)
          gnxt[a.g_off[t] + (int64_t)n0[t] * H + idx] = 0.0f;
    }
    __syncthreads();
    for (int r = 0; r < kRel; ++r) {
      const int s = kRelSrc[r], d = kRelDst[r];
      const int K = kdim(a, l, r);
      const SbConv& cv = a.conv[l][r];
      const int rows = n1[d] - n0[d];
      const float slope = cv.slope[0];
      const float* zb = a.zb + a.zb_off[l][r];
      const float* comb = a.comb + a.comb_off[l][r];
      const float* gy = gcur + a.g_off[d];
      float* gz = a.gz + a.gz_off[d] + (int64_t)n0[d] * H;   // this graph's rows of d
      float* gc = a.gc + a.gc_off[d] + (int64_t)n0[d] * a.kmax;   // rows of stride kmax: graph-disjoint
      // g_z, the slope partial (sum over z <= 0 of g_y z)
      float spart = 0.0f;
      for (int idx = tid; idx < rows * H; idx += kSbThreads) {
        const int64_t q = (int64_t)n0[d] * H + idx;
        const float z = zb[q], g = gy[q];
        if (z <= 0.0f) spart = fmaf(g, z, spart);
        gz[idx] = z > 0.0f ? g : __fmul_rn(slope, g);
      }
      const float ssum = block_sum(spart, red);
      if (tid == 0) part[cv.goff + (int64_t)H * K + H] = ssum;
      // g_W[h][k] = sum_i g_z[i][h] comb[i][k] (row groups, then the groups in order); g_b[h] = sum_i g_z[i][h]
      {
        const int P = H * (K + 1);                 // K weight columns + the bias column
        const int RG = P >= kSbThreads ? 1 : kSbThreads / P;
        for (int base = 0; base < P; base += kSbThreads) {
          const int pidx = base + (RG > 1 ? tid % P : tid);
          const int rg = RG > 1 ? tid / P : 0;
          float v = 0.0f;
          const bool live = pidx < P && rg < RG;
          if (live) {
            const int h = pidx / (K + 1), k = pidx % (K + 1);
            for (int i = rg; i < rows; i += RG) {
              const float g = gz[i * H + h];
              v = k < K ? fmaf(g, comb[((int64_t)n0[d] + i) * K + k], v) : __fadd_rn(v, g);
            }
          }
          __syncthreads();
          red[tid] = v;
          __syncthreads();
          if (rg == 0 && pidx < P) {
            float t = red[tid];
            for (int g2 = 1; g2 < RG; ++g2) t = __fadd_rn(t, red[g2 * P + tid]);
            const int h = pidx / (K + 1), k = pidx % (K + 1);
            part[cv.goff + (k < K ? (int64_t)h * K + k : (int64_t)H * K + h)] = t;
          }
          if (RG > 1) break;
        }
      }
      // g_comb = g_z W: the self term's gradient (eps; x_dst above the first layer) and the aggregate's
      const int fs = l == 0 ? a.fdim[s] : 0;   // first self column (concat) / 0 (add: every column)
      const float sc = __fadd_rn(1.0f, cv.eps[0]);
      float epart = 0.0f;
      for (int idx = tid; idx < rows * K; idx += kSbThreads) {
        const int i = idx / K, k = idx % K;
        float gcv = 0.0f;
        for (int h = 0; h < H; ++h) gcv = fmaf(gz[i * H + h], cv.w[(int64_t)h * K + k], gcv);
        const int64_t row = (int64_t)n0[d] + i;
        if (l == 0) {
          if (k >= fs) epart = fmaf(gcv, a.x[d][row * a.ldx[d] + a.cols[d][k - fs]], epart);
        } else {
          epart = fmaf(gcv, a.act[a.act_off[l - 1][d] + row * H + k], epart);
          float* gx = gnxt + a.g_off[d] + row * H + k;
          *gx = __fadd_rn(*gx, __fmul_rn(sc, gcv));
        }
        gc[(int64_t)i * a.kmax + k] = gcv;
      }
      const float esum = block_sum(epart, red);   // (also the barrier before the CSC pass reads gc)
      if (tid == 0) part[cv.goff + (int64_t)H * K + H + 1] = esum;
      if (l > 0) {   // the aggregate's input gradient, by source rows (CSC of the relation), edge order
        const int32_t* cp = a.cptr[r];
        const int32_t* cd = a.cdst[r];
        const int srows = n1[s] - n0[s];
        for (int idx = tid; idx < srows * H; idx += kSbThreads) {
          const int u = n0[s] + idx / H, k = idx % H;
          float v = 0.0f;
          for (int e = cp[u]; e < cp[u + 1]; ++e) v = __fadd_rn(v, gc[(int64_t)(cd[e] - n0[d]) * a.kmax + k]);
          float* gx = gnxt + a.g_off[s] + (int64_t)u * H + k;
          *gx = __fadd_rn(*gx, v);
        }
      }
      __syncthreads();
    }
    float* t = gcur;
    gcur = gnxt;
    gnxt = t;
  }
}

__global__ __launch_bounds__(kSbThreads) void k_sb_final(SbArgs a) {
  __shared__ float red[kSbThreads];
  __shared__ float scale_s;
  const int m = a.m_valid[0];
  const int ntile = (m + kSbRows - 1) / kSbRows;
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int t = 0; t < ntile; ++t) s = __fadd_rn(s, a.loss_part[t]);
    const float lv = __fdiv_rn(__fmul_rn(100.0f, s), (float)m);       // 100 * mean |u| (train.py:12-13)
    scale_s = __fdiv_rn(__fdiv_rn(100.0f, (float)m), __fmul_rn(2.0f, sqrtf(lv)));
    if (blockIdx.x == 0) a.loss_value[0] = lv;
  }
  __syncthreads();
  const float scale = scale_s;
  const int64_t P = a.p_gin + a.p_ro;
  for (int64_t e = (int64_t)blockIdx.x * kSbThreads + threadIdx.x; e < P; e += (int64_t)gridDim.x * kSbThreads) {
    float s = 0.0f;
    if (e < a.p_gin) {
      for (int g = 0; g < a.G; ++g) s = __fadd_rn(s, a.part_gin[(int64_t)g * a.p_gin + e]);
    } else {
      for (int t = 0; t < ntile; ++t) s = __fadd_rn(s, a.part_ro[(int64_t)t * a.p_ro + (e - a.p_gin)]);
    }
    a.gflat[e] = __fmul_rn(s, scale);
  }
  (void)red;
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_sb_readout_lds_bytes(int64_t H, int64_t f_path, int concat_path, int nhid, const int32_t* widths,
                                         size_t* bytes) {
  HGIN_ARG_CHECK(bytes && widths && nhid >= 1 && nhid <= kSbMaxHid && H >= 1, "hgin_sb_readout_lds_bytes: bad args");
  const int64_t w0 = H + (concat_path ? f_path : 0);
  int64_t maxw = w0, tot = w0;
  for (int i = 0; i < nhid; ++i) {
    tot += 2 * widths[i];
    maxw = widths[i] > maxw ? widths[i] : maxw;
  }
  *bytes = sizeof(float) * (size_t)(kSbRows * (tot + 2 * maxw) + kSbRows);
  return HGIN_OK;
}

// args: a host pointer to the filled SbArgs struct (layout in hgin/smallbatch.py); n_tiles = ceil(cap_path / 16).
extern "C" int hgin_sb_step(const void* args, size_t args_bytes, size_t readout_lds, void* stream) {
  HGIN_ARG_CHECK(args && args_bytes == sizeof(SbArgs), "hgin_sb_step: args %zu bytes, expected %zu", args_bytes,
                 sizeof(SbArgs));
  SbArgs a;
  std::memcpy(&a, args, sizeof(SbArgs));
  HGIN_ARG_CHECK(a.G >= 1 && a.L >= 1 && a.L <= kSbMaxL && a.H >= 1 && a.H <= 64 && a.nhid >= 1 &&
                     a.nhid <= kSbMaxHid && a.n_tiles >= 1 && readout_lds <= 160 * 1024,
                 "hgin_sb_step: unsupported shape");
  hipStream_t s = as_stream(stream);
  HGIN_TRACE("k_sb_step");
  // the readout kernel's dynamic LDS may use what its static reduction array leaves of the CU's 160 KiB
  static const int dyn_max = [] {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_sb_readout)) != hipSuccess) return -1;
    const int m = 160 * 1024 - (int)fa.sharedSizeBytes;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(k_sb_readout),
                               hipFuncAttributeMaxDynamicSharedMemorySize, m) == hipSuccess ? m : -1;
  }();
  if (dyn_max < 0) {
    set_error("hgin_sb_step: could not raise the readout kernel's dynamic LDS limit");
    return (int)hipErrorInvalidValue;
  }
  HGIN_ARG_CHECK((int64_t)readout_lds <= dyn_max, "hgin_sb_step: readout LDS %zu above %d", readout_lds, dyn_max);
  k_sb_gin_fwd<<<a.G, kSbThreads, 0, s>>>(a);
  k_sb_readout<<<a.n_tiles, kSbThreads, readout_lds, s>>>(a);
  k_sb_gin_bwd<<<a.G, kSbThreads, 0, s>>>(a);
  const int64_t P = a.p_gin + a.p_ro;
  const int64_t fb = ceil_div(P, kSbThreads);
  k_sb_final<<<(unsigned)(fb < 256 ? fb : 256), kSbThreads, 0, s>>>(a);
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
                          (int64_t)offsetof(SbArgs, loss_value)};
  const int64_t k = (int64_t)(sizeof(offs) / sizeof(offs[0]));
  HGIN_ARG_CHECK(out && n >= k, "hgin_sb_args_offsets: need %lld slots", (long long)k);
  for (int64_t i = 0; i < k; ++i) out[i] = offs[i];
  return HGIN_OK;
}

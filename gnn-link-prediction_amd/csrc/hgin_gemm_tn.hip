// A9 — weight-gradient GEMMs of the GIN update and the readout (backward of Linear: dW = g_z^T X).
//
// Reference: the autograd of torch.nn.Linear inside GINLayer.mlp (models.py:236-239) and the readout
// (models.py:300-330), reached from loss.backward() at train.py:43, where the reduction dimension is every
// node of a type (1e5 .. 1e7 rows) and the output only H x K; a library GEMM tiles the small output and
// leaves most CUs idle (hipBLASLt: 32 workgroups for 128 x 256).  Here the row range is split across
// workgroups that each write an fp32 partial slab; the slabs are added in a fixed order (two levels), so
// the result is bitwise reproducible.
#include "hgin_common.h"

namespace hgin {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

// ---------------------------------------------------------------------------------------------------
// Weight-gradient GEMM "TN":  out[N, K] = A^T [B1 | B2],  A [M, N], B1 [M, K1], B2 [M, K - K1].
// The reduction runs over M (every node of a type: 1e5..1e7 rows) and the output is small (H x K), so
// the M range is split over S workgroups per output tile (S chosen to fill the 256 CUs); each writes an
// fp32 partial slab, and k_slab_reduce adds the slabs in split order — deterministic, no atomics.
// Inner tile: 32 rows of M per stage.  A thread loads 4 consecutive rows x 4 columns of A (and of B):
// read as row float4s (8 lanes cover a 128-B segment of a row) and written transposed — the same 16
// values regrouped as column float4s over the 4 rows, no shuffles — into [n][m] / [k][m] LDS images with
// 36-float rows.  Lane half h owns rows m = 16h .. 16h+15 of the stage, so an MFMA k-step st pairs rows st
// and 16 + st and a lane reads 4 k-steps of its operand with one ds_read_b128 (conflict-free: the 16 lanes
// of a b128 group read 16 rows 144 B apart).  The B operand is concatenated from two sources so
// [aggregate | x_dst] needs no materialised copy.
constexpr int kTnBM = 32;       // rows of M per stage
constexpr int kTnLd = kTnBM + 4;   // [col][m] image row stride (floats)

// 1-D grid over (output tile, split) pairs, tiles of one split consecutive in the logical order, which is
// XCD-contiguous (hgin_common.h): the workgroups reading the same rows of A / B share one XCD's L2.
struct TnGrid {
  int64_t tile_n;    // output-tile rows along N (128, or 32 for N <= 32)
  int64_t tiles_n;   // tiles along N
  int64_t tiles;     // tiles_n * tiles along K (of this launch)
  int64_t n_work;    // tiles * splits
  int xcd;
  int64_t kt0 = 0;   // first K tile of this launch
};
struct TnWork {
  int64_t n0, k0, split;
  bool valid;
};
__device__ __forceinline__ TnWork tn_work(const TnGrid& g) {
  const int64_t q = g.xcd ? xcd_logical(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  TnWork w;
  w.valid = q < g.n_work;
  const int64_t t = q % g.tiles;
  w.split = q / g.tiles;
  w.n0 = (t % g.tiles_n) * g.tile_n;
  w.k0 = (g.kt0 + t / g.tiles_n) * 128;
  return w;
}

// Fused PReLU-backward prologue (hgin_gin_mlp_bwd_w_*): the A operand is formed on its way into LDS as
// g_z = z > 0 ? g_y : slope * g_y from the g_y / z streams (the g_z stream of a separate PReLU-backward pass
// is never written and re-read), and the workgroups of the first K tile also produce the bias / slope
// gradients as per-split partials (column sums of g_z; sum of z * g_y over z <= 0), summed afterwards in a
// fixed order.  gz != NULL: the workgroups of the first K tile also store the g_z they formed (the dX GEMM's
// operand, when the layer needs an input gradient).  Reference: autograd of PReLU + Linear bias
// (models.py:237-238) reached from train.py:43.
struct TnPro {
  const void* z;        // [M, N] pre-activation, row stride ldz (A's element type)
  int64_t ldz;
  const float* slope;   // device float[1]
  float* pcol;          // [N][S] column-sum partials
  float* ps;            // [N tiles][S] slope-sum partials
  int64_t S;
  float* gz = nullptr;  // optional g_z output [M, N] (fp32), row stride ldgz
  int64_t ldgz = 0;
};

// Fixed-order combine of the per-thread prologue partials of one workgroup: 8 row groups of csum per
// column (in group order) and a fixed tree over 256 slope partials.  red: >= 8 * cols + 256 floats.
template <int CPT>
__device__ __forceinline__ void pro_partials(const TnPro& pro, float* red, int cols, int rg, int c0, bool active,
                                             const float (&csum)[CPT], const float (&ssc)[CPT], int64_t n0,
                                             int64_t N, int64_t split) {
  const int tid = threadIdx.x;
  float ssum = 0.0f;
#pragma unroll
  for (int q = 0; q < CPT; ++q) ssum = __fadd_rn(ssum, ssc[q]);
  __syncthreads();   // the LDS operand images are no longer read
  if (active) {
#pragma unroll
    for (int q = 0; q < CPT; ++q) red[rg * cols + c0 + q] = csum[q];
  }
  float* rs = red + 8 * cols;
  rs[tid] = active ? ssum : 0.0f;
  __syncthreads();
  if (tid < cols && n0 + tid < N) {
    float s = 0.0f;
#pragma unroll
    for (int g = 0; g < 8; ++g) s = __fadd_rn(s, red[g * cols + tid]);
    pro.pcol[(n0 + tid) * pro.S + split] = s;
  }
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) rs[tid] = __fadd_rn(rs[tid], rs[tid + off]);
    __syncthreads();
  }
  if (tid == 0) pro.ps[(n0 / cols) * pro.S + split] = rs[0];   // [N tile][S]
}

// TNR = output-tile rows along N: 128 (2 x 2 waves of 64 x 64) or 32 for narrow gradients such as the
// readout's Linear(128, 32) (4 waves of 32 x 32 along K: no MFMA work on rows that do not exist; wave 0
// alone stages the 32-column A block).
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

// kSplit: fp32 operands on the bf16 matrix cores (hgin_common.h split4): the transposed column runs of 4 m
// are written as three bf16 planes ([col][3 x 32 m + pad] rows of kSplitRowWords words) and a lane reads
// 8 consecutive m of a plane (one 16-deep k-block) per ds_read_b128.
// kPro: A = g_y and the PReLU-backward prologue above (TnPro).  kGz: the first K tile's workgroups also store the
// g_z they form (TnPro::gz; its own instantiation: the store code in the others made the kLateZ kernel spill, 38
// scratch ops, fused dW 6.6 -> 8.7 ms per cfg3 layer-0 launch).  kLateZ: z is loaded when the stage is
// written to LDS instead of with the register prefetch (16 fewer VGPRs live across the MFMA cluster).
template <bool kClean, int TNR, bool kSplit, bool kPro, bool kLateZ, bool kGz>
__device__ __forceinline__ void tn_partial_body(const float* __restrict__ A, int64_t lda, const float* __restrict__ B1,
                                                int64_t ldb1, const float* __restrict__ B2, int64_t ldb2, int64_t K1,
                                                int64_t M, int64_t N, int64_t K, int64_t rows_per_split, bool vec,
                                                float* __restrict__ slab, const TnPro& pro, float* smem,
                                                const TnWork& work) {
  constexpr int WGN = TNR == 128 ? 2 : 4;        // waves along K
  constexpr int BMN = TNR == 128 ? 2 : 1;        // 32 x 32 MFMA blocks per wave along N
  constexpr int BMK = TNR == 128 ? 2 : 1;        // ... and along K
  constexpr int kRowW = kSplit ? kSplitRowWords : kTnLd;
  float* At = smem;                  // [n][m]
  float* Bt = smem + TNR * kRowW;    // [k][m]
  uint32_t* Ath = reinterpret_cast<uint32_t*>(At);
  uint32_t* Bth = reinterpret_cast<uint32_t*>(Bt);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t n0 = work.n0;
  const int64_t k0 = work.k0;
  const int64_t mb = work.split * rows_per_split;
  const int64_t me = mb + rows_per_split < M ? mb + rows_per_split : M;

  f32x16 acc[BMN][BMK];
#pragma unroll
  for (int a = 0; a < BMN; ++a)
#pragma unroll
    for (int b = 0; b < BMK; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  // Row quads vary fastest across lanes: the 8 lanes of one column quad cover the stage's 32 rows, so each
  // 16-lane store group writes two column runs of 16 words each (conflict-free banks; with columns varying
  // fastest all 16 lanes hit the same in-row offset of rows 4 apart: 8-way conflicts, SQ_LDS_BANK_CONFLICT
  // 3.8x the LDS-active cycles).  Global loads stay full 128-B row segments (8 column quads per row).
  const int c4 = (tid >> 3) * 4;   // B: 4 columns inside the 128-wide tile
  const int r4 = (tid & 7) * 4;    // B: 4 rows inside the 32-row stage
  // A: the same 4 x 4 blocks over TNR columns (TNR = 32: threads 0-63 only)
  const int c4a = TNR == 128 ? c4 : (tid >> 3) * 4;
  const int r4a = TNR == 128 ? r4 : (tid & 7) * 4;
  const bool stage_a = TNR == 128 || tid < 64;   // wave-uniform
  float4 va[4], vb[4];
  float4 vz[4];                                  // kPro: z of the A block
  const float* Z = static_cast<const float*>(pro.z);
  const int64_t ldz = pro.ldz;
  // kClean (16-B rows; N, K and K1 multiples of 128, so every A tile lies inside N and every B tile wholly
  // inside B1 or B2): the source pointers are fixed per workgroup and a stage is loaded without per-load
  // branches (the selection below is between loaded values; a select between the two kernel arguments'
  // addresses would put them in scratch).  A ragged last stage (the final split at M) loads clamped rows
  // and zeroes them.  Otherwise every element is bounds-checked.
  const bool from1 = k0 < K1;
  const uintptr_t ub = from1 ? reinterpret_cast<uintptr_t>(B1 + k0) : reinterpret_cast<uintptr_t>(B2 + (k0 - K1));
  const float* pb0 = reinterpret_cast<const float*>(ub);
  const int64_t ldb = from1 ? ldb1 : ldb2;
  const float* pa0 = A + n0;
  const uint32_t oa = (uint32_t)(r4a * lda + c4a), ob = (uint32_t)(r4 * ldb + c4);
  const float* pz0 = kPro ? Z + n0 : nullptr;
  const uint32_t oz = kPro ? (uint32_t)(r4a * ldz + c4a) : 0u;
  int64_t m_ld = mb;   // first row of the stage held in va / vb
  // kPro: z of the A block, rows m0 + r4a .. + 3 (zero past me, as the A loads)
  auto load_z = [&](int64_t m0) {
    if (!stage_a) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gm = m0 + r4a + j;
      const bool ok = gm < me;
      if (kClean) {
        const float4 zz = *reinterpret_cast<const float4*>(pz0 + (ok ? gm : me - 1) * ldz + c4a);
        vz[j] = make_float4(ok ? zz.x : 0.f, ok ? zz.y : 0.f, ok ? zz.z : 0.f, ok ? zz.w : 0.f);
      } else {
        const int64_t gn = n0 + c4a;
        float z4[4] = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (gn + q < N) z4[q] = Z[gm * ldz + gn + q];
        }
        vz[j] = make_float4(z4[0], z4[1], z4[2], z4[3]);
      }
    }
  };
  auto load_stage = [&](int64_t m0) {
    m_ld = m0;
    if constexpr (kPro && !kLateZ) load_z(m0);
    if constexpr (kClean) {
      if (m0 + kTnBM <= me) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (stage_a) {
            const float4 a = *reinterpret_cast<const float4*>(pa0 + (m0 + j) * lda + oa);
            va[j] = a;
          }
          const float4 b = *reinterpret_cast<const float4*>(pb0 + (m0 + j) * ldb + ob);
          vb[j] = b;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (stage_a) {
            const int64_t gm = m0 + r4a + j;
            const bool ok = gm < me;
            const float4 a = *reinterpret_cast<const float4*>(pa0 + (ok ? gm : me - 1) * lda + c4a);
            va[j] = make_float4(ok ? a.x : 0.f, ok ? a.y : 0.f, ok ? a.z : 0.f, ok ? a.w : 0.f);
          }
          const int64_t gm = m0 + r4 + j;
          const bool ok = gm < me;
          const float4 b = *reinterpret_cast<const float4*>(pb0 + (ok ? gm : me - 1) * ldb + c4);
          vb[j] = make_float4(ok ? b.x : 0.f, ok ? b.y : 0.f, ok ? b.z : 0.f, ok ? b.w : 0.f);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (stage_a) {
          const int64_t gm = m0 + r4a + j;
          float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
          const int64_t gn = n0 + c4a;
          if (gm < me) {
            const float* pa = A + gm * lda + gn;
            if (gn + 0 < N) a0 = pa[0];
            if (gn + 1 < N) a1 = pa[1];
            if (gn + 2 < N) a2 = pa[2];
            if (gn + 3 < N) a3 = pa[3];
          }
          va[j] = make_float4(a0, a1, a2, a3);
        }
        const int64_t gm = m0 + r4 + j;
        float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
        if (gm < me) {
          const int64_t gk = k0 + c4;
          auto bk = [&](int64_t k) { return k < K ? (k < K1 ? B1[gm * ldb1 + k] : B2[gm * ldb2 + (k - K1)]) : 0.0f; };
          b0 = bk(gk);
          b1 = bk(gk + 1);
          b2 = bk(gk + 2);
          b3 = bk(gk + 3);
        }
        vb[j] = make_float4(b0, b1, b2, b3);
      }
    }
  };
  // kPro: g_z of the loaded A block (zero rows stay zero), its partial sums, and the optional g_z stream
  float csum[4] = {0.f, 0.f, 0.f, 0.f};   // per-column fixed-order chains, branch-free (see the bf16 kernel)
  float ssc[4] = {0.f, 0.f, 0.f, 0.f};
  const float slope = kPro ? pro.slope[0] : 0.0f;
  auto prologue = [&]() {
    if (!stage_a) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // branch-free (a data-dependent branch per element splits the block and
                                    // the scheduler then keeps every loaded value alive: heavy spilling)
      float g[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
      const float zz[4] = {vz[j].x, vz[j].y, vz[j].z, vz[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool pos = zz[q] > 0.0f;
        ssc[q] = __fadd_rn(ssc[q], pos ? 0.0f : __fmul_rn(zz[q], g[q]));
        g[q] = pos ? g[q] : __fmul_rn(slope, g[q]);
        csum[q] = __fadd_rn(csum[q], g[q]);
      }
      va[j] = make_float4(g[0], g[1], g[2], g[3]);
    }
  };
  // the 4 x 4 block regrouped: column c4 + t gets (row r4 .. r4 + 3) as one float4
  const bool store_gz = kPro && kGz && work.k0 == 0 && stage_a;   // workgroup / wave-uniform
  auto store_stage = [&]() {
    if constexpr (kPro && kLateZ) load_z(m_ld);
    if constexpr (kPro) prologue();
    if constexpr (kPro) {
      if (kGz && store_gz) {   // rows m_ld + r4a + j, columns n0 + c4a .. + 3 (rows past me were zeroed: skipped)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t gm = m_ld + r4a + j;
          const int64_t gn = n0 + c4a;
          if (gm >= me) continue;
          float* dst = pro.gz + gm * pro.ldgz + gn;
          if (kClean) {
            *reinterpret_cast<float4*>(dst) = va[j];
          } else {
            const float g[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (gn + q < N) dst[q] = g[q];
          }
        }
      }
    }
    if constexpr (kSplit) {
      auto put = [&](uint32_t* img, int col, int r, const float4 v) {
        uint2 o[3];
        split4(v, o);
        uint32_t* row = img + col * kSplitRowWords + (r >> 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(row + p * 16) = o[p];
      };
      if (stage_a) {
        put(Ath, c4a + 0, r4a, make_float4(va[0].x, va[1].x, va[2].x, va[3].x));
        put(Ath, c4a + 1, r4a, make_float4(va[0].y, va[1].y, va[2].y, va[3].y));
        put(Ath, c4a + 2, r4a, make_float4(va[0].z, va[1].z, va[2].z, va[3].z));
        put(Ath, c4a + 3, r4a, make_float4(va[0].w, va[1].w, va[2].w, va[3].w));
      }
      put(Bth, c4 + 0, r4, make_float4(vb[0].x, vb[1].x, vb[2].x, vb[3].x));
      put(Bth, c4 + 1, r4, make_float4(vb[0].y, vb[1].y, vb[2].y, vb[3].y));
      put(Bth, c4 + 2, r4, make_float4(vb[0].z, vb[1].z, vb[2].z, vb[3].z));
      put(Bth, c4 + 3, r4, make_float4(vb[0].w, vb[1].w, vb[2].w, vb[3].w));
      return;
    }
    if (stage_a) {
      *reinterpret_cast<float4*>(At + (c4a + 0) * kTnLd + r4a) = make_float4(va[0].x, va[1].x, va[2].x, va[3].x);
      *reinterpret_cast<float4*>(At + (c4a + 1) * kTnLd + r4a) = make_float4(va[0].y, va[1].y, va[2].y, va[3].y);
      *reinterpret_cast<float4*>(At + (c4a + 2) * kTnLd + r4a) = make_float4(va[0].z, va[1].z, va[2].z, va[3].z);
      *reinterpret_cast<float4*>(At + (c4a + 3) * kTnLd + r4a) = make_float4(va[0].w, va[1].w, va[2].w, va[3].w);
    }
    *reinterpret_cast<float4*>(Bt + (c4 + 0) * kTnLd + r4) = make_float4(vb[0].x, vb[1].x, vb[2].x, vb[3].x);
    *reinterpret_cast<float4*>(Bt + (c4 + 1) * kTnLd + r4) = make_float4(vb[0].y, vb[1].y, vb[2].y, vb[3].y);
    *reinterpret_cast<float4*>(Bt + (c4 + 2) * kTnLd + r4) = make_float4(vb[0].z, vb[1].z, vb[2].z, vb[3].z);
    *reinterpret_cast<float4*>(Bt + (c4 + 3) * kTnLd + r4) = make_float4(vb[0].w, vb[1].w, vb[2].w, vb[3].w);
  };
  // Register-prefetch pipeline (as in hgin_gemm_nt.hip): stage s+1 is loaded under stage s's MFMAs.
  load_stage(mb);
  store_stage();
  __syncthreads();
  for (int64_t m0 = mb; m0 < me; m0 += kTnBM) {
    const bool more = m0 + kTnBM < me;
    if (more) load_stage(m0 + kTnBM);
    __builtin_amdgcn_s_setprio(1);   // keep the MFMA cluster together (T5)
    if constexpr (kSplit) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        bf16x8 fa[BMN][3], fb[BMK][3];
#pragma unroll
        for (int t = 0; t < BMN; ++t)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fa[t][p] = *reinterpret_cast<const bf16x8*>(Ath + (wm * 32 * BMN + t * 32 + li) * kSplitRowWords + p * 16 +
                                                        kb * 8 + lh * 4);
#pragma unroll
        for (int t = 0; t < BMK; ++t)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[t][p] = *reinterpret_cast<const bf16x8*>(Bth + (wn * 32 * BMK + t * 32 + li) * kSplitRowWords + p * 16 +
                                                        kb * 8 + lh * 4);
#pragma unroll
        for (int tm = 0; tm < BMN; ++tm)
#pragma unroll
          for (int tn = 0; tn < BMK; ++tn) {   // smallest terms first
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][2], fb[tn][0], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[tn][1], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][2], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[tn][0], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][1], acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][0], acc[tm][tn], 0, 0, 0);
          }
      }
    } else {
  #pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 fa[BMN], fb[BMK];
  #pragma unroll
        for (int t = 0; t < BMN; ++t)
          fa[t] = *reinterpret_cast<const float4*>(At + (wm * 32 * BMN + t * 32 + li) * kTnLd + lh * 16 + 4 * q);
  #pragma unroll
        for (int t = 0; t < BMK; ++t)
          fb[t] = *reinterpret_cast<const float4*>(Bt + (wn * 32 * BMK + t * 32 + li) * kTnLd + lh * 16 + 4 * q);
  #pragma unroll
        for (int tm = 0; tm < BMN; ++tm)
  #pragma unroll
          for (int tn = 0; tn < BMK; ++tn) {
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
      store_stage();
      __syncthreads();
    }
  }
  if constexpr (kPro) {
    if (work.k0 == 0)   // workgroup-uniform
      pro_partials<4>(pro, smem, TNR, r4a >> 2, c4a, stage_a, csum, ssc, n0, N, work.split);
  }
  float* out = slab + work.split * N * K;
#pragma unroll
  for (int tm = 0; tm < BMN; ++tm)
#pragma unroll
    for (int tn = 0; tn < BMK; ++tn) {
      const int64_t k = k0 + wn * 32 * BMK + tn * 32 + li;
      if (k >= K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t n = n0 + wm * 32 * BMN + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (n < N) out[n * K + k] = acc[tm][tn][e];
      }
    }
}

template <bool kClean, int TNR, bool kSplit, bool kPro, bool kLateZ = false, bool kGz = false>
__global__ __launch_bounds__(256, (kPro && !kLateZ) ? 2 : 3) void k_gemm_tn_partial(const float* __restrict__ A, int64_t lda,
                                                            const float* __restrict__ B1, int64_t ldb1,
                                                            const float* __restrict__ B2, int64_t ldb2, int64_t K1,
                                                            int64_t M, int64_t N, int64_t K, int64_t rows_per_split,
                                                            bool vec, float* __restrict__ slab, TnGrid grid,
                                                            TnPro pro) {
  constexpr int kRowW = kSplit ? kSplitRowWords : kTnLd;
  __shared__ __attribute__((aligned(16))) float smem[(TNR + 128) * kRowW];
  const TnWork work = tn_work(grid);
  if (!work.valid) return;
  tn_partial_body<kClean, TNR, kSplit, kPro, kLateZ, kGz>(A, lda, B1, ldb1, B2, ldb2, K1, M, N, K, rows_per_split, vec,
                                                          slab, pro, smem, work);
}

// Small weight gradients (N or K < 16, e.g. the readout head Linear(32, 1)): no MFMA tile to fill, so a
// block owns a chunk of M rows and thread (r, p) accumulates pair p = (n, k) over rows r, r + R, ... in
// order; the R row-lanes are combined in LDS in lane order.  Output: the same [split][N*K] slabs.
template <typename T>
__global__ __launch_bounds__(256) void k_tn_small(const T* __restrict__ A, int64_t lda, const T* __restrict__ B1,
                                                  int64_t ldb1, const T* __restrict__ B2, int64_t ldb2, int64_t K1,
                                                  int64_t M, int N, int K, int64_t rows_per_split,
                                                  float* __restrict__ slab) {
  __shared__ float red[256];
  const int P = N * K;
  const int PW = P < 256 ? P : 256;
  const int R = 256 / PW;
  const int t = threadIdx.x;
  const int rl = t / PW;
  const int64_t mb = (int64_t)blockIdx.x * rows_per_split;
  const int64_t me = mb + rows_per_split < M ? mb + rows_per_split : M;
  for (int p0 = 0; p0 < P; p0 += PW) {
    const int p = p0 + t % PW;
    float acc = 0.0f;
    if (rl < R && p < P) {
      const int n = p / K, k = p % K;
      const T* bcol = k < K1 ? B1 + k : B2 + (k - K1);
      const int64_t ldb = k < K1 ? ldb1 : ldb2;
      for (int64_t m = mb + rl; m < me; m += R)
        acc = __fadd_rn(acc, __fmul_rn(Elem<T>::ld(A + m * lda + n), Elem<T>::ld(bcol + m * ldb)));
    }
    red[t] = acc;
    __syncthreads();
    if (rl == 0 && p < P) {
      float s = 0.0f;
      for (int j = 0; j < R; ++j) s = __fadd_rn(s, red[j * PW + t]);
      slab[(int64_t)blockIdx.x * P + p] = s;
    }
    __syncthreads();
  }
}

// Deterministic two-level slab sum: level 1 adds groups of kSlabGroup consecutive slabs (float4 per
// thread, many workgroups in flight), level 2 adds the group sums in group order.
constexpr int kSlabGroup = 16;

__global__ __launch_bounds__(256) void k_slab_reduce1(const float* __restrict__ slab, int64_t S, int64_t NK,
                                                      float* __restrict__ part) {
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= NK) return;
  const int64_t g = blockIdx.y;
  const int64_t s0 = g * kSlabGroup;
  const int64_t s1 = s0 + kSlabGroup < S ? s0 + kSlabGroup : S;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  const bool full = i4 + 3 < NK && (NK & 3) == 0;
  for (int64_t j = s0; j < s1; ++j) {
    const float* p = slab + j * NK + i4;
    if (full) {
      const float4 v = *reinterpret_cast<const float4*>(p);
      a[0] = __fadd_rn(a[0], v.x); a[1] = __fadd_rn(a[1], v.y); a[2] = __fadd_rn(a[2], v.z); a[3] = __fadd_rn(a[3], v.w);
    } else {
      for (int c = 0; c < 4 && i4 + c < NK; ++c) a[c] = __fadd_rn(a[c], p[c]);
    }
  }
  float* q = part + g * NK + i4;
  for (int c = 0; c < 4 && i4 + c < NK; ++c) q[c] = a[c];
}

__global__ __launch_bounds__(256) void k_slab_reduce2(const float* __restrict__ part, int64_t G, int64_t NK,
                                                      float* __restrict__ out, int64_t K, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NK) return;
  float s = 0.0f;
  for (int64_t j = 0; j < G; ++j) s = __fadd_rn(s, part[j * NK + i]);
  out[(i / K) * ldo + (i % K)] = s;
}

// Both levels of the slab sum in ONE launch, with the same arithmetic (bit-identical to k_slab_reduce1 +
// k_slab_reduce2): a workgroup owns 64 consecutive outputs; its 16 thread rows x 16 float4 lanes form the
// group sums (group g by row g mod 16) into LDS, then 64 threads add the group sums in group order.  The
// level-2 pass no longer re-reads G x NK partials from HBM, and a launch + kernel boundary goes per call.
// With `pro` the last N + 1 workgroups are k_pro_final's (independent work, uniform per workgroup).
constexpr int kSlabMaxG = 64;   // S <= 1024 (tn_splits) -> G = ceil(S / kSlabGroup) <= 64
constexpr int kSlabCols = 64;

__global__ __launch_bounds__(256) void k_slab_reduce(const float* __restrict__ slab, int64_t S, int64_t NK,
                                                     float* __restrict__ out, int64_t K, int64_t ldo,
                                                     int64_t n_red, const float* __restrict__ pcol,
                                                     const float* __restrict__ ps, int64_t n_ps,
                                                     float* __restrict__ g_bias, float* __restrict__ g_prelu) {
  __shared__ float part[kSlabMaxG * kSlabCols];
  const int t = threadIdx.x;
  if ((int64_t)blockIdx.x >= n_red) {   // k_pro_final workgroups
    float* red = part;
    const int64_t c = (int64_t)blockIdx.x - n_red;
    const bool slope = c == (int64_t)gridDim.x - n_red - 1;
    const int64_t n = slope ? n_ps : S;
    const float* p = slope ? ps : pcol + c * S;
    float s = 0.0f;
    for (int64_t b = t; b < n; b += 256) s = __fadd_rn(s, p[b]);
    red[t] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (t < off) red[t] = __fadd_rn(red[t], red[t + off]);
      __syncthreads();
    }
    if (t == 0) {
      if (slope) g_prelu[0] = red[0];
      else g_bias[c] = red[0];
    }
    return;
  }
  const int q = t & 15, r = t >> 4;
  const int64_t base = (int64_t)blockIdx.x * kSlabCols;
  const int64_t i4 = base + q * 4;
  const int64_t G = (S + kSlabGroup - 1) / kSlabGroup;
  const bool full = i4 + 3 < NK && (NK & 3) == 0;
  for (int64_t g = r; g < G; g += 16) {
    const int64_t s0 = g * kSlabGroup;
    const int64_t s1 = s0 + kSlabGroup < S ? s0 + kSlabGroup : S;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (full) {
      for (int64_t j = s0; j < s1; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(slab + j * NK + i4);
        a[0] = __fadd_rn(a[0], v.x); a[1] = __fadd_rn(a[1], v.y); a[2] = __fadd_rn(a[2], v.z); a[3] = __fadd_rn(a[3], v.w);
      }
    } else {
      for (int64_t j = s0; j < s1; ++j)
        for (int c = 0; c < 4 && i4 + c < NK; ++c) a[c] = __fadd_rn(a[c], slab[j * NK + i4 + c]);
    }
    for (int c = 0; c < 4; ++c) part[g * kSlabCols + q * 4 + c] = a[c];
  }
  __syncthreads();
  if (t < kSlabCols && base + t < NK) {
    float s = 0.0f;
    for (int64_t g = 0; g < G; ++g) s = __fadd_rn(s, part[g * kSlabCols + t]);
    const int64_t i = base + t;
    out[(i / K) * ldo + (i % K)] = s;
  }
}

constexpr bool slab_fused_enabled() { return true; }

// ---------------------------------------------------------------------------------------------------
// bf16 operands (cfg5): 64 rows of M per stage.  (A register-transposing bf16 dW kernel, measured 1.9x slower than
// the transposed-read kernel below, was removed: DESIGN.md §3.)
constexpr int kTnBMh = 64;

using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
typedef bf16x4 __attribute__((address_space(3))) lds_bf16x4;

__device__ __forceinline__ int tr_img_off(int row, int ch) {   // byte offset in a [64][256 B] image
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

template <bool kVec>
__global__ __launch_bounds__(256, 2) void k_gemm_tn_bf16_tr(const uint16_t* __restrict__ A, int64_t lda,
                                                            const uint16_t* __restrict__ B1, int64_t ldb1,
                                                            const uint16_t* __restrict__ B2, int64_t ldb2, int64_t K1,
                                                            int64_t M, int64_t N, int64_t K, int64_t rows_per_split,
                                                            float* __restrict__ slab, TnGrid grid) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 64 * 128];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const TnWork work = tn_work(grid);
  if (!work.valid) return;
  const int64_t n0 = work.n0;
  const int64_t k0 = work.k0;
  const int64_t mb = work.split * rows_per_split;
  const int64_t me = mb + rows_per_split < M ? mb + rows_per_split : M;
  const bool isB = tid >= 128;
  const int ch = tid & 15;            // 16-B chunk (8 columns) of a 256-B row
  const int r0 = (tid & 127) >> 4;    // rows r0 + 8 i of the 64-row stage
  char* const img = reinterpret_cast<char*>(smem) + (isB ? 64 * 256 : 0);

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  uint4 v[8];
  const int64_t c0 = (isB ? k0 : n0) + 8 * ch;
  const int64_t lim = isB ? K : N;
  const uint16_t* vbase = !isB ? A + c0 : (c0 < K1 ? B1 + c0 : B2 + (c0 - K1));
  const int64_t vld = !isB ? lda : (c0 < K1 ? ldb1 : ldb2);
  // kVec (16-B aligned rows, N, K, K1 multiples of 8): a chunk lies wholly inside or outside its matrix
  auto load_stage = [&](int64_t m0) {
    if constexpr (kVec) {
      const bool cin = c0 < lim;
      const uint16_t* p = vbase + (m0 + r0) * vld;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bool ok = cin && m0 + r0 + 8 * i < me;
        v[i] = ok ? *reinterpret_cast<const uint4*>(p + 8 * i * vld) : make_uint4(0u, 0u, 0u, 0u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t gm = m0 + r0 + 8 * i;
        uint32_t t[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int64_t k = c0 + c;
          t[c] = 0u;
          if (gm < me && k < lim)
            t[c] = !isB ? A[gm * lda + k] : (k < K1 ? B1[gm * ldb1 + k] : B2[gm * ldb2 + (k - K1)]);
        }
        v[i] = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
      }
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(img + tr_img_off(r0 + 8 * i, ch)) = v[i];
  };
  // per-lane byte offsets of the two transposed reads of each fragment (kb adds 16 rows = 4096 B):
  // lane 4q + p of 16-lane group g reads rows 8 (g >> 1) + 4 half + q, columns cb + 16 (g & 1) + 4p .. + 3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  int ra[2][2], rbo[2][2];   // [tile][half]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * (g >> 1) + 4 * h + q;
      const int ca = wm * 64 + t * 32 + 16 * (g & 1);
      const int cb = wn * 64 + t * 32 + 16 * (g & 1);
      ra[t][h] = tr_img_off(row, ca / 8 + (pp >> 1)) + 8 * (pp & 1);
      rbo[t][h] = 64 * 256 + tr_img_off(row, cb / 8 + (pp >> 1)) + 8 * (pp & 1);
    }
  const char* lds = reinterpret_cast<const char*>(smem);
  auto tr = [&](int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + off));
  };
  load_stage(mb);
  store_stage();
  __syncthreads();
  for (int64_t m0 = mb; m0 < me; m0 += kTnBMh) {
    const bool more = m0 + kTnBMh < me;
    if (more) load_stage(m0 + kTnBMh);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < kTnBMh / 16; ++kb) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x4 a0 = tr(ra[t][0] + kb * 4096), a1 = tr(ra[t][1] + kb * 4096);
        const bf16x4 b0 = tr(rbo[t][0] + kb * 4096), b1 = tr(rbo[t][1] + kb * 4096);
        fa[t] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        fb[t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      __syncthreads();
      store_stage();
      __syncthreads();
    }
  }
  float* out = slab + work.split * N * K;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int64_t k = k0 + wn * 64 + tn * 32 + li;
      if (k >= K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t n = n0 + wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (n < N) out[n * K + k] = acc[tm][tn][e];
      }
    }
}


// ---------------------------------------------------------------------------------------------------
// k_wsd_bf16 — weight-gradient (dW = A^T B, A = g_z [M, N], B = comb [M, K]) in the streaming form of
// k_ws_bf16 (hgin_gemm_nt.hip) for N, K in {128, 256}: one persistent workgroup per CU of 8 waves holds the
// WHOLE N x K output in registers (each wave 64 n x K/WK k; 128 accumulator VGPRs at N = K = 256), so A and B are
// each read exactly once from HBM (the tiled kernel reads every row twice: two 128-column output tiles each).
// 32-row m-blocks of A and B stream HBM -> LDS by inline-asm LDS-DMA into a 4-deep ring with counted vmcnt
// waits (nothing else touches vector memory inside the loop); the images are m-major rows with image (b) of
// k_gemm_tn_bf16_tr (16-B chunk ch of row r at ch ^ (((r & 3) << 2) | ((r >> 2) & 3))), the DMA lanes fetching
// pre-swizzled sources, and every MFMA fragment is gathered by two ds_read_b64_tr_b16 reads.  Rows past M in
// the last block are zeroed in LDS before use.  Each workgroup's N x K partial goes to its fp32 slab; the slabs
// are added by k_slab_reduce in fixed order: deterministic (a different M partition from the tiled kernel,
// so equal within fp32 reassociation, not bitwise).
// PRO (the PReLU backward folded in, hgin_gin_mlp_bwd_w_bf16 when g_z is wanted): the A image is DMA'd as g_y
// with a second image of z beside it (same rows, same swizzle, so a chunk of one lines up with the same elements of
// the other); once a block has landed, every thread rewrites its fixed chunks of the A image in place as
// g_z = z > 0 ? g_y : slope * g_y (fp32 arithmetic, one RNE rounding: k_rows_bwd<0>'s), stores them to the g_z
// output (the dX GEMM's operand) and keeps per-thread column sums of the unrounded g_z and the slope sum
// (z <= 0 ? z * g_y), reduced per workgroup in fixed order into the [N][slabs] / [slabs] partials k_slab_reduce
// finishes.  g_w is bit-identical to k_rows_bwd<0> + the plain kernel (same g_z, same grid).
// zy (pro.yalt, round 6): the forward left z unwritten (hgin_gin_mlp_fwd_zy_bf16, slope > 0), so the z image is
// DMA'd from y = prelu(z): y > 0 exactly where z > 0, so g_z (and g_w, the column sums) are the same bits; the slope
// sum is sum(y g) / slope over y <= 0 (y = bf16(slope z) there: the same sum up to bf16 rounding of z).
template <int N, int K, bool PRO = false>
struct WsdCfg {
  static constexpr int NT = 512;
  static constexpr int WM = N / 64;                  // waves along n (64 rows each)
  static constexpr int WK = 8 / WM;                  // waves along k
  static constexpr int TK = K / WK / 32;             // 32-col MFMA tiles per wave along k
  static constexpr int BM = 32;                      // m rows per block
  static constexpr int RA = N * 2, RB = K * 2;       // image row bytes
  static constexpr int A_BYTES = BM * RA, B_BYTES = BM * RB;
  static constexpr int Z_BYTES = PRO ? A_BYTES : 0;  // the z image (PRO)
  static constexpr int SLOT = A_BYTES + Z_BYTES + B_BYTES;
  static constexpr int NST = PRO ? 3 : 4;
  static constexpr int PA = A_BYTES / 1024 / 8, PB = B_BYTES / 1024 / 8;   // DMA pieces per wave per block
  static constexpr int P = PA + (PRO ? PA : 0) + PB;
  static constexpr int CH = A_BYTES / 16 / NT;       // PRO: A chunks per thread per block = g_z stores per wave
  static_assert(TK >= 1 && A_BYTES % 8192 == 0 && B_BYTES % 8192 == 0 && SLOT * NST <= 147456, "shape");
};

// vmcnt bound before block i of a weight-stationary dW ring: the DMA pieces of the (NST - 2) later blocks plus the
// PRO stores issued after block i's DMA (min(i, NST - 1) blocks' worth: fewer while the ring fills).
template <int NST, int P, int S>
__device__ __forceinline__ void wsd_wait(int64_t i) {
  if constexpr (S == 0) {
    wait_vm<(NST - 2) * P>();
  } else {
    static_assert(NST == 2 || NST == 3, "wsd_wait");
    if (i == 0) wait_vm<(NST - 2) * P>();
    else if (NST == 3 && i == 1) wait_vm<(NST - 2) * P + S>();
    else wait_vm<(NST - 2) * P + (NST - 1) * S>();
  }
}

__device__ __forceinline__ int wsd_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

struct WsdPro {   // the PRO variant's extra operands (unused otherwise)
  const void* z;
  int64_t ldz;
  const float* slope;
  void* gz;          // g_z output [M, N] (ld ldgz)
  int64_t ldgz;
  float* pcol;       // [N][gridDim.x] column sums of g_z
  float* ps;         // [gridDim.x] slope sums
  char* dump;        // 16-B store target of the lanes whose rows are past M (every wave issues the same stores)
  const void* yalt = nullptr;   // bf16 zy: y = prelu(z) of a forward without accum; read in place of z when slope > 0
};

template <int N, int K, bool PRO>
__global__ __launch_bounds__(512, 1) void k_wsd_bf16(const uint16_t* __restrict__ A, int64_t lda,
                                                     const uint16_t* __restrict__ B1, int64_t ldb1,
                                                     const uint16_t* __restrict__ B2, int64_t ldb2, int64_t K1,
                                                     int64_t M, float* __restrict__ slab, int64_t ld_slab,
                                                     bool nt_in, WsdPro pro) {
  using C = WsdCfg<N, K, PRO>;
  constexpr int NST = C::NST;
  extern __shared__ __attribute__((aligned(16))) char wsd_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WM, wk = wave / C::WM;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;

  auto tid_o = [&]() {   // opaque: keeps the per-lane DMA offsets from being hoisted into registers
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto dma = [&](const void* src, void* dst) {
    if (nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  const int k1 = (int)K1;
  const float sl = PRO ? pro.slope[0] : 0.0f;
  const bool zy = PRO && pro.yalt != nullptr && sl > 0.0f;   // (wave-uniform)
  const uint16_t* zsrc = static_cast<const uint16_t*>(zy ? pro.yalt : pro.z);
  auto issue = [&](int64_t i) {
    char* base = wsd_smem + (int)(i % NST) * C::SLOT;
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const int ln = tid_o() & 63;
    const uint16_t* ab = A + r0 * lda;
    const uint16_t* b1 = B1 + r0 * ldb1;
    const uint16_t* b2 = B2 + r0 * ldb2;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / C::RA;
      const int c = ((off % C::RA) >> 4) ^ wsd_swz(r);
      r = r < rmax ? r : rmax;                       // (rows past M are zeroed in LDS before use)
      dma(ab + (r * (int)lda + c * 8), base + piece * 1024);
      if constexpr (PRO)                             // z: the same rows and swizzle, the image beside A
        dma(zsrc + (r0 + r) * pro.ldz + c * 8, base + C::A_BYTES + piece * 1024);
    }
#pragma unroll
    for (int q = 0; q < C::PB; ++q) {
      const int piece = wave * C::PB + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / C::RB;
      const int c = ((off % C::RB) >> 4) ^ wsd_swz(r);
      r = r < rmax ? r : rmax;
      const int k = c * 8;
      dma(k < k1 ? b1 + (r * (int)ldb1 + k) : b2 + (r * (int)ldb2 + (k - k1)),
          base + C::A_BYTES + C::Z_BYTES + piece * 1024);
    }
  };
  // PRO: per-thread partial sums over every block of this workgroup (fixed chunks -> fixed columns)
  float csum[PRO ? C::CH : 1][8];
  float ssum = 0.0f;
#pragma unroll
  for (int q = 0; q < (PRO ? C::CH : 1); ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) csum[q][j] = 0.0f;

  f32x16 acc[2][C::TK];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < C::TK; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  // per-lane byte offsets of the two transposed reads of each fragment (k-step kb adds 16 rows):
  // lane 4q + p of 16-lane group g reads rows 8 (g >> 1) + 4 half + q, columns cb + 16 (g & 1) + 4p .. + 3
  const int g = lane >> 4, q4 = (lane >> 2) & 3, pp = lane & 3;
  auto tr_off = [&](int rowbytes, int row, int col) {   // col: first of 4 bf16 read by the lane
    return rowbytes * row + 16 * ((col >> 3) ^ wsd_swz(row)) + 2 * (col & 7);
  };
  const char* lds = wsd_smem;
  auto tr = [&](int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + off)); };

#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < my) issue(i);

  for (int64_t i = 0; i < my; ++i) {
    if (i + NST - 2 < my) wsd_wait<NST, C::P, PRO ? C::CH : 0>(i); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();                  // block i landed for every wave; slot of block i-1 is free
    asm volatile("" ::: "memory");
    if (i + NST - 1 < my) issue(i + NST - 1);
    const int sbase = (int)(i % NST) * C::SLOT;
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    if (r0 + C::BM > M) {                          // the partial last block: zero its rows past M
      const int valid = (int)(M - r0);
      uint4* p = reinterpret_cast<uint4*>(wsd_smem + sbase);
      for (int ch = tid; ch < C::SLOT / 16; ch += C::NT) {
        const int ob = ch * 16;
        const int inb = ob >= C::A_BYTES + C::Z_BYTES;
        const int row = inb ? (ob - C::A_BYTES - C::Z_BYTES) / C::RB : (ob % C::A_BYTES) / C::RA;
        if (row >= valid) p[ch] = make_uint4(0u, 0u, 0u, 0u);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr (PRO) {   // g_z in place of g_y, its store, the partial sums (zeroed rows contribute 0)
#pragma unroll
      for (int q = 0; q < C::CH; ++q) {
        const int ch = q * C::NT + tid;
        const int row = ch / (C::RA / 16);
        const int c = (ch % (C::RA / 16)) ^ wsd_swz(row);   // logical 8-column chunk
        uint4* pa = reinterpret_cast<uint4*>(wsd_smem + sbase + ch * 16);
        const uint4 gy = *pa, zz = *reinterpret_cast<const uint4*>(wsd_smem + sbase + C::A_BYTES + ch * 16);
        const uint32_t gw[4] = {gy.x, gy.y, gy.z, gy.w}, zw[4] = {zz.x, zz.y, zz.z, zz.w};
        uint32_t ow[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          float o2[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float g = h ? bf_hi(gw[w]) : bf_lo(gw[w]);
            const float zv = h ? bf_hi(zw[w]) : bf_lo(zw[w]);
            const bool pos = zv > 0.0f;
            o2[h] = pos ? g : __fmul_rn(sl, g);
            csum[q][2 * w + h] = __fadd_rn(csum[q][2 * w + h], o2[h]);
            if (!pos) ssum = __fadd_rn(ssum, __fmul_rn(zv, g));
          }
          ow[w] = pack_bf2(o2[0], o2[1]);
        }
        const uint4 o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        *pa = o;
        const int64_t gr = r0 + row;
        uint16_t* gzp = static_cast<uint16_t*>(pro.gz) + gr * pro.ldgz + c * 8;
        uint4* dst = gr < M ? reinterpret_cast<uint4*>(gzp) : reinterpret_cast<uint4*>(pro.dump + (int64_t)ch * 16);
        *dst = o;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                // every thread's g_z chunks are in the image
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < C::BM / 16; ++kb) {
      bf16x8 fa[2], fb[C::TK];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int col = wm * 64 + t * 32 + 16 * (g & 1) + 4 * pp;
        const int row = 16 * kb + 8 * (g >> 1) + q4;
        const bf16x4 a0 = tr(sbase + tr_off(C::RA, row, col)), a1 = tr(sbase + tr_off(C::RA, row + 4, col));
        fa[t] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int t = 0; t < C::TK; ++t) {
        const int col = wk * (C::TK * 32) + t * 32 + 16 * (g & 1) + 4 * pp;
        const int row = 16 * kb + 8 * (g >> 1) + q4;
        const int bb = sbase + C::A_BYTES + C::Z_BYTES;
        const bf16x4 b0 = tr(bb + tr_off(C::RB, row, col)), b1 = tr(bb + tr_off(C::RB, row + 4, col));
        fb[t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < C::TK; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the slot are done
  }
  if constexpr (PRO) {   // fixed-order workgroup sums: column n over the 32 image rows, the slope over the threads
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* red = reinterpret_cast<float*>(wsd_smem);   // [NT][CH * 8], then [NT] slope partials
#pragma unroll
    for (int q = 0; q < C::CH; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[tid * (C::CH * 8) + q * 8 + j] = csum[q][j];
    red[C::NT * C::CH * 8 + tid] = ssum;
    __syncthreads();
    constexpr int CPR = C::RA / 16;   // chunks per image row
    for (int n = tid; n < N; n += C::NT) {
      const int c = n >> 3, j = n & 7;
      float tot = 0.0f;
      for (int row = 0; row < C::BM; ++row) {
        const int ch = row * CPR + (c ^ wsd_swz(row));
        tot = __fadd_rn(tot, red[(ch % C::NT) * (C::CH * 8) + (ch / C::NT) * 8 + j]);
      }
      pro.pcol[(int64_t)n * gridDim.x + blockIdx.x] = tot;
    }
    float* sr = red + C::NT * C::CH * 8;
    for (int off = C::NT / 2; off > 0; off >>= 1) {
      __syncthreads();
      if (tid < off) sr[tid] = __fadd_rn(sr[tid], sr[tid + off]);
    }
    if (tid == 0) pro.ps[blockIdx.x] = zy ? __fdiv_rn(sr[0], sl) : sr[0];
  }
  // this workgroup's slab [N][ld_slab] (the caller offsets slab to its column block)
  float* out = slab + (int64_t)blockIdx.x * N * ld_slab;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < C::TK; ++tn) {
      const int k = wk * (C::TK * 32) + tn * 32 + li;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        out[n * ld_slab + k] = acc[tm][tn][e];
      }
    }
}

// zy fallback (shapes the PRO kernel does not take): z restored in place from y where the forward skipped it —
// z = y > 0 ? y : bf16(y / slope) when slope > 0 (otherwise the forward wrote z and nothing changes)
__global__ __launch_bounds__(256) void k_zy_restore(const uint16_t* __restrict__ y, int64_t ldy, uint16_t* z, int64_t ldz,
                                                    int64_t M, int64_t N, const float* __restrict__ slope) {
  const float sl = slope[0];
  if (!(sl > 0.0f)) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M * N; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / N, c = i - r * N;
    const float v = bf2f(y[r * ldy + c]);
    z[r * ldz + c] = v > 0.0f ? y[r * ldy + c] : (uint16_t)f2bf(__fdiv_rn(v, sl));
  }
}

// k_wsd_f32 — the fp32 weight gradient in the same streaming form (split mode: six bf16 products per pair, the
// k_gemm_tn_partial arithmetic).  16-row m-blocks of A and B (fp32, linear images) stream HBM -> LDS by DMA into
// a 3-deep ring; per block one pass splits both into three bf16 planes (each element once per CU, into
// swizzled m-major plane images read by ds_read_b64_tr_b16), then each wave runs its 2 x TK tiles x 6 products.
// PRO (N = 256: every thread splits exactly one 8-column group of A per block): A is DMA'd as g_y with z beside it;
// the split pass forms g_z = z > 0 ? g_y : slope * g_y (k_rows_bwd<0>'s arithmetic), stores it (fp32, the dX GEMM's
// operand), keeps the column / slope partial sums, then splits g_z — g_w bit-identical to the two-pass form.  The z
// image costs the ring one slot (2 deep).
template <int N, int K, bool PRO = false>
struct WsdF32Cfg {
  static constexpr int NT = 512;
  static constexpr int WM = N / 64, WK = 8 / WM, TK = K / WK / 32;
  static constexpr int BM = 16;                              // one 16-deep MFMA k-step per block
  static constexpr int A_BYTES = BM * N * 4, B_BYTES = BM * K * 4;
  static constexpr int Z_BYTES = PRO ? A_BYTES : 0;
  static constexpr int SLOT = A_BYTES + Z_BYTES + B_BYTES;
  static constexpr int NST = PRO ? 2 : 3;
  static constexpr int PA_ROW = N * 2, PB_ROW = K * 2;       // plane image row bytes (bf16)
  static constexpr int PA_BYTES = BM * PA_ROW, PB_BYTES = BM * PB_ROW;   // one plane
  static constexpr int PLANES = 3 * (PA_BYTES + PB_BYTES);
  static constexpr int LDS = SLOT * NST + PLANES;
  static constexpr int PA = A_BYTES / 1024 / 8, PB = B_BYTES / 1024 / 8;
  static constexpr int P = PA + (PRO ? PA : 0) + PB;
  static constexpr int CA = BM * N / 4;                      // A float4 groups (thread t: t, t + NT, ...)
  static constexpr int S = PRO ? CA / NT : 0;                // g_z stores (16 B) per thread per block
  static_assert(TK >= 1 && A_BYTES % 8192 == 0 && B_BYTES % 8192 == 0 && LDS <= 163840, "shape");
  static_assert(!PRO || (CA % NT == 0 && CA / NT <= 2 && NT % (N / 4) == 0), "PRO: fixed columns per thread");
};

template <int N, int K, bool PRO>
__global__ __launch_bounds__(512, 1) void k_wsd_f32(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ B1, int64_t ldb1,
                                                    const float* __restrict__ B2, int64_t ldb2, int64_t K1, int64_t M,
                                                    float* __restrict__ slab, int64_t ld_slab, bool nt_in,
                                                    WsdPro pro) {
  using C = WsdF32Cfg<N, K, PRO>;
  constexpr int NST = C::NST;
  extern __shared__ __attribute__((aligned(16))) char wsdf_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WM, wk = wave / C::WM;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;
  char* const planes = wsdf_smem + C::SLOT * NST;

  auto tid_o = [&]() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto dma = [&](const void* src, void* dst) {
    if (nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  const int k1 = (int)K1;
  auto issue = [&](int64_t i) {
    char* base = wsdf_smem + (int)(i % NST) * C::SLOT;
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const int ln = tid_o() & 63;
    const float* ab = A + r0 * lda;
    const float* b1 = B1 + r0 * ldb1;
    const float* b2 = B2 + r0 * ldb2;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (N * 4);
      r = r < rmax ? r : rmax;                       // (rows past M are zeroed at the split)
      dma(ab + (r * (int)lda + (off % (N * 4)) / 4), base + piece * 1024);
      if constexpr (PRO)
        dma(static_cast<const float*>(pro.z) + (r0 + r) * pro.ldz + (off % (N * 4)) / 4,
            base + C::A_BYTES + piece * 1024);
    }
#pragma unroll
    for (int q = 0; q < C::PB; ++q) {
      const int piece = wave * C::PB + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (K * 4);
      r = r < rmax ? r : rmax;
      const int k = (off % (K * 4)) / 4;
      dma(k < k1 ? b1 + (r * (int)ldb1 + k) : b2 + (r * (int)ldb2 + (k - k1)),
          base + C::A_BYTES + C::Z_BYTES + piece * 1024);
    }
  };
  float csum[4];
  float ssum = 0.0f;
  const float sl = PRO ? pro.slope[0] : 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) csum[j] = 0.0f;

  f32x16 acc[2][C::TK];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < C::TK; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  const int g = lane >> 4, q4 = (lane >> 2) & 3, pp = lane & 3;
  auto tr_off = [&](int rowbytes, int row, int col) {
    return rowbytes * row + 16 * ((col >> 3) ^ wsd_swz(row)) + 2 * (col & 7);
  };
  auto tr = [&](int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(wsdf_smem + off)); };

#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < my) issue(i);

  for (int64_t i = 0; i < my; ++i) {
    if (i + NST - 2 < my) {
      wsd_wait<NST, C::P, C::S>(i);
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();   // block i landed for every wave; slot i-1 and the plane images are free
    asm volatile("" ::: "memory");
    if (i + NST - 1 < my) issue(i + NST - 1);
    const char* fbase = wsdf_smem + (int)(i % NST) * C::SLOT;
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int valid = M - r0 < C::BM ? (int)(M - r0) : C::BM;
    {   // split both fp32 images into three bf16 planes, one float4 (half a 16-B plane chunk) per lane and step:
        // consecutive lanes read consecutive 16-B pieces (conflict-free; 32 B per lane was 2-way conflicted)
      const int t = tid_o();
      constexpr int CA = C::CA, CT = C::BM * (N + K) / 4;   // float4 groups
#pragma unroll
      for (int q = 0; q < (CT + C::NT - 1) / C::NT; ++q) {
        const int grp = q * C::NT + t;
        if (CT % C::NT != 0 && grp >= CT) break;
        const bool isA = grp < CA;
        const int e0 = (isA ? grp : grp - CA) * 4;
        const int row = isA ? e0 / N : e0 / K, col = isA ? e0 % N : e0 % K;   // constant divisors: shifts
        const float* src = reinterpret_cast<const float*>(fbase + (isA ? 0 : C::A_BYTES + C::Z_BYTES)) + e0;
        float4 v = *reinterpret_cast<const float4*>(src);
        if (row >= valid) v = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (PRO) {
          if (isA) {   // g_z from g_y and z; its store; the partial sums (columns fixed per thread)
            const float* zs = reinterpret_cast<const float*>(fbase + C::A_BYTES) + e0;
            float4 z4 = *reinterpret_cast<const float4*>(zs);
            if (row >= valid) z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            float gg[4] = {v.x, v.y, v.z, v.w};
            const float zz[4] = {z4.x, z4.y, z4.z, z4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const bool pos = zz[j] > 0.0f;
              const float o = pos ? gg[j] : __fmul_rn(sl, gg[j]);
              csum[j] = __fadd_rn(csum[j], o);
              if (!pos) ssum = __fadd_rn(ssum, __fmul_rn(zz[j], gg[j]));
              gg[j] = o;
            }
            v = make_float4(gg[0], gg[1], gg[2], gg[3]);
            const int64_t gr = r0 + row;
            float* gzp = gr < M ? static_cast<float*>(pro.gz) + gr * pro.ldgz + col
                                : reinterpret_cast<float*>(pro.dump + (int64_t)t * 32 + 16 * q);
            *reinterpret_cast<float4*>(gzp) = v;
          }
        }
        uint2 o[3];
        split4(v, o);
        const int prow = isA ? C::PA_ROW : C::PB_ROW;
        char* pl = planes + (isA ? 0 : 3 * C::PA_BYTES);
        const int pbytes = isA ? C::PA_BYTES : C::PB_BYTES;
        const int off = prow * row + 16 * ((col >> 3) ^ wsd_swz(row)) + 8 * ((col >> 2) & 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(pl + p * pbytes + off) = o[p];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int pa0 = C::SLOT * NST, pb0 = pa0 + 3 * C::PA_BYTES;
    bf16x8 fa[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int col = wm * 64 + t * 32 + 16 * (g & 1) + 4 * pp;
      const int row = 8 * (g >> 1) + q4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int o = pa0 + p * C::PA_BYTES;
        const bf16x4 a0 = tr(o + tr_off(C::PA_ROW, row, col)), a1 = tr(o + tr_off(C::PA_ROW, row + 4, col));
        fa[t][p] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int tn = 0; tn < C::TK; ++tn) {
      bf16x8 fb[3];
      const int col = wk * (C::TK * 32) + tn * 32 + 16 * (g & 1) + 4 * pp;
      const int row = 8 * (g >> 1) + q4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int o = pb0 + p * C::PB_BYTES;
        const bf16x4 b0 = tr(o + tr_off(C::PB_ROW, row, col)), b1 = tr(o + tr_off(C::PB_ROW, row + 4, col));
        fb[p] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {   // k_gemm_tn_partial's order: smallest terms first
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][2], fb[0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[2], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[0], acc[tm][tn], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (PRO) {   // fixed-order workgroup sums: column n over the threads that own it, the slope over all
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* red = reinterpret_cast<float*>(wsdf_smem);   // [NT][4], then [NT] slope partials
    *reinterpret_cast<float4*>(red + tid * 4) = make_float4(csum[0], csum[1], csum[2], csum[3]);
    red[C::NT * 4 + tid] = ssum;
    __syncthreads();
    for (int n = tid; n < N; n += C::NT) {   // thread t owns columns (t % (N / 4)) * 4 .. + 3
      float tot = 0.0f;
      for (int m = 0; m < C::NT / (N / 4); ++m) tot = __fadd_rn(tot, red[(m * (N / 4) + (n >> 2)) * 4 + (n & 3)]);
      pro.pcol[(int64_t)n * gridDim.x + blockIdx.x] = tot;
    }
    float* sr = red + C::NT * 4;
    for (int off = C::NT / 2; off > 0; off >>= 1) {
      __syncthreads();
      if (tid < off) sr[tid] = __fadd_rn(sr[tid], sr[tid + off]);
    }
    if (tid == 0) pro.ps[blockIdx.x] = sr[0];
  }
  float* out = slab + (int64_t)blockIdx.x * N * ld_slab;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < C::TK; ++tn) {
      const int k = wk * (C::TK * 32) + tn * 32 + li;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        out[n * ld_slab + k] = acc[tm][tn][e];
      }
    }
}

// k_wsp_f32 — k_wsd_f32 at N = K = 256 (the GIN width) as a two-stage software pipeline: iteration i runs the MFMAs
// of block i on plane buffer i & 1 and the split (PRO: the g_z formation, its store, the partial sums) of block i + 1
// into plane buffer (i + 1) & 1 — independent work, so one barrier per block.  Waves 0-3 split first and waves 4-7
// multiply first: the two waves sharing a SIMD (w, w + 4) run the VALU split and the MFMAs side by side instead of
// both splitting, then both multiplying (MI355X_MICROARCH.md, "try a stagger").
// The fp32 staging is ONE slot (g_y | z | B, 48 KB): wave w splits exactly rows 2 w, 2 w + 1 of each image, which
// is what its own DMA pieces wrote, so a wave waits only on its own vmcnt before splitting and refills its slice
// with the next block as soon as its split has read it — no cross-wave hazard on the slot, and the fill has a whole
// block of MFMAs to land.  LDS: 48 KB slot + two 48 KB plane buffers = 144 KB.
// Same blocks per workgroup, planes and per-element products in the same order as k_wsd_f32: g_w and g_z are
// bit-identical to it; the bias / slope partials are summed in another fixed order (round 5: the lane -> column map
// that makes the slice reads conflict-free).  k_wsd_f32 no longer serves N = K = 256.
struct WspF32Cfg {
  static constexpr int N = 256, K = 256, NT = 512, WM = 4, TK = 4, BM = 16;
  static constexpr int A_BYTES = BM * N * 4, B_BYTES = BM * K * 4;
  template <bool PRO>
  static constexpr int slot() { return A_BYTES * (PRO ? 2 : 1) + B_BYTES; }
  static constexpr int PA_ROW = N * 2, PB_ROW = K * 2, PA_BYTES = BM * PA_ROW, PB_BYTES = BM * PB_ROW;
  static constexpr int PLANES = 3 * (PA_BYTES + PB_BYTES);
  template <bool PRO>
  static constexpr int lds() { return slot<PRO>() + 2 * PLANES; }
  static constexpr int PA = A_BYTES / 1024 / 8, PB = B_BYTES / 1024 / 8;   // DMA pieces per wave per image
  static_assert(2 * A_BYTES + B_BYTES + 2 * PLANES <= 163840 && BM * N / 8 == NT && BM * K / 8 == NT,
                "one A and one B group per thread");
  static_assert(PA * 1024 * 8 == A_BYTES && 32 * NT == A_BYTES, "thread t's 32 B lie in its own wave's pieces");
};

template <bool PRO>
__global__ __launch_bounds__(512, 1) void k_wsp_f32(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ B1, int64_t ldb1,
                                                    const float* __restrict__ B2, int64_t ldb2, int64_t K1, int64_t M,
                                                    float* __restrict__ slab, int64_t ld_slab, bool nt_in,
                                                    WsdPro pro) {
  using C = WspF32Cfg;
  constexpr int N = C::N, K = C::K;
  constexpr int Z_OFF = C::A_BYTES, B_OFF = C::A_BYTES * (PRO ? 2 : 1);
  extern __shared__ __attribute__((aligned(16))) char wsp_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % C::WM, wk = wave / C::WM;
  const int64_t nblk = (M + C::BM - 1) / C::BM;
  const int64_t G = gridDim.x;
  if ((int64_t)blockIdx.x >= nblk) return;
  const int64_t my = (nblk - 1 - blockIdx.x) / G + 1;
  char* const planes0 = wsp_smem + C::slot<PRO>();

  auto tid_o = [&]() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
    return t;
  };
  auto dma = [&](const void* src, void* dst) {
    if (nt_in) glds16_asm<true>(src, dst); else glds16_asm(src, dst);
  };
  const int k1 = (int)K1;
  auto issue = [&](int64_t i) {   // this wave's slice of block i: g_y [, z] and B pieces
    const int64_t r0 = ((int64_t)blockIdx.x + i * G) * C::BM;
    const int rmax = (int)(M - 1 - r0 < C::BM ? M - 1 - r0 : C::BM - 1);
    const int ln = tid_o() & 63;
    const float* ab = A + r0 * lda;
    const float* b1 = B1 + r0 * ldb1;
    const float* b2 = B2 + r0 * ldb2;
#pragma unroll
    for (int q = 0; q < C::PA; ++q) {
      const int piece = wave * C::PA + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (N * 4);
      r = r < rmax ? r : rmax;                       // (rows past M are zeroed at the split)
      dma(ab + (r * (int)lda + (off % (N * 4)) / 4), wsp_smem + piece * 1024);
      if constexpr (PRO)
        dma(static_cast<const float*>(pro.z) + (r0 + r) * pro.ldz + (off % (N * 4)) / 4,
            wsp_smem + Z_OFF + piece * 1024);
    }
#pragma unroll
    for (int q = 0; q < C::PB; ++q) {
      const int piece = wave * C::PB + q;
      const int off = piece * 1024 + ln * 16;
      int r = off / (K * 4);
      r = r < rmax ? r : rmax;
      const int k = (off % (K * 4)) / 4;
      dma(k < k1 ? b1 + (r * (int)ldb1 + k) : b2 + (r * (int)ldb2 + (k - k1)), wsp_smem + B_OFF + piece * 1024);
    }
  };
  float csum[4];
  float ssum = 0.0f;
  const float sl = PRO ? pro.slope[0] : 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) csum[j] = 0.0f;

  f32x16 acc[2][C::TK];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < C::TK; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  const int g = lane >> 4, q4 = (lane >> 2) & 3, pp = lane & 3;
  auto tr_off = [&](int rowbytes, int row, int col) {
    return rowbytes * row + 16 * ((col >> 3) ^ wsd_swz(row));
  };
  auto tr = [&](int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(wsp_smem + off)); };

  // block j (landed in this wave's slice) -> plane buffer j & 1, then the slice is refilled with block j + 1.
  // Wave w's slice is rows 2 w, 2 w + 1 of each image; lane l splits columns 4 l .. 4 l + 3 of both rows, so every
  // ds_read_b128 of the slice is 64 consecutive 16-B pieces (conflict-free; the earlier 32-B-per-lane reads were 2-way
  // conflicted: SQ_LDS_BANK_CONFLICT 32 % of the LDS-active cycles, profiles/r04/gpu_b/gemm_pmc2_sq.txt), and each
  // plane row half-chunk goes out as one ds_write_b64 (16 contiguous lanes = 128 contiguous bytes).
  auto split = [&](int64_t j) {
    wait_vm<0>();                                    // this wave's pieces of block j (and its older stores)
    char* pl = planes0 + (int)(j & 1) * C::PLANES;
    const int64_t r0 = ((int64_t)blockIdx.x + j * G) * C::BM;
    const int valid = M - r0 < C::BM ? (int)(M - r0) : C::BM;
    const int ln = tid_o() & 63;
    const int rw = 2 * wave;
    float4 va[2], vb[2], zv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = (rw + h) * (N * 4) + 16 * ln;   // N == K: the images share the row pitch
      va[h] = *reinterpret_cast<const float4*>(wsp_smem + o);
      vb[h] = *reinterpret_cast<const float4*>(wsp_smem + B_OFF + o);
      zv[h] = PRO ? *reinterpret_cast<const float4*>(wsp_smem + Z_OFF + o) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slice is read: refill it
    if (j + 1 < my) issue(j + 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = rw + h;
      if (row >= valid) va[h] = vb[h] = zv[h] = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (PRO) {   // g_z from g_y and z; its store; the partial sums (k_rows_bwd<0>'s arithmetic)
        float gg[4] = {va[h].x, va[h].y, va[h].z, va[h].w};
        const float zz[4] = {zv[h].x, zv[h].y, zv[h].z, zv[h].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool pos = zz[e] > 0.0f;
          const float o = pos ? gg[e] : __fmul_rn(sl, gg[e]);
          csum[e] = __fadd_rn(csum[e], o);
          if (!pos) ssum = __fadd_rn(ssum, __fmul_rn(zz[e], gg[e]));
          gg[e] = o;
        }
        va[h] = make_float4(gg[0], gg[1], gg[2], gg[3]);
        const int64_t gr = r0 + row;
        float* gzp = gr < M ? static_cast<float*>(pro.gz) + gr * pro.ldgz + 4 * ln
                            : reinterpret_cast<float*>(pro.dump + (int64_t)(wave * 64 + ln) * 32 + 16 * h);
        *reinterpret_cast<float4*>(gzp) = va[h];
      }
      const int off = C::PA_ROW * row + 16 * ((ln >> 1) ^ wsd_swz(row)) + 8 * (ln & 1);   // PA_ROW == PB_ROW
      uint2 o[3];
      split4(va[h], o);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(pl + p * C::PA_BYTES + off) = o[p];
      split4(vb[h], o);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(pl + 3 * C::PA_BYTES + p * C::PB_BYTES + off) = o[p];
    }
  };
  // block i's products from plane buffer i & 1 (k_wsd_f32's fragments and order)
  auto mfma = [&](int64_t i) {
    const int pa0 = C::slot<PRO>() + (int)(i & 1) * C::PLANES, pb0 = pa0 + 3 * C::PA_BYTES;
    bf16x8 fa[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int col = wm * 64 + t * 32 + 16 * (g & 1) + 4 * pp;
      const int row = 8 * (g >> 1) + q4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int o = pa0 + p * C::PA_BYTES + 2 * (col & 7);
        const bf16x4 a0 = tr(o + tr_off(C::PA_ROW, row, col)), a1 = tr(o + tr_off(C::PA_ROW, row + 4, col));
        fa[t][p] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
#pragma unroll
    for (int tn = 0; tn < C::TK; ++tn) {
      bf16x8 fb[3];
      const int col = wk * (C::TK * 32) + tn * 32 + 16 * (g & 1) + 4 * pp;
      const int row = 8 * (g >> 1) + q4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int o = pb0 + p * C::PB_BYTES + 2 * (col & 7);
        const bf16x4 b0 = tr(o + tr_off(C::PB_ROW, row, col)), b1 = tr(o + tr_off(C::PB_ROW, row + 4, col));
        fb[p] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][2], fb[0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[2], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[0], acc[tm][tn], 0, 0, 0);
      }
    }
  };

  issue(0);
  split(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int64_t i = 0; i + 1 < my; ++i) {
    __builtin_amdgcn_s_barrier();   // planes of block i written by every wave; those of block i - 1 read by every wave
    asm volatile("" ::: "memory");
    if (wave < 4) {
      split(i + 1);
      mfma(i);
    } else {
      mfma(i);
      split(i + 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's plane writes and fragment reads are done
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  mfma(my - 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (PRO) {   // fixed-order workgroup sums: column n = 4 l + e over the 8 waves' row pairs
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float* red = reinterpret_cast<float*>(wsp_smem);   // [NT][4], then [NT] slope partials
    *reinterpret_cast<float4*>(red + tid * 4) = make_float4(csum[0], csum[1], csum[2], csum[3]);
    red[C::NT * 4 + tid] = ssum;
    __syncthreads();
    for (int n = tid; n < N; n += C::NT) {
      float tot = 0.0f;
      for (int w = 0; w < C::NT / 64; ++w) tot = __fadd_rn(tot, red[(w * 64 + (n >> 2)) * 4 + (n & 3)]);
      pro.pcol[(int64_t)n * gridDim.x + blockIdx.x] = tot;
    }
    float* sr = red + C::NT * 4;
    for (int off = C::NT / 2; off > 0; off >>= 1) {
      __syncthreads();
      if (tid < off) sr[tid] = __fadd_rn(sr[tid], sr[tid + off]);
    }
    if (tid == 0) pro.ps[blockIdx.x] = sr[0];
  }
  float* out = slab + (int64_t)blockIdx.x * N * ld_slab;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < C::TK; ++tn) {
      const int k = wk * (C::TK * 32) + tn * 32 + li;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        out[n * ld_slab + k] = acc[tm][tn][e];
      }
    }
}

// Weight-stationary dW launch (HGIN_TN_WS = 0 / 1; default on): bf16, N in {128, 256}, K in {128, 256, 512},
// k1 a multiple of 8, 16-B aligned rows (leading dimensions multiples of 8, below 2^24).  Returns the slab
// count, or 0 when it does not apply.
bool wsd_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_TN_WS");
    return !(v && v[0] == '0');
  }();
  return on;
}

// HGIN_WSD_PRO = 0 keeps the separate PReLU-backward pass (k_rows_bwd<0>) ahead of the weight-stationary dW.
bool wsd_pro_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_WSD_PRO");
    return !(v && v[0] == '0');
  }();
  return on;
}

int64_t wsd_cus() {
  static const int64_t g = [] {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return int64_t(256);
    return (int64_t)prop.multiProcessorCount;
  }();
  return g;
}

template <int NV, int KV, bool PRO = false>
int64_t launch_wsd(const uint16_t* a, int64_t lda, const uint16_t* b1, int64_t ldb1, const uint16_t* b2,
                   int64_t ldb2, int64_t k1, int64_t M, float* slab, int64_t ld_slab, int64_t grid, hipStream_t s,
                   const WsdPro& pro = WsdPro{}) {
  constexpr bool nt = true;   // non-temporal DMA of the streamed rows (1-3 % faster, profiles/r02/gemm_ws_bf16.txt)
  constexpr int lds = WsdCfg<NV, KV, PRO>::SLOT * WsdCfg<NV, KV, PRO>::NST;
  auto kern = k_wsd_bf16<NV, KV, PRO>;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (attr != hipSuccess) return 0;
  HGIN_TRACE("k_wsd_bf16<%d,%d%s>", NV, KV, PRO ? ",prelu_bwd_fused" : "");
  kern<<<(unsigned)grid, 512, lds, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, slab, ld_slab, nt, pro);
  return grid;
}

template <int NV, int KV, bool PRO = false>
int64_t launch_wsd(const float* a, int64_t lda, const float* b1, int64_t ldb1, const float* b2, int64_t ldb2,
                   int64_t k1, int64_t M, float* slab, int64_t ld_slab, int64_t grid, hipStream_t s,
                   const WsdPro& pro = WsdPro{}) {
  constexpr bool nt = true;   // non-temporal DMA of the streamed rows (1-3 % faster, profiles/r02/gemm_ws_bf16.txt)
  if constexpr (NV == 256 && KV == 256) {   // the GIN width: the pipelined form (k_wsd_f32 measured 3-8 % slower
    auto kp = k_wsp_f32<PRO>;                 // here, profiles/r04/gpu_a/; removed from this shape in round 5)
    constexpr int plds = WspF32Cfg::lds<PRO>();
    static const hipError_t pattr = hipFuncSetAttribute(reinterpret_cast<const void*>(kp),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, plds);
    if (pattr != hipSuccess) return 0;
    HGIN_TRACE("k_wsp_f32<%d,%d%s>", NV, KV, PRO ? ",prelu_bwd_fused" : "");
    kp<<<(unsigned)grid, 512, plds, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, slab, ld_slab, nt, pro);
    return grid;
  } else {
    constexpr int lds = WsdF32Cfg<NV, KV, PRO>::LDS;
    auto kern = k_wsd_f32<NV, KV, PRO>;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (attr != hipSuccess) return 0;
    HGIN_TRACE("k_wsd_f32<%d,%d%s>", NV, KV, PRO ? ",prelu_bwd_fused" : "");
    kern<<<(unsigned)grid, 512, lds, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, slab, ld_slab, nt, pro);
    return grid;
  }
}

// One weight-stationary pass over output columns [c0, c0 + KV) of B = [b1 (k1 columns) | b2].
template <int NV, int KV, typename T>
int64_t wsd_cols(const T* a, int64_t lda, const T* b1, int64_t ldb1, int64_t k1, const T* b2,
                 int64_t ldb2, int64_t c0, int64_t M, float* slab, int64_t ld_slab, int64_t grid, hipStream_t s) {
  // the column block's two sources: [c0, k1) from b1, [max(c0, k1), c0 + KV) from b2
  const int64_t kk1 = k1 > c0 ? (k1 - c0 < KV ? k1 - c0 : KV) : 0;
  const T* p1 = kk1 > 0 ? b1 + c0 : b2;
  const int64_t l1 = kk1 > 0 ? ldb1 : ldb2;
  const T* p2 = kk1 < KV ? b2 + (c0 + kk1 - k1) : p1;
  const int64_t l2 = kk1 < KV ? ldb2 : l1;
  return launch_wsd<NV, KV>(a, lda, p1, l1, p2, l2, kk1, M, slab + c0, ld_slab, grid, s);
}

// Column passes of the PReLU-fused dW: [0, KV) with the fold (forms + stores g_z, the partial sums), then for K = 512
// at N = 256 [256, 512) as the plain kernel on the stored g_z — the same two passes, slabs and product order as the
// unfused K = 512 path, so g_w stays bit-identical to it.  N = 128, K = 512 (the readout's first Linear on
// [x_path | raw]) fits the whole 128 x 512 output in the registers of one pass (the 256 x 256 accumulator footprint):
// g_y, z and B are streamed once and nothing re-reads g_z; per output element the products and their order are the
// two-pass form's, so g_w is bit-identical to it as well.
template <typename T>
int64_t wsd_pro_passes(const T* gy, int64_t ldgy, const T* b1, int64_t ldb1, int64_t k1, const T* b2, int64_t ldb2,
                       int64_t M, int64_t N, int64_t K, float* slab, int64_t grid, const WsdPro& pro, hipStream_t s) {
  const int64_t KV = (K == 512 && N == 256) ? 256 : K;
  auto srcs = [&](int64_t c0, const T*& p1, int64_t& l1, const T*& p2, int64_t& l2, int64_t& kk1) {
    kk1 = k1 > c0 ? (k1 - c0 < KV ? k1 - c0 : KV) : 0;
    p1 = kk1 > 0 ? b1 + c0 : b2;
    l1 = kk1 > 0 ? ldb1 : ldb2;
    p2 = kk1 < KV ? b2 + (c0 + kk1 - k1) : p1;
    l2 = kk1 < KV ? ldb2 : l1;
  };
  const T* p1;
  const T* p2;
  int64_t l1, l2, kk1;
  srcs(0, p1, l1, p2, l2, kk1);
  int64_t g;
#define HGIN_PRO_PASS(NV, KVV) g = launch_wsd<NV, KVV, true>(gy, ldgy, p1, l1, p2, l2, kk1, M, slab, K, grid, s, pro);
  if (N == 256 && KV == 256) { HGIN_PRO_PASS(256, 256) }
  else if (N == 256) { HGIN_PRO_PASS(256, 128) }
  else if (KV == 512) { HGIN_PRO_PASS(128, 512) }
  else if (KV == 256) { HGIN_PRO_PASS(128, 256) }
  else { HGIN_PRO_PASS(128, 128) }
#undef HGIN_PRO_PASS
  if (!g || K != 512 || KV == 512) return g;
  srcs(256, p1, l1, p2, l2, kk1);
  const T* gz = static_cast<const T*>(pro.gz);
  if (N == 256) return launch_wsd<256, 256>(gz, pro.ldgz, p1, l1, p2, l2, kk1, M, slab + 256, K, grid, s);
  return launch_wsd<128, 256>(gz, pro.ldgz, p1, l1, p2, l2, kk1, M, slab + 256, K, grid, s);
}

// The PReLU-backward-fused weight-stationary dW (bf16, single column pass: N in {128, 256}, K in {128, 256}):
// g_w slabs + g_z + bias / slope partials in one launch.  Returns the slab count, or 0 when it does not apply.
template <typename T>
int64_t try_wsd_pro(const T* gy, int64_t ldgy, const T* b1, int64_t ldb1, int64_t k1, const T* b2, int64_t ldb2,
                    int64_t M, int64_t N, int64_t K, float* slab, int64_t max_slabs, const WsdPro& pro,
                    hipStream_t s) {
  if constexpr (sizeof(T) == 4) {   // fp32 (split mode): N in {128, 256}, K in {128, 256, 512}
    constexpr int64_t vw = 4;
    if (!wsd_enabled() || !wsd_pro_enabled() || !gemm_split_enabled() || M < 1 || (N != 128 && N != 256) ||
        (K != 128 && K != 256 && K != 512) || k1 % vw)
      return 0;
    auto ok = [](const void* p, int64_t ld) { return aligned16(p) && ld % vw == 0 && ld < (int64_t(1) << 24); };
    if (!ok(gy, ldgy) || !ok(pro.z, pro.ldz) || !ok(pro.gz, pro.ldgz) || (k1 > 0 && !ok(b1, ldb1)) ||
        (k1 < K && !ok(b2, ldb2)))
      return 0;
    int64_t grid = wsd_cus();
    const int64_t nblk = ceil_div(M, (int64_t)16);
    if (grid > nblk) grid = nblk;
    if (grid > max_slabs) grid = max_slabs;
    return wsd_pro_passes<T>(gy, ldgy, b1, ldb1, k1, b2, ldb2, M, N, K, slab, grid, pro, s);
  } else {
    constexpr int64_t vw = 8;
    if (!wsd_enabled() || !wsd_pro_enabled() || M < 1 || (N != 128 && N != 256) ||
        (K != 128 && K != 256 && K != 512) || k1 % vw)
      return 0;
    auto ok = [](const void* p, int64_t ld) { return aligned16(p) && ld % vw == 0 && ld < (int64_t(1) << 24); };
    if (!ok(gy, ldgy) || !ok(pro.z, pro.ldz) || !ok(pro.gz, pro.ldgz) || (k1 > 0 && !ok(b1, ldb1)) ||
        (k1 < K && !ok(b2, ldb2)))
      return 0;
    int64_t grid = wsd_cus();
    const int64_t nblk = ceil_div(M, (int64_t)32);
    if (grid > nblk) grid = nblk;
    if (grid > max_slabs) grid = max_slabs;
    return wsd_pro_passes<T>(gy, ldgy, b1, ldb1, k1, b2, ldb2, M, N, K, slab, grid, pro, s);
  }
}

template <typename T>
int64_t try_wsd(const T* a, int64_t lda, const T* b1, int64_t ldb1, int64_t k1, const T* b2, int64_t ldb2,
                int64_t M, int64_t N, int64_t K, float* slab, int64_t max_slabs, hipStream_t s) {
  constexpr int64_t vw = 16 / sizeof(T);   // elements per 16-B chunk
  if (!wsd_enabled() || M < 1 || (N != 128 && N != 256) || (K != 128 && K != 256 && K != 512) || k1 % vw) return 0;
  if (sizeof(T) == 4 && !gemm_split_enabled()) return 0;   // the exact-f32 MFMA mode keeps the tiled kernel
  auto ok = [](const void* p, int64_t ld) { return aligned16(p) && ld % vw == 0 && ld < (int64_t(1) << 24); };
  if (!ok(a, lda) || (k1 > 0 && !ok(b1, ldb1)) || (k1 < K && !ok(b2, ldb2))) return 0;
  const int64_t nblk = ceil_div(M, (int64_t)(sizeof(T) == 2 ? 32 : 16));
  int64_t grid = wsd_cus();
  if (grid > nblk) grid = nblk;
  if (grid > max_slabs) grid = max_slabs;
  // K = 512 (the first layer's [aggregate | x_dst]): two 256-column passes into the same slabs (A read twice,
  // B once; the tiled kernel reads both twice)
  if (K == 512) {
    if (N == 256) {
      if (!wsd_cols<256, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s)) return 0;
      return wsd_cols<256, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 256, M, slab, K, grid, s);
    }
    if (!wsd_cols<128, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s)) return 0;
    return wsd_cols<128, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 256, M, slab, K, grid, s);
  }
  if (N == 256 && K == 256) return wsd_cols<256, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s);
  if (N == 256 && K == 128) return wsd_cols<256, 128>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s);
  if (N == 128 && K == 256) return wsd_cols<128, 256>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s);
  return wsd_cols<128, 128>(a, lda, b1, ldb1, k1, b2, ldb2, 0, M, slab, K, grid, s);
}

bool tn_is_small(int64_t N, int64_t K) { return N < 16 || K < 16; }

// Workgroups a split-M launch aims for (<= 1024 = the workspace sizing target).  768 = one resident round at 3
// workgroups per CU: measured (profiles/r01_gemm_variants_*.txt) 1.35x faster than 1024 (1.33 rounds, the last one a
// third full) for the bf16 kernel, 4-6 % for fp32.
constexpr int64_t tn_target_wgs() { return 768; }

int64_t tn_splits(int64_t M, int64_t N, int64_t K, int64_t stage_rows = kTnBM, int64_t target = 1024) {
  int64_t S;
  if (tn_is_small(N, K)) {
    S = ceil_div(M, 128);          // >= 128 rows per workgroup: small graphs (the F1 batches) still get
                                   // dozens of workgroups instead of a handful of long serial loops
    if (S > 1024) S = 1024;
  } else {
    const int64_t tiles = ceil_div(N, 128) * ceil_div(K, 128);
    S = ceil_div(target, tiles);                           // ~3-4 workgroups per CU
    const int64_t max_s = ceil_div(M, 8 * stage_rows);     // keep >= 8 stages per split
    if (S > max_s) S = max_s;
  }
  return S < 1 ? 1 : S;
}

// Slabs the workspace holds: the split count, or one per CU (up to 256) for the weight-stationary bf16 dW.
int64_t tn_ws_slabs(int64_t M, int64_t N, int64_t K) {
  const int64_t S = tn_splits(M, N, K);
  if (tn_is_small(N, K) || N > 256 || K > 512) return S;
  const int64_t w = ceil_div(M > 0 ? M : 1, 32) < 256 ? ceil_div(M > 0 ? M : 1, 32) : 256;
  return S > w ? S : w;
}

size_t tn_ws_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t S = tn_ws_slabs(M, N, K);
  return align_up(sizeof(float) * (size_t)(S * N * K), 256) + align_up(sizeof(float) * (size_t)(ceil_div(S, kSlabGroup) * N * K), 256);
}

// Prologue partials of hgin_gin_mlp_bwd_w_*: [N][S] column sums + [N tiles][S] slope sums.
size_t pro_ws_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t S = tn_splits(M, N, K);
  return align_up(sizeof(float) * (size_t)(N * S), 256) + align_up(sizeof(float) * (size_t)(ceil_div(N, 32) * S), 256);
}

// Final fixed-order sums of the prologue partials (one workgroup per column; one for the slope).
__global__ __launch_bounds__(256) void k_pro_final(const float* __restrict__ pcol, const float* __restrict__ ps,
                                                   int64_t S, int64_t n_ps, float* __restrict__ g_bias,
                                                   float* __restrict__ g_prelu) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  const int64_t n = c < (int)gridDim.x - 1 ? S : n_ps;
  const float* p = c < (int)gridDim.x - 1 ? pcol + (int64_t)c * S : ps;
  float s = 0.0f;
  for (int64_t b = threadIdx.x; b < n; b += 256) s = __fadd_rn(s, p[b]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] = __fadd_rn(red[threadIdx.x], red[threadIdx.x + off]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (c < (int)gridDim.x - 1) g_bias[c] = red[0];
    else g_prelu[0] = red[0];
  }
}

// Shared host path of hgin_gemm_tn_* (pro == NULL) and hgin_gin_mlp_bwd_w_* (pro: A = g_y, z, slope, ...).
template <typename T>
int gemm_tn_impl(const char* what, const T* a, int64_t lda, const T* b1, int64_t ldb1, int64_t k1, const T* b2,
                 int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out, int64_t ldo, void* workspace,
                 size_t workspace_bytes, hipStream_t s, const TnPro* pro_in, float* g_bias, float* g_prelu) {
  constexpr bool kHalf = sizeof(T) == 2;
  const size_t need = tn_ws_bytes(M, N, K);
  const size_t need_pro = pro_in ? pro_ws_bytes(M, N, K) : 0;
  if (workspace_bytes < need + need_pro || !workspace) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need + need_pro);
    return HGIN_E_WORKSPACE;
  }
  if (M == 0) {
    for (int64_t n = 0; n < N; ++n) {
      int rc = memset_async(out + n * ldo, 0, sizeof(float) * (size_t)K, s, what);
      if (rc) return rc;
    }
    if (pro_in) {
      int rc = memset_async(g_bias, 0, sizeof(float) * (size_t)N, s, what);
      if (rc == HGIN_OK) rc = memset_async(g_prelu, 0, sizeof(float), s, what);
      return rc;
    }
    return HGIN_OK;
  }
  HGIN_ARG_CHECK(a && lda >= N && (k1 == 0 || (b1 && ldb1 >= k1)) && (k1 == K || (b2 && ldb2 >= K - k1)),
                 "%s: bad operand", what);
  constexpr int64_t vw = kHalf ? 8 : 4;   // elements per 16 B
  bool vec = aligned16(a) && lda % vw == 0 && (k1 == 0 || (aligned16(b1) && ldb1 % vw == 0)) &&
             (k1 == K || (aligned16(b2) && ldb2 % vw == 0)) && k1 % vw == 0;
  if (pro_in) vec = vec && aligned16(pro_in->z) && pro_in->ldz % vw == 0;
  const bool small = tn_is_small(N, K);
  const int64_t stage = (kHalf && !small) ? kTnBMh : kTnBM;
  const int64_t S = tn_splits(M, N, K, stage, tn_target_wgs());   // <= the workspace's split count
  const int64_t rows = ceil_div(ceil_div(M, S), stage) * stage;
  int64_t S_eff = ceil_div(M, rows);
  const int64_t NK = N * K;
  float* slab = static_cast<float*>(workspace);
  float* part = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                         align_up(sizeof(float) * (size_t)(tn_ws_slabs(M, N, K) * NK), 256));
  TnPro pro{};
  if (pro_in) {
    pro = *pro_in;
    pro.pcol = reinterpret_cast<float*>(static_cast<char*>(workspace) + need);
    pro.ps = reinterpret_cast<float*>(static_cast<char*>(workspace) + need +
                                      align_up(sizeof(float) * (size_t)(N * tn_splits(M, N, K)), 256));
    pro.S = S_eff;
  }
  int64_t tile_n = 128;
  if (small) {
    HGIN_ARG_CHECK(!pro_in, "%s: no fused prologue for N or K < 16", what);
    HGIN_TRACE("k_tn_small<N%lld,K%lld>", (long long)N, (long long)K);
    k_tn_small<T><<<(unsigned)S_eff, 256, 0, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, (int)N, (int)K, rows, slab);
  } else if (int64_t g = (!pro_in && vec) ? try_wsd<T>(a, lda, b1, ldb1, k1, b2, ldb2, M, N, K, slab,
                                                        tn_ws_slabs(M, N, K), s)
                                          : 0) {
    S_eff = g;   // one slab per weight-stationary workgroup
  } else if constexpr (kHalf) {
    const int64_t tiles_n = ceil_div(N, 128);
    const TnGrid tg{128, tiles_n, tiles_n * ceil_div(K, 128), tiles_n * ceil_div(K, 128) * S_eff, xcd_remap_enabled()};
    dim3 grid((unsigned)(tg.xcd ? round_up8(tg.n_work) : tg.n_work));
    HGIN_ARG_CHECK(!pro_in, "%s: no fused prologue for bf16", what);
    HGIN_TRACE("k_gemm_tn_bf16<tr,N%lld,K%lld>", (long long)N, (long long)K);
    if (vec && N % 8 == 0 && K % 8 == 0)
      k_gemm_tn_bf16_tr<true><<<grid, 256, 0, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, N, K, rows, slab, tg);
    else
      k_gemm_tn_bf16_tr<false><<<grid, 256, 0, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, N, K, rows, slab, tg);
  } else {
    tile_n = N <= 32 ? 32 : 128;
    const int64_t tiles_n = ceil_div(N, tile_n);
    const TnGrid tg{tile_n, tiles_n, tiles_n * ceil_div(K, 128), tiles_n * ceil_div(K, 128) * S_eff,
                    xcd_remap_enabled()};
    dim3 grid((unsigned)(tg.xcd ? round_up8(tg.n_work) : tg.n_work));
    // register prefetch at 3 waves/SIMD (profiles/r01_tn_variants.txt: 12 % faster than the unpipelined
    // loop, 3-5 % faster than prefetch at 2 waves)
    const bool clean = vec && N % tile_n == 0 && K % 128 == 0 && k1 % 128 == 0;
    const bool split = gemm_split_enabled();
    HGIN_TRACE("k_gemm_tn_partial<%s,%s,N%lld,K%lld>",
               pro_in ? (pro_in->gz ? "prelu_bwd_fused+gz" : "prelu_bwd_fused") : "plain", split ? "split" : "mfma32",
               (long long)N, (long long)K);
#define HGIN_TN_LAUNCH(CLEAN, TNR, SPLIT, PRO, LATE, GZ)                                                           \
  k_gemm_tn_partial<CLEAN, TNR, SPLIT, PRO, LATE, GZ><<<grid, 256, 0, s>>>(a, lda, b1, ldb1, b2, ldb2, k1, M, N, K, \
                                                                            rows, vec, slab, tg, pro)
#define HGIN_TN_PRO(CLEAN, TNR, SPLIT)                                                \
  if (!pro_in) HGIN_TN_LAUNCH(CLEAN, TNR, SPLIT, false, false, false);                \
  else if (pro_in->gz) HGIN_TN_LAUNCH(CLEAN, TNR, SPLIT, true, false, true); /* (late z + gz spills) */ \
  else HGIN_TN_LAUNCH(CLEAN, TNR, SPLIT, true, true, false);
#define HGIN_TN_CLEAN(TNR, SPLIT) \
  if (clean) { HGIN_TN_PRO(true, TNR, SPLIT) } else { HGIN_TN_PRO(false, TNR, SPLIT) }
    if (tile_n == 32) {
      if (split) { HGIN_TN_CLEAN(32, true) } else { HGIN_TN_CLEAN(32, false) }
    } else {
      if (split) { HGIN_TN_CLEAN(128, true) } else { HGIN_TN_CLEAN(128, false) }
    }
#undef HGIN_TN_CLEAN
#undef HGIN_TN_PRO
#undef HGIN_TN_LAUNCH
  }
  const int64_t G = ceil_div(S_eff, kSlabGroup);
  if (slab_fused_enabled() && G <= kSlabMaxG) {
    const int64_t n_red = ceil_div(NK, kSlabCols);
    const int64_t n_pro = pro_in ? N + 1 : 0;
    k_slab_reduce<<<(unsigned)(n_red + n_pro), 256, 0, s>>>(slab, S_eff, NK, out, K, ldo, n_red, pro.pcol, pro.ps,
                                                           ceil_div(N, tile_n) * S_eff, g_bias, g_prelu);
    return check_launch(what);
  }
  dim3 g1((unsigned)ceil_div(ceil_div(NK, 4), 256), (unsigned)G);
  k_slab_reduce1<<<g1, 256, 0, s>>>(slab, S_eff, NK, part);
  k_slab_reduce2<<<(unsigned)ceil_div(NK, 256), 256, 0, s>>>(part, G, NK, out, K, ldo);
  if (pro_in)
    k_pro_final<<<(unsigned)(N + 1), 256, 0, s>>>(pro.pcol, pro.ps, S_eff, ceil_div(N, tile_n) * S_eff, g_bias, g_prelu);
  return check_launch(what);
}

template <typename T>
int gemm_tn_entry(const char* what, const T* a, int64_t lda, const T* b1, int64_t ldb1, int64_t k1, const T* b2,
                  int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out, int64_t ldo, void* workspace,
                  size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0 && k1 >= 0 && k1 <= K, "%s: bad sizes", what);
  HGIN_ARG_CHECK(N <= 65535 * 128 && K <= 65535 * 128, "%s: N/K too large", what);
  if (N == 0 || K == 0) return HGIN_OK;
  HGIN_ARG_CHECK(out && ldo >= K, "%s: bad output", what);
  return gemm_tn_impl<T>(what, a, lda, b1, ldb1, k1, b2, ldb2, M, N, K, out, ldo, workspace, workspace_bytes,
                         as_stream(stream), nullptr, nullptr, nullptr);
}

// hgin_gin_mlp_bwd_w_*: fp32 with an MFMA tile and no g_z requested -> the fused prologue; otherwise the
// PReLU backward into g_z (the caller's buffer, or workspace scratch) followed by the plain TN GEMM.
bool mlp_bwd_w_fused(int64_t N, int64_t K, size_t elem) { return elem == 4 && !tn_is_small(N, K); }

// the weight-stationary PRO kernel's partials: [N][slabs] column sums, [slabs] slope sums, the 16-B dump of every
// thread's out-of-range g_z stores (NT x CH chunks)
size_t wsd_pro_ws_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t S = tn_ws_slabs(M, N, K);
  return align_up(sizeof(float) * (size_t)(N * S), 256) + align_up(sizeof(float) * (size_t)S, 256) +
         align_up((size_t)16 * 512 * 2, 256);
}

size_t mlp_bwd_w_ws_bytes(int64_t M, int64_t N, int64_t K, size_t elem, bool have_gz) {
  if (mlp_bwd_w_fused(N, K, elem) && !have_gz) return tn_ws_bytes(M, N, K) + pro_ws_bytes(M, N, K);
  size_t pw = 0;
  hgin_prelu_bwd_workspace_size(M, N, &pw);
  const size_t two_pass = align_up(pw, 256) + tn_ws_bytes(M, N, K) + (have_gz ? 0 : align_up(elem * (size_t)(M * N), 256));
  const size_t pro = tn_ws_bytes(M, N, K) + wsd_pro_ws_bytes(M, N, K);
  const size_t tiled = tn_ws_bytes(M, N, K) + pro_ws_bytes(M, N, K);   // the tiled prologue storing g_z
  const size_t m = two_pass > pro ? two_pass : pro;
  return m > tiled ? m : tiled;
}

template <typename T>
int mlp_bwd_w_entry(const char* what, const T* g_y, int64_t ld_gy, const T* z, int64_t ldz, const float* prelu,
                    const T* b1, int64_t ldb1, int64_t k1, const T* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K,
                    float* g_w, int64_t ldw, float* g_prelu, float* g_bias, T* g_z, int64_t ld_gz, void* workspace,
                    size_t workspace_bytes, void* stream, const T* yalt = nullptr) {
  HGIN_ARG_CHECK(M >= 0 && N >= 0 && K >= 0 && k1 >= 0 && k1 <= K, "%s: bad sizes", what);
  HGIN_ARG_CHECK(N >= 1 && N <= 65535 * 128 && K >= 1 && K <= 65535 * 128, "%s: N/K out of range", what);
  HGIN_ARG_CHECK(prelu && g_prelu && g_bias && g_w && ldw >= K, "%s: NULL output / bad ldw", what);
  HGIN_ARG_CHECK(M == 0 || (g_y && ld_gy >= N && z && ldz >= N), "%s: bad g_y / z", what);
  HGIN_ARG_CHECK(!g_z || ld_gz >= N, "%s: ld_gz < N", what);
  const size_t need = mlp_bwd_w_ws_bytes(M, N, K, sizeof(T), g_z != nullptr);
  if (workspace_bytes < need || !workspace) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if (mlp_bwd_w_fused(N, K, sizeof(T)) && !g_z) {
    TnPro pro{z, ldz, prelu, nullptr, nullptr, 0};
    return gemm_tn_impl<T>(what, g_y, ld_gy, b1, ldb1, k1, b2, ldb2, M, N, K, g_w, ldw, workspace, workspace_bytes,
                           s, &pro, g_bias, g_prelu);
  }
  if (g_z && M > 0 && prelu && g_y && z) {   // the weight-stationary dW with the PReLU backward folded in
    char* ws = static_cast<char*>(workspace);
    const size_t tw = tn_ws_bytes(M, N, K);
    const int64_t S = tn_ws_slabs(M, N, K);
    WsdPro pro{z, ldz, prelu, g_z, ld_gz, reinterpret_cast<float*>(ws + tw), nullptr, nullptr, yalt};
    pro.ps = reinterpret_cast<float*>(ws + tw + align_up(sizeof(float) * (size_t)(N * S), 256));
    pro.dump = ws + tw + align_up(sizeof(float) * (size_t)(N * S), 256) + align_up(sizeof(float) * (size_t)S, 256);
    float* slab = reinterpret_cast<float*>(ws);
    if (const int64_t g = try_wsd_pro<T>(g_y, ld_gy, b1, ldb1, k1, b2, ldb2, M, N, K, slab, S, pro, s)) {
      const int64_t NK = N * K;
      const int64_t G = ceil_div(g, kSlabGroup);
      if (slab_fused_enabled() && G <= kSlabMaxG) {
        const int64_t n_red = ceil_div(NK, kSlabCols);
        k_slab_reduce<<<(unsigned)(n_red + N + 1), 256, 0, s>>>(slab, g, NK, g_w, K, ldw, n_red, pro.pcol, pro.ps, g,
                                                                 g_bias, g_prelu);
        return check_launch(what);
      }
      float* part = reinterpret_cast<float*>(ws + align_up(sizeof(float) * (size_t)(S * NK), 256));
      dim3 g1((unsigned)ceil_div(ceil_div(NK, 4), 256), (unsigned)G);
      k_slab_reduce1<<<g1, 256, 0, s>>>(slab, g, NK, part);
      k_slab_reduce2<<<(unsigned)ceil_div(NK, 256), 256, 0, s>>>(part, G, NK, g_w, K, ldw);
      k_pro_final<<<(unsigned)(N + 1), 256, 0, s>>>(pro.pcol, pro.ps, g, g, g_bias, g_prelu);
      return check_launch(what);
    }
    // fp32 shapes the weight-stationary kernels do not take (e.g. the readout's Linear(128, 32)): the tiled dW with
    // the prologue, its first-K-tile workgroups storing the g_z they form (no separate PReLU-backward pass).
    // HGIN_WSD_PRO=0 turns this fold off as well (the separate pass + plain dW below).
    if (wsd_pro_enabled() && mlp_bwd_w_fused(N, K, sizeof(T)) && ld_gz % 4 == 0) {
      TnPro pro2{z, ldz, prelu, nullptr, nullptr, 0};
      pro2.gz = reinterpret_cast<float*>(g_z);
      pro2.ldgz = ld_gz;
      if (tn_ws_bytes(M, N, K) + pro_ws_bytes(M, N, K) <= workspace_bytes)
        return gemm_tn_impl<T>(what, g_y, ld_gy, b1, ldb1, k1, b2, ldb2, M, N, K, g_w, ldw, workspace,
                               workspace_bytes, s, &pro2, g_bias, g_prelu);
    }
  }
  if (yalt && M > 0) {   // zy, a shape the PRO kernel did not take: restore z from y first (no-op when slope <= 0)
    if constexpr (sizeof(T) == 2) {
      const int64_t n = M * N;
      const unsigned nb = (unsigned)(ceil_div(n, 256) < 4096 ? ceil_div(n, 256) : 4096);
      k_zy_restore<<<nb, 256, 0, s>>>(yalt, N, const_cast<T*>(z), ldz, M, N, prelu);
      if (int rc = check_launch(what)) return rc;
    }
  }
  size_t pw = 0;
  hgin_prelu_bwd_workspace_size(M, N, &pw);
  char* ws = static_cast<char*>(workspace);
  const size_t tw = tn_ws_bytes(M, N, K);
  T* gz = g_z;
  int64_t ldg = ld_gz;
  if (!gz) {
    gz = reinterpret_cast<T*>(ws + align_up(pw, 256) + tw);
    ldg = N;
  }
  int rc;
  if constexpr (sizeof(T) == 2) {
    HGIN_ARG_CHECK(ldg == N, "%s: bf16 g_z must be dense (ld_gz == N)", what);
    rc = hgin_prelu_bwd_bf16(g_y, ld_gy, z, M, N, prelu, gz, g_prelu, g_bias, ws, pw, stream);
  } else {
    HGIN_ARG_CHECK(ldg == N, "%s: g_z must be dense (ld_gz == N)", what);
    rc = hgin_prelu_bwd_f32(g_y, ld_gy, z, M, N, prelu, gz, g_prelu, g_bias, ws, pw, stream);
  }
  if (rc) return rc;
  return gemm_tn_impl<T>(what, gz, ldg, b1, ldb1, k1, b2, ldb2, M, N, K, g_w, ldw, ws + align_up(pw, 256), tw, s,
                         nullptr, nullptr, nullptr);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_gemm_tn_workspace_size(int64_t M, int64_t N, int64_t K, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && M >= 0 && N >= 0 && K >= 0, "hgin_gemm_tn_workspace_size: bad args");
  *bytes = tn_ws_bytes(M, N, K);
  return HGIN_OK;
}

extern "C" int hgin_gemm_tn_f32(const float* a, int64_t lda, const float* b1, int64_t ldb1, int64_t k1,
                                const float* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out,
                                int64_t ldo, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_tn_entry<float>("hgin_gemm_tn_f32", a, lda, b1, ldb1, k1, b2, ldb2, M, N, K, out, ldo, workspace,
                              workspace_bytes, stream);
}

extern "C" int hgin_gemm_tn_bf16(const uint16_t* a, int64_t lda, const uint16_t* b1, int64_t ldb1, int64_t k1,
                                 const uint16_t* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out,
                                 int64_t ldo, void* workspace, size_t workspace_bytes, void* stream) {
  return gemm_tn_entry<uint16_t>("hgin_gemm_tn_bf16", a, lda, b1, ldb1, k1, b2, ldb2, M, N, K, out, ldo, workspace,
                                 workspace_bytes, stream);
}

extern "C" int hgin_gin_mlp_bwd_w_workspace_size(int64_t M, int64_t N, int64_t K, int elem_bytes, int have_gz,
                                                 size_t* bytes) {
  HGIN_ARG_CHECK(bytes && M >= 0 && N >= 0 && K >= 0 && (elem_bytes == 2 || elem_bytes == 4),
                 "hgin_gin_mlp_bwd_w_workspace_size: bad args");
  *bytes = mlp_bwd_w_ws_bytes(M, N, K, (size_t)elem_bytes, have_gz != 0);
  return HGIN_OK;
}

extern "C" int hgin_gin_mlp_bwd_w_f32(const float* g_y, int64_t ld_gy, const float* z, int64_t ldz, const float* prelu,
                                      const float* b1, int64_t ldb1, int64_t k1, const float* b2, int64_t ldb2,
                                      int64_t M, int64_t N, int64_t K, float* g_w, int64_t ldw, float* g_prelu,
                                      float* g_bias, float* g_z, int64_t ld_gz, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  return mlp_bwd_w_entry<float>("hgin_gin_mlp_bwd_w_f32", g_y, ld_gy, z, ldz, prelu, b1, ldb1, k1, b2, ldb2, M, N, K,
                                g_w, ldw, g_prelu, g_bias, g_z, ld_gz, workspace, workspace_bytes, stream);
}

extern "C" int hgin_gin_mlp_bwd_w_bf16(const uint16_t* g_y, int64_t ld_gy, const uint16_t* z, int64_t ldz,
                                       const float* prelu, const uint16_t* b1, int64_t ldb1, int64_t k1,
                                       const uint16_t* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K, float* g_w,
                                       int64_t ldw, float* g_prelu, float* g_bias, uint16_t* g_z, int64_t ld_gz,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  return mlp_bwd_w_entry<uint16_t>("hgin_gin_mlp_bwd_w_bf16", g_y, ld_gy, z, ldz, prelu, b1, ldb1, k1, b2, ldb2, M, N,
                                   K, g_w, ldw, g_prelu, g_bias, g_z, ld_gz, workspace, workspace_bytes, stream);
}

extern "C" int hgin_gin_mlp_bwd_w_zy_bf16(const uint16_t* g_y, int64_t ld_gy, uint16_t* z, const uint16_t* y,
                                          const float* prelu, const uint16_t* b1, int64_t ldb1, int64_t k1,
                                          const uint16_t* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K,
                                          float* g_w, int64_t ldw, float* g_prelu, float* g_bias, uint16_t* g_z,
                                          int64_t ld_gz, void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(M == 0 || (z && y && g_z), "hgin_gin_mlp_bwd_w_zy_bf16: z, y and g_z are required");
  return mlp_bwd_w_entry<uint16_t>("hgin_gin_mlp_bwd_w_zy_bf16", g_y, ld_gy, z, N, prelu, b1, ldb1, k1, b2, ldb2, M, N,
                                   K, g_w, ldw, g_prelu, g_bias, g_z, ld_gz, workspace, workspace_bytes, stream, y);
}

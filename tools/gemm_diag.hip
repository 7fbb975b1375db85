// Diagnostic (not part of libhgin): where does the fp32 NT GEMM's time go at the GIN shapes?
// The production kernel's loop (hgin_gemm_nt.hip, 128 x 128 tile, BK 32, register prefetch, LDS restage
// with two barriers per K-tile, LDS-staged epilogue) rebuilt with switches that remove one cost at a time:
//   NOLOAD    no in-loop global loads (the prologue tile is reused: MFMA + LDS + barriers only)
//   NOSTORE   epilogue computes but does not store
//   NORESTAGE no LDS restage / barriers inside the K loop
//   PRIO      s_setprio(1) around each MFMA cluster
//   DBUF      two LDS buffers, one barrier per K-tile (2 workgroups per CU)
//   BK64      64-deep K-tiles (half the barriers; 2 workgroups per CU)
// Build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/gemm_diag tools/gemm_diag.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

using f32x16 = __attribute__((ext_vector_type(16))) float;

enum { NOLOAD = 1, NOSTORE = 2, NORESTAGE = 4, PRIO = 8, DBUF = 16, BK64 = 32, OCC4 = 64 };

template <int BKv>
__device__ __forceinline__ void load_tile(float4 (&r)[4 * BKv / 32], const float* p, int64_t ld, int64_t row0,
                                          int64_t rows, int64_t k0, int tid) {
  constexpr int kC = BKv / 4;           // float4 per row
  constexpr int kR = 256 / kC;          // rows per pass
#pragma unroll
  for (int i = 0; i < 4 * BKv / 32; ++i) {
    const int64_t gr = row0 + tid / kC + kR * i;
    r[i] = gr < rows ? *reinterpret_cast<const float4*>(p + gr * ld + k0 + (tid % kC) * 4)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int BKv>
__device__ __forceinline__ void store_tile(float* dst, const float4 (&r)[4 * BKv / 32], int tid) {
  constexpr int kC = BKv / 4, kR = 256 / kC, kL = BKv + 4;
#pragma unroll
  for (int i = 0; i < 4 * BKv / 32; ++i)
    *reinterpret_cast<float4*>(dst + (tid / kC + kR * i) * kL + (tid % kC) * 4) = r[i];
}

template <int F>
__global__ __launch_bounds__(256, (F & (DBUF | BK64)) ? 2 : ((F & OCC4) ? 4 : 3)) void k_diag(const float* A, const float* B, float* Y,
                                                                          int64_t M, int64_t N, int64_t K,
                                                                          int64_t tiles) {
  constexpr int BK = (F & BK64) ? 64 : 32;
  constexpr int kL = BK + 4;
  constexpr int NB = (F & DBUF) ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float smem[NB * 256 * kL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t L = blockIdx.x, G = gridDim.x;
  const int64_t q = (L % 8) * (G / 8) + L / 8;
  if (q >= tiles) return;
  const int64_t ntn = N / 128;
  const int64_t m0 = (q / ntn) * 128, n0 = (q % ntn) * 128;
  f32x16 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  float4 ra[4 * BK / 32], rb[4 * BK / 32];
  load_tile<BK>(ra, A, K, m0, M, 0, tid);
  load_tile<BK>(rb, B, K, n0, N, 0, tid);
  store_tile<BK>(smem, ra, tid);
  store_tile<BK>(smem + 128 * kL, rb, tid);
  __syncthreads();
  int cur = 0;
  for (int64_t k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more && !(F & NOLOAD)) {
      load_tile<BK>(ra, A, K, m0, M, k0 + BK, tid);
      load_tile<BK>(rb, B, K, n0, N, k0 + BK, tid);
    }
    const float* As = smem + cur * 256 * kL;
    const float* Bs = As + 128 * kL;
    if (F & PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < BK / 8; ++c) {
      float4 fa[2], fb[2];
      for (int t = 0; t < 2; ++t) {
        fa[t] = *reinterpret_cast<const float4*>(As + (wm * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
        fb[t] = *reinterpret_cast<const float4*>(Bs + (wn * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
      }
      for (int tm = 0; tm < 2; ++tm)
        for (int tn = 0; tn < 2; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].x, fb[tn].x, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].y, fb[tn].y, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].z, fb[tn].z, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].w, fb[tn].w, acc[tm][tn], 0, 0, 0);
        }
    }
    if (F & PRIO) __builtin_amdgcn_s_setprio(0);
    if (more && !(F & NORESTAGE)) {
      if (F & DBUF) {
        float* nxt = smem + (cur ^ 1) * 256 * kL;
        store_tile<BK>(nxt, ra, tid);
        store_tile<BK>(nxt + 128 * kL, rb, tid);
        __syncthreads();
        cur ^= 1;
      } else {
        __syncthreads();
        store_tile<BK>(smem, ra, tid);
        store_tile<BK>(smem + 128 * kL, rb, tid);
        __syncthreads();
      }
    }
  }
  // epilogue: park 32 rows per wave in LDS, write row-contiguous float4s
  constexpr int kLc = 68;
  float* Cw = smem + wave * 32 * kLc;
  const int c = (lane % 16) * 4, r0 = lane / 16;
  __syncthreads();
  for (int tm = 0; tm < 2; ++tm) {
    for (int tn = 0; tn < 2; ++tn)
      for (int e = 0; e < 16; ++e) Cw[((e & 3) + 8 * (e >> 2) + 4 * lh) * kLc + tn * 32 + li] = acc[tm][tn][e];
    __syncthreads();
    for (int j = 0; j < 8; ++j) {
      const int r = r0 + 4 * j;
      const int64_t row = m0 + wm * 64 + tm * 32 + r;
      if (row >= M) continue;
      const float4 v = *reinterpret_cast<const float4*>(Cw + r * kLc + c);
      float* dst = Y + row * N + n0 + wn * 64 + c;
      if (!(F & NOSTORE) || v.x == 1234.5f) *reinterpret_cast<float4*>(dst) = v;
    }
    if (tm == 0) __syncthreads();
  }
}

// Persistent, deferred epilogue: a workgroup walks tiles q, q + G, ...; tile i's results stay in VGPRs
// (MFMA layout) and are stored 1/8 per K-tile during tile i+1's loop, so the output stream overlaps MFMA
// work instead of arriving as one burst at every round's end.  2 workgroups per CU.
template <int F>
__global__ __launch_bounds__(256, 2) void k_persist(const float* A, const float* B, float* Y, int64_t M, int64_t N,
                                                    int64_t K, int64_t tiles) {
  constexpr int BK = 32, kL = BK + 4;
  __shared__ __attribute__((aligned(16))) float smem[256 * kL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t G = gridDim.x;
  const int64_t ntn = N / 128;
  float prev[64];
  int64_t pm0 = -1, pn0 = 0;
  // part p: 8 of the 64 values, held (after p shifts) in prev[0..7]: block b = p >> 1, e in [8 (p & 1), +8)
  auto store_part = [&](int part) {
    const int b = part >> 1, tm = b >> 1, tn = b & 1;
    if (pm0 >= 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = (part & 1) * 8 + i;
        const int64_t row = pm0 + wm * 64 + tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (row < M) Y[row * N + pn0 + wn * 64 + tn * 32 + li] = prev[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 56; ++i) prev[i] = prev[i + 8];
  };
  for (int64_t q = blockIdx.x; q < tiles; q += G) {
    const int64_t m0 = (q / ntn) * 128, n0 = (q % ntn) * 128;
    f32x16 acc[2][2];
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    float4 ra[4], rb[4];
    load_tile<BK>(ra, A, K, m0, M, 0, tid);
    load_tile<BK>(rb, B, K, n0, N, 0, tid);
    __syncthreads();   // previous tile's last MFMAs are done reading LDS
    store_tile<BK>(smem, ra, tid);
    store_tile<BK>(smem + 128 * kL, rb, tid);
    __syncthreads();
    int part = 0;
    for (int64_t k0 = 0; k0 < K; k0 += BK) {
      const bool more = k0 + BK < K;
      if (more) {
        load_tile<BK>(ra, A, K, m0, M, k0 + BK, tid);
        load_tile<BK>(rb, B, K, n0, N, k0 + BK, tid);
      }
      if (F & PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int c = 0; c < BK / 8; ++c) {
        float4 fa[2], fb[2];
        for (int t = 0; t < 2; ++t) {
          fa[t] = *reinterpret_cast<const float4*>(smem + (wm * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
          fb[t] = *reinterpret_cast<const float4*>(smem + 128 * kL + (wn * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
        }
        for (int tm = 0; tm < 2; ++tm)
          for (int tn = 0; tn < 2; ++tn) {
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].x, fb[tn].x, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].y, fb[tn].y, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].z, fb[tn].z, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].w, fb[tn].w, acc[tm][tn], 0, 0, 0);
          }
      }
      if (F & PRIO) __builtin_amdgcn_s_setprio(0);
      if (part < 8) store_part(part++);
      if (more) {
        __syncthreads();
        store_tile<BK>(smem, ra, tid);
        store_tile<BK>(smem + 128 * kL, rb, tid);
        __syncthreads();
      }
    }
    while (part < 8) store_part(part++);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) prev[b * 16 + e] = acc[b >> 1][b & 1][e];
    pm0 = m0;
    pn0 = n0;
  }
  for (int p = 0; p < 8; ++p) store_part(p);
}

// 8 waves, 256 x 128 tile (4 x 2 waves of 64 x 64), BK 32, register prefetch: 2 workgroups = 16 waves per
// CU (4 per SIMD) at <= 128 VGPRs, B tile reused over twice the rows.
template <int F>
__global__ __launch_bounds__(512, 2) __attribute__((amdgpu_num_vgpr(128))) void k_w8(const float* A, const float* B, float* Y, int64_t M, int64_t N,
                                               int64_t K, int64_t tiles) {
  constexpr int BK = 32, kL = BK + 4;
  __shared__ __attribute__((aligned(16))) float smem[384 * kL];
  float* As = smem;
  float* Bs = smem + 256 * kL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t L = blockIdx.x, G = gridDim.x;
  const int64_t q = (L % 8) * (G / 8) + L / 8;
  if (q >= tiles) return;
  const int64_t ntn = N / 128;
  const int64_t m0 = (q / ntn) * 256, n0 = (q % ntn) * 128;
  f32x16 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  float4 ra[4], rb[2];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t gr = m0 + (tid >> 3) + 64 * i;
      gr = gr < M ? gr : M - 1;
      const float4 v = *reinterpret_cast<const float4*>(A + gr * K + k0 + (tid & 7) * 4);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t gr = n0 + (tid >> 3) + 64 * i;
      const float4 v = *reinterpret_cast<const float4*>(B + gr * K + k0 + (tid & 7) * 4);
      rb[i] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float4*>(As + ((tid >> 3) + 64 * i) * kL + (tid & 7) * 4) = ra[i];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *reinterpret_cast<float4*>(Bs + ((tid >> 3) + 64 * i) * kL + (tid & 7) * 4) = rb[i];
  };
  load(0);
  store();
  __syncthreads();
  for (int64_t k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) load(k0 + BK);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < BK / 8; ++c) {
      float4 fa[2], fb[2];
      for (int t = 0; t < 2; ++t) {
        fa[t] = *reinterpret_cast<const float4*>(As + (wm * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
        fb[t] = *reinterpret_cast<const float4*>(Bs + (wn * 64 + t * 32 + li) * kL + c * 8 + lh * 4);
      }
      for (int tm = 0; tm < 2; ++tm)
        for (int tn = 0; tn < 2; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].x, fb[tn].x, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].y, fb[tn].y, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].z, fb[tn].z, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tm].w, fb[tn].w, acc[tm][tn], 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      __syncthreads();
      store();
      __syncthreads();
    }
  }
  constexpr int kLc = 68;
  float* Cw = smem + wave * 32 * kLc;
  const int c = (lane % 16) * 4, r0 = lane / 16;
  __syncthreads();
  for (int tm = 0; tm < 2; ++tm) {
    for (int tn = 0; tn < 2; ++tn)
      for (int e = 0; e < 16; ++e) Cw[((e & 3) + 8 * (e >> 2) + 4 * lh) * kLc + tn * 32 + li] = acc[tm][tn][e];
    __syncthreads();
    for (int j = 0; j < 8; ++j) {
      const int r = r0 + 4 * j;
      const int64_t row = m0 + wm * 64 + tm * 32 + r;
      if (row >= M) continue;
      const float4 v = *reinterpret_cast<const float4*>(Cw + r * kLc + c);
      *reinterpret_cast<float4*>(Y + row * N + n0 + wn * 64 + c) = v;
    }
    if (tm == 0) __syncthreads();
  }
}

template <int F>
float run_w8(const float* A, const float* B, float* Y, int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = (M + 255) / 256 * (N / 128);
  const unsigned grid = (unsigned)((tiles + 7) / 8 * 8);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int i = 0; i < 3; ++i) k_w8<F><<<grid, 512>>>(A, B, Y, M, N, K, tiles);
  const int reps = 20;
  hipEventRecord(s);
  for (int i = 0; i < reps; ++i) k_w8<F><<<grid, 512>>>(A, B, Y, M, N, K, tiles);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3f / reps;
}

// fp32 GEMM on the bf16 matrix cores: every fp32 operand is split a = a1 + a2 + a3 (bf16 each, RNE; the
// residuals are exact in fp32) when it is staged into LDS, and six bf16 MFMA products
// (a1b1, a1b2, a2b1, a1b3, a2b2, a3b1; dropped terms < 2^-25 |a||b|) accumulate in fp32.
// LDS row: 3 planes x 32 bf16 + 16 B pad = 208 B (13 x 16 B: ds_read_b128 conflict-free).
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
template <int NP>
__device__ __forceinline__ void split4(const float4 v, uint2 (&o)[3]) {
  float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t h[3][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 b1 = (__bf16)x[i];
    const float r1 = x[i] - (float)b1;
    const __bf16 b2 = (__bf16)r1;
    const float r2 = r1 - (float)b2;
    const __bf16 b3 = (__bf16)r2;
    h[0][i] = __builtin_bit_cast(uint16_t, b1);
    h[1][i] = __builtin_bit_cast(uint16_t, b2);
    h[2][i] = __builtin_bit_cast(uint16_t, b3);
  }
#pragma unroll
  for (int p = 0; p < 3; ++p) o[p] = make_uint2(h[p][0] | (h[p][1] << 16), h[p][2] | (h[p][3] << 16));
}

template <int F>
__global__ __launch_bounds__(256, 3) void k_split(const float* A, const float* B, float* Y, int64_t M, int64_t N,
                                                  int64_t K, int64_t tiles) {
  constexpr int BK = 32;
  constexpr int kRow = 52;   // uint32 words per LDS row
  __shared__ __attribute__((aligned(16))) uint32_t smem[256 * kRow];
  uint32_t* As = smem;
  uint32_t* Bs = smem + 128 * kRow;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t L = blockIdx.x, G = gridDim.x;
  const int64_t q = (L % 8) * (G / 8) + L / 8;
  if (q >= tiles) return;
  const int64_t ntn = N / 128;
  const int64_t m0 = (q / ntn) * 128, n0 = (q % ntn) * 128;
  f32x16 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  float4 ra[4], rb[4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t gr = m0 + (tid >> 3) + 32 * i;
      gr = gr < M ? gr : M - 1;
      const float4 v = *reinterpret_cast<const float4*>(A + gr * K + k0 + (tid & 7) * 4);
      ra[i] = v;
      const float4 w = *reinterpret_cast<const float4*>(B + (n0 + (tid >> 3) + 32 * i) * K + k0 + (tid & 7) * 4);
      rb[i] = w;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint2 o[3];
      const int r = (tid >> 3) + 32 * i;
      split4<3>(ra[i], o);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(As + r * kRow + p * 16 + (tid & 7) * 2) = o[p];
      split4<3>(rb[i], o);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(Bs + r * kRow + p * 16 + (tid & 7) * 2) = o[p];
    }
  };
  load(0);
  store();
  __syncthreads();
  for (int64_t k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) load(k0 + BK);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8 fa[2][3], fb[2][3];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          fa[t][p] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + t * 32 + li) * kRow + p * 16 + kb * 8 + lh * 4);
          fb[t][p] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + t * 32 + li) * kRow + p * 16 + kb * 8 + lh * 4);
        }
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][2], fb[tn][0], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[tn][1], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][2], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][1], fb[tn][0], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][1], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[tm][0], fb[tn][0], acc[tm][tn], 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      __syncthreads();
      store();
      __syncthreads();
    }
  }
  constexpr int kLc = 68;
  float* Cw = reinterpret_cast<float*>(smem) + wave * 32 * kLc;
  const int c = (lane % 16) * 4, r0 = lane / 16;
  __syncthreads();
  for (int tm = 0; tm < 2; ++tm) {
    for (int tn = 0; tn < 2; ++tn)
      for (int e = 0; e < 16; ++e) Cw[((e & 3) + 8 * (e >> 2) + 4 * lh) * kLc + tn * 32 + li] = acc[tm][tn][e];
    __syncthreads();
    for (int j = 0; j < 8; ++j) {
      const int r = r0 + 4 * j;
      const int64_t row = m0 + wm * 64 + tm * 32 + r;
      if (row >= M) continue;
      const float4 v = *reinterpret_cast<const float4*>(Cw + r * kLc + c);
      *reinterpret_cast<float4*>(Y + row * N + n0 + wn * 64 + c) = v;
    }
    if (tm == 0) __syncthreads();
  }
}

template <int F>
float run_split(const float* A, const float* B, float* Y, int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = (M + 127) / 128 * (N / 128);
  const unsigned grid = (unsigned)((tiles + 7) / 8 * 8);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int i = 0; i < 3; ++i) k_split<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  const int reps = 20;
  hipEventRecord(s);
  for (int i = 0; i < reps; ++i) k_split<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3f / reps;
}

template <int F>
float run_persist(const float* A, const float* B, float* Y, int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = (M + 127) / 128 * (N / 128);
  int per_cu = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_persist<F>, 256, 0);
  const unsigned grid = (unsigned)(per_cu * 256 < tiles ? per_cu * 256 : tiles);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int i = 0; i < 3; ++i) k_persist<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  const int reps = 20;
  hipEventRecord(s);
  for (int i = 0; i < reps; ++i) k_persist<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, s, e);
  return ms * 1e3f / reps;
}

template <int F>
float run(const float* A, const float* B, float* Y, int64_t M, int64_t N, int64_t K) {
  if (F & 1024) return run_persist<F>(A, B, Y, M, N, K);
  if (F & 2048) return run_w8<F>(A, B, Y, M, N, K);
  if (F & 4096) return run_split<F>(A, B, Y, M, N, K);
  const int64_t tiles = (M + 127) / 128 * (N / 128);
  const unsigned grid = (unsigned)((tiles + 7) / 8 * 8);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int i = 0; i < 3; ++i) k_diag<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  const int reps = 20;
  hipEventRecord(s);
  for (int i = 0; i < reps; ++i) k_diag<F><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, s, e);
  hipEventDestroy(s);
  hipEventDestroy(e);
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 294912, K = argc > 2 ? atoll(argv[2]) : 256,
                N = argc > 3 ? atoll(argv[3]) : 128;
  std::vector<float> h((size_t)M * K);
  uint32_t x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (float)((x >> 8) & 0xffff) / 65536.0f - 0.5f;
  }
  float *A, *B, *Y;
  hipMalloc(&A, M * K * 4);
  hipMalloc(&B, N * K * 4);
  hipMalloc(&Y, M * N * 4);
  hipMemcpy(A, h.data(), M * K * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), N * K * 4, hipMemcpyHostToDevice);
  const double gf = 2.0 * M * N * K / 1e9;
  printf("M=%lld K=%lld N=%lld (%.1f GF)\n", (long long)M, (long long)K, (long long)N, gf);
#define R(F, name)                                                                        \
  {                                                                                       \
    float best = 1e30f;                                                                   \
    for (int rep = 0; rep < 3; ++rep) {                                                   \
      float us = run<F>(A, B, Y, M, N, K);                                                \
      best = us < best ? us : best;                                                       \
    }                                                                                     \
    printf("  %-28s %8.1f us %7.1f TF/s\n", name, best, gf / (best * 1e-6) / 1e3);        \
  }
  R(0, "baseline");
  R(NOLOAD, "noload");
  R(NOSTORE, "nostore");
  R(NOLOAD | NOSTORE, "noload+nostore");
  R(NOLOAD | NOSTORE | NORESTAGE, "mfma+ldsread only");
  R(PRIO, "prio");
  R(DBUF, "dbuf");
  R(DBUF | PRIO, "dbuf+prio");
  R(BK64, "bk64");
  R(BK64 | DBUF, "bk64+dbuf");
  R(4096, "bf16x3 split, 6 products");
  // accuracy of the split GEMM and of the f32 MFMA GEMM against fp64, on a slice of rows
  {
    float* Y2;
    hipMalloc(&Y2, M * N * 4);
    const int64_t tiles = (M + 127) / 128 * (N / 128);
    const unsigned grid = (unsigned)((tiles + 7) / 8 * 8);
    k_diag<0><<<grid, 256>>>(A, B, Y, M, N, K, tiles);
    k_split<0><<<grid, 256>>>(A, B, Y2, M, N, K, tiles);
    const int64_t R = 4096;
    std::vector<float> y1((size_t)R * N), y2((size_t)R * N), hb((size_t)N * K);
    hipMemcpy(y1.data(), Y, R * N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(y2.data(), Y2, R * N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hb.data(), B, N * K * 4, hipMemcpyDeviceToHost);
    double e1 = 0, e2 = 0, r1 = 0, r2 = 0;
    for (int64_t i = 0; i < R; ++i)
      for (int64_t j = 0; j < N; ++j) {
        double ref = 0, mag = 0;
        for (int64_t k = 0; k < K; ++k) {
          ref += (double)h[i * K + k] * hb[j * K + k];
          mag += fabs((double)h[i * K + k] * hb[j * K + k]);
        }
        const double d1 = fabs(y1[i * N + j] - ref) / mag, d2 = fabs(y2[i * N + j] - ref) / mag;
        e1 = d1 > e1 ? d1 : e1;
        e2 = d2 > e2 ? d2 : e2;
        r1 += d1;
        r2 += d2;
      }
    printf("  max |err| / sum|ab|: f32 MFMA %.3g (mean %.3g), bf16x3 split %.3g (mean %.3g)\n", e1, r1 / (R * N), e2,
           r2 / (R * N));
  }
  return 0;
}

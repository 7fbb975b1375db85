// Global mean / max pooling of the path features per graph (models.py:347-352: torch_geometric.nn.global_mean_pool
// and global_max_pool of origin_input["path"] by path_batch, each broadcast back to its graph's rows with
// torch.gather): GLOBAL_FEATS (config.json:25) readout inputs.
//
// path_batch comes from PyG collation (dataset.py:239-244): non-decreasing graph ids, so every graph's rows are one
// contiguous segment — a CSR without a sort.  No host synchronisation, no atomics on data, no id-indexed scratch
// (graph ids may skip values: graphs without path rows).  Three launches:
//   k_seg_pool: workgroups stride over 256-row windows; a row whose graph id differs from its predecessor's starts a
//   segment (compacted into an LDS list) and a descending id sets HGIN_STATUS_UNSORTED in the caller's status word.
//   For each start the segment's end is found by binary search; a segment of at most kPoolLong rows is reduced right
//   there — lane c walks column c over the known row range, summing sequentially in row order (fp32, no FMA:
//   bit-identical to CPU scatter_add / scatter_reduce "mean" = sum, then one true division by the row count) and
//   keeping its running max (first maximum; NaN propagates) — and all lanes write the graph's [mean | max] into each
//   of its rows (out[r, 0:f] = mean, out[r, f:2f] = max: the gathered layout of torch.gather at models.py:350-351).
//   k_seg_long_partial / k_seg_long_final: a longer segment (one big graph: a single-graph batch of a cfg2-cfg5
//   sized graph has millions of path rows) is cut at kPoolChunk-row chunk boundaries; one workgroup per chunk reduces
//   its piece(s) sequentially into a partial (sum, max), and then every chunk of the segment adds the segment's
//   partials in chunk order and writes its own rows.  Deterministic run to run; the long segments' sums are
//   re-associated (chunk partials), within fp32 rounding of the sequential sum.
#include "hgin_common.h"

namespace hgin {
namespace {

constexpr int64_t kPoolLong = 4096;   // longest segment reduced sequentially by one workgroup (bit-exact)
constexpr int64_t kPoolChunk = 2048;  // rows per chunk of the long-segment path (<= kPoolLong: a long segment is never
                                      // interior to one chunk, so a chunk holds at most two long pieces)

// first index q in [lo, hi) with batch[q] > b (batch non-decreasing on the range)
__device__ __forceinline__ int64_t upper_bound(const int64_t* batch, int64_t lo, int64_t hi, int64_t b) {
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (batch[mid] <= b) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// first index q in [lo, hi) with batch[q] >= b
__device__ __forceinline__ int64_t lower_bound(const int64_t* batch, int64_t lo, int64_t hi, int64_t b) {
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (batch[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <typename T>
__device__ __forceinline__ void walk(const T* __restrict__ x, int64_t ldx, int c, int64_t lo, int64_t hi, float& s,
                                     float& m) {
  s = 0.0f;
  m = Elem<T>::ld(x + lo * ldx + c);
  for (int64_t q = lo; q < hi; ++q) {
    const float v = Elem<T>::ld(x + q * ldx + c);
    s = __fadd_rn(s, v);
    if (v > m || v != v) m = v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_seg_pool(const int64_t* __restrict__ batch, int64_t n,
                                                  const T* __restrict__ x, int64_t ldx, int f, T* __restrict__ out,
                                                  int64_t ld_out, int* __restrict__ status) {
  extern __shared__ float pool_smem[];   // [2 f]: mean | max of the current graph
  __shared__ int32_t starts[256];
  __shared__ int n_starts;
  __shared__ int64_t seg_hi;
  const int t = threadIdx.x;
  for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
    if (t == 0) n_starts = 0;
    __syncthreads();
    const int64_t r = base + t;
    if (r < n && (r == 0 || batch[r - 1] != batch[r])) {
      if (r > 0 && batch[r - 1] > batch[r]) atomicOr(status, HGIN_STATUS_UNSORTED);
      starts[atomicAdd(&n_starts, 1)] = t;
    }
    __syncthreads();
    const int ns = n_starts;
    for (int i = 0; i < ns; ++i) {
      const int64_t lo = base + starts[i];
      const int64_t b = batch[lo];
      if (t == 0) {
        // a short segment ends within kPoolLong rows: search there first
        const int64_t cap = lo + kPoolLong + 1 < n ? lo + kPoolLong + 1 : n;
        seg_hi = upper_bound(batch, lo, cap, b);
      }
      __syncthreads();
      const int64_t hi = seg_hi;
      if (hi - lo <= kPoolLong && (hi == n || batch[hi] != b)) {   // else: long segment, chunked path
        for (int c = t; c < f; c += 256) {
          float s, m;
          walk(x, ldx, c, lo, hi, s, m);
          pool_smem[c] = __fdiv_rn(s, (float)(hi - lo));
          pool_smem[f + c] = m;
        }
        __syncthreads();
        const int64_t cells = (hi - lo) * (int64_t)(2 * f);
        for (int64_t j = t; j < cells; j += 256) {
          const int64_t row = lo + j / (2 * f);
          const int c = (int)(j % (2 * f));
          Elem<T>::st(out + row * ld_out + c, pool_smem[c]);
        }
      }
      __syncthreads();
    }
  }
}

// The long pieces of chunk [c0, c1): slot 0 = the segment holding row c0 (if long), slot 1 = the segment holding row
// c1 - 1 (if long and different).  Segment bounds by binary search over the whole (sorted) batch vector.
struct LongPiece {
  int64_t seg_lo, seg_hi, lo, hi, b;
  bool valid;
};
__device__ __forceinline__ LongPiece long_piece(const int64_t* batch, int64_t n, int64_t c0, int64_t c1, int slot) {
  LongPiece p{};
  const int64_t row = slot == 0 ? c0 : c1 - 1;
  p.b = batch[row];
  p.valid = !(slot == 1 && batch[c0] == p.b);
  if (!p.valid) return p;
  p.seg_lo = lower_bound(batch, 0, row + 1, p.b);
  p.seg_hi = upper_bound(batch, row, n, p.b);
  p.valid = p.seg_hi - p.seg_lo > kPoolLong;
  p.lo = p.seg_lo > c0 ? p.seg_lo : c0;
  p.hi = p.seg_hi < c1 ? p.seg_hi : c1;
  return p;
}

// partial: [chunks][2 slots][2 f] (sum | max)
template <typename T>
__global__ __launch_bounds__(256) void k_seg_long_partial(const int64_t* __restrict__ batch, int64_t n,
                                                          const T* __restrict__ x, int64_t ldx, int f,
                                                          float* __restrict__ partial) {
  __shared__ LongPiece pc[2];
  const int64_t chunk = blockIdx.x;
  const int64_t c0 = chunk * kPoolChunk;
  const int64_t c1 = c0 + kPoolChunk < n ? c0 + kPoolChunk : n;
  if (threadIdx.x < 2) pc[threadIdx.x] = long_piece(batch, n, c0, c1, (int)threadIdx.x);
  __syncthreads();
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const LongPiece p = pc[slot];
    if (!p.valid) continue;
    float* dst = partial + (chunk * 2 + slot) * (int64_t)(2 * f);
    for (int c = threadIdx.x; c < f; c += 256) {
      float s, m;
      walk(x, ldx, c, p.lo, p.hi, s, m);
      dst[c] = s;
      dst[f + c] = m;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_seg_long_final(const int64_t* __restrict__ batch, int64_t n, int f,
                                                        const float* __restrict__ partial, T* __restrict__ out,
                                                        int64_t ld_out) {
  extern __shared__ float pool_smem[];   // [2 f]
  __shared__ LongPiece pc[2];
  const int64_t chunk = blockIdx.x;
  const int64_t c0 = chunk * kPoolChunk;
  const int64_t c1 = c0 + kPoolChunk < n ? c0 + kPoolChunk : n;
  if (threadIdx.x < 2) pc[threadIdx.x] = long_piece(batch, n, c0, c1, (int)threadIdx.x);
  __syncthreads();
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const LongPiece p = pc[slot];
    if (!p.valid) continue;
    const int64_t ca = p.seg_lo / kPoolChunk, cb = (p.seg_hi - 1) / kPoolChunk;
    for (int c = threadIdx.x; c < f; c += 256) {
      float s = 0.0f, m = 0.0f;
      for (int64_t j = ca; j <= cb; ++j) {   // chunk order
        // the segment is slot 0 of chunk j when it holds the chunk's first row, else slot 1
        const int sl = batch[j * kPoolChunk] == p.b ? 0 : 1;
        const float* src = partial + (j * 2 + sl) * (int64_t)(2 * f);
        const float ps = src[c], pm = src[f + c];
        s = __fadd_rn(s, ps);
        if (j == ca || pm > m || pm != pm) m = pm;   // the walk's rule: NaN propagates
      }
      pool_smem[c] = __fdiv_rn(s, (float)(p.seg_hi - p.seg_lo));
      pool_smem[f + c] = m;
    }
    __syncthreads();
    const int64_t cells = (p.hi - p.lo) * (int64_t)(2 * f);
    for (int64_t j = threadIdx.x; j < cells; j += 256) {
      const int64_t row = p.lo + j / (2 * f);
      const int c = (int)(j % (2 * f));
      Elem<T>::st(out + row * ld_out + c, pool_smem[c]);
    }
    __syncthreads();
  }
}

size_t pool_ws_bytes(int64_t n, int64_t f) {
  return (size_t)ceil_div(n > 0 ? n : 1, kPoolChunk) * 2 * (size_t)(2 * (f > 0 ? f : 1)) * sizeof(float);
}

template <typename T>
int global_pool(const char* what, const int64_t* batch, int64_t n, const T* x, int64_t ldx, int64_t f, T* out,
                int64_t ld_out, int* status, void* workspace, size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(n >= 0 && f >= 0, "%s: negative size", what);
  if (n == 0 || f == 0) return HGIN_OK;
  HGIN_ARG_CHECK(f <= 4096, "%s: at most 4096 pooled columns", what);
  HGIN_ARG_CHECK(batch && x && out && status && ldx >= f && ld_out >= 2 * f, "%s: bad operand / leading dimension",
                 what);
  const size_t need = pool_ws_bytes(n, f);
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu", what, workspace_bytes, need);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  HGIN_TRACE("k_seg_pool<%s,F%lld>", sizeof(T) == 4 ? "f32" : "bf16", (long long)f);
  const int64_t windows = ceil_div(n, 256);
  const int64_t grid = windows < 1024 ? windows : 1024;
  const size_t lds = 2 * f * sizeof(float);
  k_seg_pool<T><<<(unsigned)grid, 256, lds, s>>>(batch, n, x, ldx, (int)f, out, ld_out, status);
  if (n > kPoolLong) {   // a segment longer than kPoolLong exists only then
    const int64_t chunks = ceil_div(n, kPoolChunk);
    float* partial = static_cast<float*>(workspace);
    k_seg_long_partial<T><<<(unsigned)chunks, 256, 0, s>>>(batch, n, x, ldx, (int)f, partial);
    k_seg_long_final<T><<<(unsigned)chunks, 256, lds, s>>>(batch, n, (int)f, partial, out, ld_out);
  }
  return check_launch(what);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_global_pool_workspace_size(int64_t n_rows, int64_t f, size_t* bytes) {
  HGIN_ARG_CHECK(bytes && n_rows >= 0 && f >= 0, "hgin_global_pool_workspace_size: bad args");
  *bytes = pool_ws_bytes(n_rows, f);
  return HGIN_OK;
}

extern "C" int hgin_global_pool_f32(const int64_t* batch, int64_t n_rows, const float* x, int64_t ldx, int64_t f,
                                    float* out, int64_t ld_out, int* d_status, void* workspace, size_t workspace_bytes,
                                    void* stream) {
  return global_pool<float>("hgin_global_pool_f32", batch, n_rows, x, ldx, f, out, ld_out, d_status, workspace,
                            workspace_bytes, stream);
}

extern "C" int hgin_global_pool_bf16(const int64_t* batch, int64_t n_rows, const uint16_t* x, int64_t ldx, int64_t f,
                                     uint16_t* out, int64_t ld_out, int* d_status, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return global_pool<uint16_t>("hgin_global_pool_bf16", batch, n_rows, x, ldx, f, out, ld_out, d_status, workspace,
                               workspace_bytes, stream);
}

// A12 — stable COO -> CSR / CSC on gfx950.
//
// The reference never sorts (PyG scatters unsorted COO with atomics, models.py:208).  The build sorts
// each relation once by its destination (CSR, forward) and by its source (CSC, backward) with a stable
// LSD radix sort, so every row keeps the original edge order — the order CPU scatter_add_/index_add_
// accumulate in — and the segmented sums are bit-exact against the reference's CPU path.
//
// Layout: keys = the sorted endpoint (uint32), vals = edge id (uint32).  One pass per 8 key bits:
//   hist    : per 4096-key tile, a 256-bucket histogram in LDS (integer atomics: order-free)
//   scan    : one workgroup, exclusive scan of the digit-major [256][tiles] count matrix
//   scatter : per tile, 16 chunks of 256 keys in index order; inside a chunk each wave ranks its lanes
//             with 8 ballots (match-any on the digit), so positions are stable without atomics.
// rowptr = lower_bound over the sorted keys (one thread per row: O(n_rows log E), no serial tails).
#include "hgin_common.h"

namespace hgin {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
constexpr int kBuckets = 256;

__global__ __launch_bounds__(256) void k_extract(const int64_t* __restrict__ ei, int64_t E, int key_row,
                                                 int64_t n_rows, int64_t n_cols, uint32_t* __restrict__ keys,
                                                 uint32_t* __restrict__ vals, int32_t* __restrict__ status) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int bad_all = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += stride) {
    int64_t k = ei[(int64_t)key_row * E + i];
    const int64_t o = ei[(int64_t)(1 - key_row) * E + i];
    int bad = 0;
    if (k < 0 || k >= n_rows) {
      bad |= HGIN_STATUS_ROW_OOR;
      k = 0;  // keep the sort in range; the caller must reject the build
    }
    if (o < 0 || o >= n_cols) bad |= HGIN_STATUS_COL_OOR;
    bad_all |= bad;
    keys[i] = static_cast<uint32_t>(k);
    vals[i] = static_cast<uint32_t>(i);
  }
  if (bad_all) atomicOr(status, bad_all);
}

__global__ __launch_bounds__(256) void k_radix_hist(const uint32_t* __restrict__ keys, int64_t E, int shift,
                                                    uint32_t* __restrict__ counts, int64_t n_tiles) {
  __shared__ uint32_t h[kBuckets];
  const int t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + (int64_t)j * kThreads + t;
    if (i < E) atomicAdd(&h[(keys[i] >> shift) & (kBuckets - 1)], 1u);
  }
  __syncthreads();
  counts[(int64_t)t * n_tiles + blockIdx.x] = h[t];
}

// Exclusive scan of n entries by one 1024-thread workgroup (each thread a contiguous chunk).
__global__ __launch_bounds__(1024) void k_scan_exclusive(uint32_t* __restrict__ data, int64_t n) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t b = (int64_t)t * chunk;
  const int64_t e = b + chunk < n ? b + chunk : n;
  uint32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += data[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;  // exclusive prefix of this chunk
  for (int64_t i = b; i < e; ++i) {
    const uint32_t v = data[i];
    data[i] = run;
    run += v;
  }
}

// Multi-workgroup exclusive scan for large count arrays: (1) per-4096-chunk sums, (2) one-workgroup scan of
// the chunk sums (k_scan_exclusive), (3) per-chunk scan with the chunk offset.
constexpr int kScanChunk = 4096;   // 256 threads x 16

__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ data, int64_t n,
                                                     uint32_t* __restrict__ sums) {
  __shared__ uint32_t red[256];
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kScanChunk + (int64_t)t * 16;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (b0 + i < n) s += data[b0 + i];
  red[t] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] += red[t + off];
    __syncthreads();
  }
  if (t == 0) sums[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void k_scan_apply(uint32_t* __restrict__ data, int64_t n,
                                                    const uint32_t* __restrict__ offs) {
  __shared__ uint32_t part[256];
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kScanChunk + (int64_t)t * 16;
  uint32_t v[16];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = b0 + i < n ? data[b0 + i] : 0u;
    s += v[i];
  }
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = offs[blockIdx.x] + part[t] - s;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (b0 + i < n) data[b0 + i] = run;
    run += v[i];
  }
}

__global__ __launch_bounds__(256) void k_radix_scatter(const uint32_t* __restrict__ kin,
                                                       const uint32_t* __restrict__ vin,
                                                       uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                       int64_t E, int shift, const uint32_t* __restrict__ offs,
                                                       int64_t n_tiles) {
  __shared__ uint32_t run[kBuckets];
  __shared__ uint32_t wcnt[4][kBuckets];
  __shared__ uint32_t woff[4][kBuckets];
  const int t = threadIdx.x;
  const int wave = t >> 6;
  const int lane = t & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  run[t] = offs[(int64_t)t * n_tiles + blockIdx.x];
#pragma unroll
  for (int w = 0; w < 4; ++w) wcnt[w][t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + (int64_t)j * kThreads + t;
    const bool valid = i < E;
    const uint32_t key = valid ? kin[i] : 0u;
    const uint32_t val = valid ? vin[i] : 0u;
    const uint32_t d = (key >> shift) & (kBuckets - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    if (valid && rank == 0) wcnt[wave][d] = __popcll(peers);
    __syncthreads();
    {
      const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
      const uint32_t r = run[t];
      woff[0][t] = r;
      woff[1][t] = r + c0;
      woff[2][t] = r + c0 + c1;
      woff[3][t] = r + c0 + c1 + c2;
      run[t] = r + c0 + c1 + c2 + c3;
      wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = woff[wave][d] + rank;
      kout[pos] = key;
      vout[pos] = val;
    }
  }
}

__global__ __launch_bounds__(256) void k_rowptr(const uint32_t* __restrict__ keys, int64_t E, int64_t n_rows,
                                                int32_t* __restrict__ rowptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= n_rows; r += stride) {
    int64_t lo = 0, hi = E;  // first k with keys[k] >= r
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)keys[mid] < r) lo = mid + 1; else hi = mid;
    }
    rowptr[r] = static_cast<int32_t>(lo);
  }
}

__global__ __launch_bounds__(256) void k_finish(const uint32_t* __restrict__ vals, const int64_t* __restrict__ ei,
                                                int64_t E, int key_row, int32_t* __restrict__ col,
                                                int32_t* __restrict__ perm) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += stride) {
    const uint32_t v = vals[i];
    col[i] = static_cast<int32_t>(ei[(int64_t)(1 - key_row) * E + v]);
    if (perm) perm[i] = static_cast<int32_t>(v);
  }
}

struct CsrWorkspace {
  size_t keys_a, keys_b, vals_a, vals_b, counts, sums, total;
};

CsrWorkspace csr_layout(int64_t E) {
  CsrWorkspace w{};
  const int64_t tiles = ceil_div(E > 0 ? E : 1, kTile);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
  w.keys_a = take(sizeof(uint32_t) * (size_t)(E > 0 ? E : 1));
  w.keys_b = take(sizeof(uint32_t) * (size_t)(E > 0 ? E : 1));
  w.vals_a = take(sizeof(uint32_t) * (size_t)(E > 0 ? E : 1));
  w.vals_b = take(sizeof(uint32_t) * (size_t)(E > 0 ? E : 1));
  w.counts = take(sizeof(uint32_t) * (size_t)kBuckets * (size_t)tiles);
  w.sums = take(sizeof(uint32_t) * (size_t)ceil_div((int64_t)kBuckets * tiles, kScanChunk));
  w.total = off;
  return w;
}

int grid_for(int64_t n, int threads = 256, int64_t cap = 65536) {
  int64_t g = ceil_div(n > 0 ? n : 1, threads);
  return static_cast<int>(g < cap ? g : cap);
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_csr_workspace_size(int64_t n_edges, int64_t n_rows, size_t* bytes) {
  HGIN_ARG_CHECK(bytes != nullptr, "hgin_csr_workspace_size: bytes is NULL");
  HGIN_ARG_CHECK(n_edges >= 0 && n_edges < (int64_t(1) << 31), "hgin_csr_workspace_size: n_edges out of range");
  HGIN_ARG_CHECK(n_rows >= 0 && n_rows < (int64_t(1) << 31), "hgin_csr_workspace_size: n_rows out of range");
  *bytes = csr_layout(n_edges).total;
  return HGIN_OK;
}

extern "C" int hgin_csr_build(const int64_t* edge_index, int64_t E, int key_row, int64_t n_rows, int64_t n_cols,
                              int32_t* rowptr, int32_t* col, int32_t* perm, int32_t* d_status, void* workspace,
                              size_t workspace_bytes, void* stream) {
  HGIN_ARG_CHECK(E >= 0 && E < (int64_t(1) << 31), "hgin_csr_build: n_edges %lld out of range", (long long)E);
  HGIN_ARG_CHECK(n_rows >= 0 && n_rows < (int64_t(1) << 31), "hgin_csr_build: n_rows out of range");
  HGIN_ARG_CHECK(n_cols >= 0 && n_cols < (int64_t(1) << 31), "hgin_csr_build: n_cols out of range");
  HGIN_ARG_CHECK(key_row == 0 || key_row == 1, "hgin_csr_build: key_row must be 0 or 1");
  HGIN_ARG_CHECK(rowptr != nullptr && d_status != nullptr, "hgin_csr_build: rowptr/d_status NULL");
  HGIN_ARG_CHECK(E == 0 || (edge_index != nullptr && col != nullptr), "hgin_csr_build: edge_index/col NULL");
  const CsrWorkspace w = csr_layout(E);
  if (workspace_bytes < w.total || (E > 0 && workspace == nullptr)) {
    set_error("hgin_csr_build: workspace %zu bytes < required %zu", workspace_bytes, w.total);
    return HGIN_E_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  if (E == 0) {
    return memset_async(rowptr, 0, sizeof(int32_t) * (size_t)(n_rows + 1), s, "hgin_csr_build");
  }
  char* ws = static_cast<char*>(workspace);
  uint32_t* ka = reinterpret_cast<uint32_t*>(ws + w.keys_a);
  uint32_t* kb = reinterpret_cast<uint32_t*>(ws + w.keys_b);
  uint32_t* va = reinterpret_cast<uint32_t*>(ws + w.vals_a);
  uint32_t* vb = reinterpret_cast<uint32_t*>(ws + w.vals_b);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws + w.counts);
  uint32_t* sums = reinterpret_cast<uint32_t*>(ws + w.sums);
  const int64_t tiles = ceil_div(E, kTile);

  k_extract<<<grid_for(E), 256, 0, s>>>(edge_index, E, key_row, n_rows, n_cols, ka, va, d_status);
  int bits = 0;
  if (n_rows > 1) bits = 64 - __builtin_clzll((unsigned long long)(n_rows - 1));
  for (int shift = 0; shift < bits; shift += 8) {
    k_radix_hist<<<(unsigned)tiles, kThreads, 0, s>>>(ka, E, shift, counts, tiles);
    const int64_t nc = (int64_t)kBuckets * tiles;
    if (nc <= 8 * 1024) {
      k_scan_exclusive<<<1, 1024, 0, s>>>(counts, nc);
    } else {
      const int64_t chunks = ceil_div(nc, kScanChunk);
      k_scan_reduce<<<(unsigned)chunks, 256, 0, s>>>(counts, nc, sums);
      k_scan_exclusive<<<1, 1024, 0, s>>>(sums, chunks);
      k_scan_apply<<<(unsigned)chunks, 256, 0, s>>>(counts, nc, sums);
    }
    k_radix_scatter<<<(unsigned)tiles, kThreads, 0, s>>>(ka, va, kb, vb, E, shift, counts, tiles);
    uint32_t* t0 = ka; ka = kb; kb = t0;
    uint32_t* t1 = va; va = vb; vb = t1;
  }
  k_rowptr<<<grid_for(n_rows + 1), 256, 0, s>>>(ka, E, n_rows, rowptr);
  k_finish<<<grid_for(E), 256, 0, s>>>(va, edge_index, E, key_row, col, perm);
  return check_launch("hgin_csr_build");
}

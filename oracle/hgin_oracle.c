/*
 * ORACLE — test infrastructure only (never linked into the product).  Plain-C restatement of the
 * hot path's integer / byte work and of its sequential fp32 sums, used by tests/ to check libhgin.so.
 * Build: `make -C oracle` (gcc, -ffp-contract=off: no FMA contraction; x86-64 SSE single precision).
 *
 *   oracle_csr_build     stable counting sort of a [2, E] int64 edge_index by one endpoint.  Follows the
 *                        accumulation order of CPU scatter_add_ / index_add_ (torch_scatter.scatter sum at
 *                        PyG propagate <- reference models.py:208): within a row, original edge order.
 *   oracle_aggregate_f32 models.py:208 (propagate, aggr='add' models.py:186, identity message :219-220)
 *                        + models.py:210-215 (concat / add of (1 + eps) * x_r), sequential per row.
 *   oracle_philox4x32_10 Random123 Philox4x32-10 (Salmon et al., SC'11), published algorithm; pinned by its
 *                        published known-answer vectors in tests/test_oracle_c.py.
 *   oracle_neg_sample    build-defined sampler (NOT IN REFERENCE; include/hgin.h A10 spec).
 *   oracle_dot_decode_*  build-defined decoder (NOT IN REFERENCE; include/hgin.h A11 spec).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_csr_build(const int64_t* ei, int64_t E, int key_row, int64_t n_rows, int64_t n_cols,
                     int32_t* rowptr, int32_t* col, int32_t* perm) {
  const int64_t* key = ei + (int64_t)key_row * E;
  const int64_t* other = ei + (int64_t)(1 - key_row) * E;
  int status = 0;
  for (int64_t r = 0; r <= n_rows; ++r) rowptr[r] = 0;
  for (int64_t e = 0; e < E; ++e) {
    if (key[e] < 0 || key[e] >= n_rows) { status |= 1; continue; }
    if (other[e] < 0 || other[e] >= n_cols) status |= 2;
    rowptr[key[e] + 1]++;
  }
  if (status & 1) return status;
  for (int64_t r = 0; r < n_rows; ++r) rowptr[r + 1] += rowptr[r];
  int32_t* cursor = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_rows > 0 ? n_rows : 1));
  memcpy(cursor, rowptr, sizeof(int32_t) * (size_t)n_rows);
  for (int64_t e = 0; e < E; ++e) {  /* increasing e: stable */
    const int32_t pos = cursor[key[e]]++;
    col[pos] = (int32_t)other[e];
    if (perm) perm[pos] = (int32_t)e;
  }
  free(cursor);
  return status;
}

void oracle_aggregate_f32(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* x_src,
                          int64_t ld_src, int64_t f_src, const float* x_dst, int64_t ld_dst, int64_t f_dst,
                          float eps, int mode, float* out, int64_t ld_out) {
  const float s = 1.0f + eps;
  for (int64_t r = 0; r < n_rows; ++r) {
    float* o = out + r * ld_out;
    for (int64_t f = 0; f < f_src; ++f) {
      float acc = 0.0f;
      for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) acc += x_src[(int64_t)col[k] * ld_src + f];
      if (mode == 1) {
        const float t = s * x_dst[r * ld_dst + f];
        acc = acc + t;
      }
      o[f] = acc;
    }
    if (mode == 2)
      for (int64_t f = 0; f < f_dst; ++f) o[f_src + f] = s * x_dst[r * ld_dst + f];
  }
}

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c0;
    const uint64_t p1 = (uint64_t)M1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0;
    k1 += W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void oracle_neg_sample(uint64_t seed, uint64_t offset, int64_t n, int64_t n_dst, int32_t* out) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t c = offset + (uint64_t)i;
    const uint64_t b = c >> 2;
    const uint32_t ctr[4] = {(uint32_t)b, (uint32_t)(b >> 32), 0u, 0u};
    uint32_t x[4];
    oracle_philox4x32_10(ctr, key, x);
    out[i] = (int32_t)(((uint64_t)x[c & 3] * (uint64_t)n_dst) >> 32);
  }
}

void oracle_dot_decode_fwd_f32(const int32_t* src, const int32_t* dst, int64_t n, const float* zs, int64_t lds,
                               const float* zd, int64_t ldd, int64_t F, float* score) {
  for (int64_t e = 0; e < n; ++e) {
    double acc = 0.0; /* reference value in double; the device reduces in a different order (tolerance) */
    for (int64_t f = 0; f < F; ++f) acc += (double)zs[(int64_t)src[e] * lds + f] * (double)zd[(int64_t)dst[e] * ldd + f];
    score[e] = (float)acc;
  }
}

void oracle_dot_decode_bwd_f32(const int32_t* rowptr, const int32_t* col, const int32_t* perm, int64_t n_rows,
                               const float* g, const float* zo, int64_t ldo, int64_t F, float* gz, int64_t ldg) {
  for (int64_t r = 0; r < n_rows; ++r)
    for (int64_t f = 0; f < F; ++f) {
      float acc = 0.0f;
      for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
        const float t = g[perm[k]] * zo[(int64_t)col[k] * ldo + f];
        acc = acc + t;
      }
      gz[r * ldg + f] = acc;
    }
}

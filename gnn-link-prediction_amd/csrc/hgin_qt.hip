// F4 — queueing-theory baseline, the reference's other gather / scatter user.
//
// Reference: QTBaseline.forward (models.py:54-158) over the homogeneous sample graph, run on the CPU
// (device='cpu' forced at models.py:72-73, :89, :153) inside dataset preprocessing (dataset.py:86,
// :105-106): per iteration a Python loop over path positions k with gather / in-place multiply /
// torch_scatter sum (models.py:103-121), M/M/1/B blocking probabilities (models.py:125-132), a 32-term
// occupancy series (models.py:139-145), then a gather + scatter for the per-path delay (models.py:149-158).
//
// Here the path<->link edges are grouped once into source runs (a path's edges in route order; a link's
// edges to its paths) and a CSR by destination whose rows list edges by (position, edge id) — exactly the
// order in which the reference's per-position scatters add up.  Per iteration:
//   k_qt_traffic   thread per run: the running product traffic_k = traffic_{k-1} * (1 - bp[dst_{k-1}])
//                  written per edge (the reference's position loop, collapsed per path)
//   k_qt_link_sum  thread per vertex: T[v] = ((0 + S_0) + S_1) + ..., S_k = the in-order sum of that
//                  position's contributions (the reference's `T += scatter(...)` per k, same rounding)
//   k_qt_links     thread per link: rho, M/M/1/B blocking probability, pi_0 and the occupancy series
// and once at the end k_qt_delay, thread per run: the per-path sum of occupancy * 32000 / capacity.
#include "hgin_common.h"

namespace hgin {
namespace {

__global__ __launch_bounds__(256) void k_qt_traffic(const int32_t* __restrict__ run_ptr, int64_t n_runs,
                                                    const int32_t* __restrict__ run_src,
                                                    const int32_t* __restrict__ dst, const float* __restrict__ a,
                                                    const float* __restrict__ bp, float* __restrict__ val) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_runs) return;
  float t = a[run_src[r]];
  const int e1 = run_ptr[r + 1];
  for (int e = run_ptr[r]; e < e1; ++e) {
    val[e] = t;
    t = __fmul_rn(t, __fsub_rn(1.0f, bp[dst[e]]));
  }
}

__global__ __launch_bounds__(256) void k_qt_link_sum(const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col, const int32_t* __restrict__ pos,
                                                     const float* __restrict__ val, int64_t n_rows,
                                                     float* __restrict__ t_out) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_rows) return;
  float t = 0.0f, s = 0.0f;
  int cur = -1;
  const int k1 = rowptr[v + 1];
  for (int k = rowptr[v]; k < k1; ++k) {
    const int e = col[k];
    const int p = pos[e];
    if (p != cur) {
      if (cur >= 0) t = __fadd_rn(t, s);
      s = 0.0f;
      cur = p;
    }
    s = __fadd_rn(s, val[e]);
  }
  if (cur >= 0) t = __fadd_rn(t, s);
  t_out[v] = t;
}

__device__ __forceinline__ float pow_int(float x, int n) { return powf(x, (float)n); }

// bp must be zero for non-link vertices on entry (the reference recomputes it with rho = 0 there).
__global__ __launch_bounds__(256) void k_qt_links(const int32_t* __restrict__ link_ids, int64_t n_links,
                                                  const float* __restrict__ t_sum, const float* __restrict__ cap,
                                                  const float* __restrict__ cap_raw, int buffer,
                                                  float* __restrict__ bp, float* __restrict__ rho_out,
                                                  float* __restrict__ pi0_out, float* __restrict__ occ_out,
                                                  float* __restrict__ x_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_links) return;
  const int v = link_ids[i];
  const float rho = __fdiv_rn(t_sum[v], cap[i]);
  const float pb = pow_int(rho, buffer), pb1 = pow_int(rho, buffer + 1);
  const float om = __fsub_rn(1.0f, rho);
  bp[v] = __fdiv_rn(__fmul_rn(om, pb), __fadd_rn(__fsub_rn(1.0f, pb1), 1e-08f));
  float pi0 = __fdiv_rn(om, __fsub_rn(1.0f, pb1));
  float occ = pi0;
  for (int j = 0; j < 32; ++j) {
    pi0 = __fmul_rn(pi0, rho);
    occ = __fadd_rn(occ, __fmul_rn((float)(j + 1), pi0));
  }
  occ = __fdiv_rn(occ, 32.0f);
  rho_out[i] = rho;
  pi0_out[i] = pi0;
  occ_out[i] = occ;
  x_out[v] = __fdiv_rn(__fmul_rn(occ, 32000.0f), cap_raw[i]);
}

__global__ __launch_bounds__(256) void k_qt_delay(const int32_t* __restrict__ run_ptr, int64_t n_runs,
                                                  const int32_t* __restrict__ run_src, const int32_t* __restrict__ dst,
                                                  const float* __restrict__ x, float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_runs) return;
  float s = 0.0f;
  const int e1 = run_ptr[r + 1];
  for (int e = run_ptr[r]; e < e1; ++e) s = __fadd_rn(s, x[dst[e]]);
  out[run_src[r]] = s;
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_qt_traffic(const int32_t* run_ptr, int64_t n_runs, const int32_t* run_src, const int32_t* dst,
                               const float* a, const float* bp, float* val, void* stream) {
  HGIN_ARG_CHECK(n_runs >= 0, "hgin_qt_traffic: bad size");
  if (n_runs == 0) return HGIN_OK;
  HGIN_ARG_CHECK(run_ptr && run_src && dst && a && bp && val, "hgin_qt_traffic: NULL operand");
  k_qt_traffic<<<(unsigned)ceil_div(n_runs, 256), 256, 0, as_stream(stream)>>>(run_ptr, n_runs, run_src, dst, a, bp,
                                                                              val);
  return check_launch("hgin_qt_traffic");
}

extern "C" int hgin_qt_link_sum(const int32_t* rowptr, const int32_t* col, const int32_t* pos, const float* val,
                                int64_t n_rows, float* t_out, void* stream) {
  HGIN_ARG_CHECK(n_rows >= 0, "hgin_qt_link_sum: bad size");
  if (n_rows == 0) return HGIN_OK;
  HGIN_ARG_CHECK(rowptr && t_out, "hgin_qt_link_sum: NULL operand");
  k_qt_link_sum<<<(unsigned)ceil_div(n_rows, 256), 256, 0, as_stream(stream)>>>(rowptr, col, pos, val, n_rows, t_out);
  return check_launch("hgin_qt_link_sum");
}

extern "C" int hgin_qt_links(const int32_t* link_ids, int64_t n_links, const float* t_sum, const float* cap,
                             const float* cap_raw, int buffer, float* bp, float* rho, float* pi0, float* occ,
                             float* x, void* stream) {
  HGIN_ARG_CHECK(n_links >= 0 && buffer >= 0, "hgin_qt_links: bad size");
  if (n_links == 0) return HGIN_OK;
  HGIN_ARG_CHECK(link_ids && t_sum && cap && cap_raw && bp && rho && pi0 && occ && x, "hgin_qt_links: NULL operand");
  k_qt_links<<<(unsigned)ceil_div(n_links, 256), 256, 0, as_stream(stream)>>>(link_ids, n_links, t_sum, cap, cap_raw,
                                                                             buffer, bp, rho, pi0, occ, x);
  return check_launch("hgin_qt_links");
}

extern "C" int hgin_qt_delay(const int32_t* run_ptr, int64_t n_runs, const int32_t* run_src, const int32_t* dst,
                             const float* x, float* out, void* stream) {
  HGIN_ARG_CHECK(n_runs >= 0, "hgin_qt_delay: bad size");
  if (n_runs == 0) return HGIN_OK;
  HGIN_ARG_CHECK(run_ptr && run_src && dst && x && out, "hgin_qt_delay: NULL operand");
  k_qt_delay<<<(unsigned)ceil_div(n_runs, 256), 256, 0, as_stream(stream)>>>(run_ptr, n_runs, run_src, dst, x, out);
  return check_launch("hgin_qt_delay");
}

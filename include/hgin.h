/*
 * hgin.h — C ABI of libhgin.so, the MI355X (gfx950) heterogeneous-GIN hot path.
 *
 * The reference (youssefshoeb/GNN-Link-Prediction) has no native code: its hot path is PyG
 * `MessagePassing.propagate` + `torch_scatter.scatter` + `torch.nn.Linear`/`PReLU` reached from
 * `models.py`.  Each entry point below names the reference interface it replaces (file:line in the
 * reference tree).  The Python host (gnn-link-prediction_amd/hgin) binds this header with ctypes;
 * INTEGRATION.md shows the binding.
 *
 * Conventions (all functions):
 *   - plain C types; device pointers are `void*`/typed pointers into HBM owned and allocated by the
 *     caller; kernels never allocate.  Scratch comes from a `*_workspace_size` query + caller buffer.
 *   - every call is asynchronous on the caller's HIP stream, passed as `void* stream`
 *     (a `hipStream_t`; NULL = the default stream).  Nothing here synchronises the device, so the calls
 *     can be captured into a hipGraph.
 *   - return value: 0 = ok, > 0 = a hipError_t from the launch, < 0 = argument error (HGIN_E_*).
 *     `hgin_last_error()` returns a thread-local message for the last failing call.
 *   - row-major matrices carry an explicit leading dimension (elements, not bytes).
 *   - stateless and re-entrant; one host thread per GPU process.
 */
#ifndef HGIN_H_
#define HGIN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGIN_ABI_VERSION 8

#define HGIN_OK 0
#define HGIN_E_ARG (-1)        /* bad size / null pointer / unsupported combination */
#define HGIN_E_ALIGN (-2)      /* pointer or leading dimension misaligned for the chosen path */
#define HGIN_E_WORKSPACE (-3)  /* workspace too small */

/* combine modes of the GIN self term, models.py:210-215 */
#define HGIN_COMBINE_NONE 0    /* out = aggregate only (also: every backward aggregate)          */
#define HGIN_COMBINE_ADD 1     /* out = aggregate + (1 + eps) * x_dst          (models.py:215)    */
#define HGIN_COMBINE_CONCAT 2  /* out = [aggregate | (1 + eps) * x_dst]        (models.py:212-213) */

/* status word bits written by hgin_csr_build into *d_status (device int32) */
#define HGIN_STATUS_ROW_OOR 1  /* a row index (the sorted key) was < 0 or >= n_rows */
#define HGIN_STATUS_COL_OOR 2  /* a column index was < 0 or >= n_cols               */
#define HGIN_STATUS_UNSORTED 4 /* a batch vector was not non-decreasing (global pooling) */

int hgin_abi_version(void);
const char* hgin_last_error(void);

/* Launch trace (test / diagnostics; no reference counterpart).  hgin_trace_enable(1) clears the record and
 * starts recording, at every dispatch site, the kernel variant launched (one '\n'-terminated tag per launch,
 * e.g. "k_ws_f32<256,256,EPI1>"); hgin_trace_enable(0) stops.  hgin_trace_read copies the record into buf
 * (NUL-terminated, at most cap - 1 bytes; the record is drained when it fits) and returns its full length.
 * Host-side only: nothing is synchronised. */
int hgin_trace_enable(int on);
size_t hgin_trace_read(char* buf, size_t cap);

/* ---- A12: COO -> CSR / CSC (stable) ------------------------------------------------------------
 * Replaces nothing in the reference directly: PyG scatters unsorted COO with atomics
 * (torch_scatter.scatter <- MessagePassing.propagate <- models.py:208).  The stable sort keeps, inside
 * every row, the original edge order, which is exactly the order CPU `scatter_add_` / `index_add_`
 * accumulate in, so segmented sums over this CSR are bit-identical to the reference's CPU path.
 *
 * edge_index: int64 [2, n_edges] row-major (the PyG layout, dataset.py:112-117).
 * key_row = 1: rows are destinations (CSR for the forward aggregate); key_row = 0: rows are sources
 *              (CSC, for the backward of index_select).
 * Outputs: rowptr int32 [n_rows + 1]; col int32 [n_edges] = the other endpoint, in sorted order;
 *          perm int32 [n_edges] = original edge id of each sorted position (may be NULL).
 * d_status: device int32, OR-ed with HGIN_STATUS_* on out-of-range indices (caller zeroes it).
 * n_edges, n_rows, n_cols < 2^31. */
int hgin_csr_workspace_size(int64_t n_edges, int64_t n_rows, size_t* bytes);
int hgin_csr_build(const int64_t* edge_index, int64_t n_edges, int key_row, int64_t n_rows,
                   int64_t n_cols, int32_t* rowptr, int32_t* col, int32_t* perm, int32_t* d_status,
                   void* workspace, size_t workspace_bytes, void* stream);

/* ---- A3 + A4: GINConv message + aggregate + (1+eps) combine -------------------------------------
 * Replaces: MessagePassing.propagate (models.py:208: index_select gather + torch_scatter sum with
 * aggr='add', models.py:186; identity message models.py:219-220) fused with the self term
 * (models.py:210-215) — no [E, F] message tensor, no atomics, no separate cat / add kernel.
 *   agg[r, f]  = sum_{k = rowptr[r]}^{rowptr[r+1]-1} x_src[col[k], f]   (sequential in k, fp32, no FMA)
 *   NONE:   out[r, 0:f_src]              = agg
 *   ADD:    out[r, f]                    = agg + ((1 + eps[0]) * x_dst[r, f])   (f_dst == f_src)
 *   CONCAT: out[r, 0:f_src] = agg;  out[r, f_src:f_src+f_dst] = (1 + eps[0]) * x_dst[r, :]
 * eps: device float[1] (the GINConv eps Parameter, models.py:191-194).  Rows with no edges get 0.
 * out must not overlap x_src or x_dst (the kernels read them through restrict-qualified pointers); the
 * backward's running-gradient accumulation (ADD, eps 0) writes a fresh buffer for that reason.
 * Bit-exact against CPU scatter_add_ + cat / add on the same inputs. */
int hgin_aggregate_f32(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                       const float* x_src, int64_t ld_src, int64_t f_src,
                       const float* x_dst, int64_t ld_dst, int64_t f_dst,
                       const float* eps, int combine, float* out, int64_t ld_out, void* stream);

/* ---- A7 input: global mean / max pooling of the path features (GLOBAL_FEATS) --------------------------
 * Replaces torch_geometric.nn.global_mean_pool / global_max_pool of origin_input["path"] by path_batch and the
 * torch.gather that broadcasts them back to the rows (models.py:347-352; torch_scatter scatter mean / max):
 *   out[r, 0:f]  = mean of x[q, :] over the rows q of r's graph   (sequential row-order fp32 sum, one division)
 *   out[r, f:2f] = max  of x[q, :] over the same rows             (NaN propagates)
 * batch: int64 [n_rows] graph ids, non-decreasing (PyG collation, dataset.py:239-244: each graph's rows are one
 * contiguous run; ids may skip values); a descending pair ORs HGIN_STATUS_UNSORTED into *d_status (device int32,
 * caller zeroes it) and the outputs are then unspecified.  Deterministic; for graphs of at most 4096 rows the mean
 * is bit-identical to CPU scatter mean; longer graphs are summed in 2048-row chunk partials added in chunk order
 * (within fp32 rounding of the sequential sum).  f <= 4096; out must not overlap x.  No host synchronisation.
 * workspace: hgin_global_pool_workspace_size(n_rows, f). */
int hgin_global_pool_workspace_size(int64_t n_rows, int64_t f, size_t* bytes);
int hgin_global_pool_f32(const int64_t* batch, int64_t n_rows, const float* x, int64_t ldx, int64_t f,
                         float* out, int64_t ld_out, int* d_status, void* workspace, size_t workspace_bytes,
                         void* stream);
int hgin_global_pool_bf16(const int64_t* batch, int64_t n_rows, const uint16_t* x, int64_t ldx, int64_t f,
                          uint16_t* out, int64_t ld_out, int* d_status, void* workspace, size_t workspace_bytes,
                          void* stream);

/* ---- A9: backward of the combine -----------------------------------------------------------------
 * Replaces the autograd of `(1 + eps) * x_r` + cat/add (models.py:212-215):
 *   g_x_dst[r, f] = (1 + eps) * g[r, f]                 (written if g_x_dst != NULL)
 *   g_eps[0]      = sum_{r, f} g[r, f] * x_dst[r, f]    (deterministic two-level reduction)
 * g points at the self-term columns of the combine gradient (ld_g is its row stride).
 * workspace: hgin_combine_bwd_workspace_size(n_rows) bytes. */
int hgin_combine_bwd_workspace_size(int64_t n_rows, size_t* bytes);
int hgin_combine_bwd_f32(const float* g, int64_t ld_g, const float* x_dst, int64_t ld_dst,
                         int64_t n_rows, int64_t f_dst, const float* eps, float* g_x_dst,
                         int64_t ld_gx, float* g_eps, void* workspace, size_t workspace_bytes,
                         void* stream);

/* ---- A5: GIN MLP update on MFMA ------------------------------------------------------------------
 * Replaces GINLayer.mlp = Sequential(Linear(K, N), PReLU()) applied at models.py:217 (built at
 * models.py:236-239) and, when `accum` != NULL, the per-dst-type sum of HeteroConv(aggr='sum')
 * (models.py:286-298) for the second relation into the same node type:
 *   z = [a1 | a2] @ w^T + bias;  y = (z > 0 ? z : prelu[0] * z) [+ accum]
 * The A operand is the column concatenation of a1 ([M, k1], lda1) and a2 ([M, K - k1], lda2; NULL when
 * k1 == K), which also replaces the readout's torch.cat((x_path, raw path features)) (models.py:362-371).
 * a2_eps (device float[1], may be NULL): the a2 columns enter as (1 + a2_eps[0]) * a2 — the concat GINConv's
 * self term cat(aggregate, (1 + eps) * x_dst) (models.py:212-213) formed as the tile is loaded (the same
 * single-rounded fp32 product the aggregate's epilogue would store), so the [N_dst, F_src + F_dst] concat
 * need not be materialised.
 * w: [N, K] row-major (torch Linear.weight), bias: [N], prelu: device float[1].  Output rows are N wide.
 * z (pre-activation, saved for backward) may be NULL.  fp32 in, fp32 results (hgin_gemm_nt.hip: f32 MFMA
 * or the exact bf16 3-way operand split). */
int hgin_gin_mlp_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                         const float* a2_eps, const float* w, const float* bias, const float* prelu,
                         const float* accum, float* z, float* y, int64_t M, int64_t N, int64_t K,
                         const void* w_planes, void* stream);

/* ---- readout Linear without activation (models.py:326-330, the head Linear(mlp_layers[-1], 1)) ------
 *   y = [a1 | a2] @ w^T + bias     (same operand conventions as hgin_gin_mlp_fwd_f32) */
int hgin_linear_fwd_f32(const float* a1, int64_t lda1, int64_t k1, const float* a2, int64_t lda2,
                        const float* w, const float* bias, float* y, int64_t M, int64_t N, int64_t K,
                        const void* w_planes, void* stream);

/* ---- A3 / A9: long rows (degree skew) ------------------------------------------------------------------
 * The neighbour sums of rows too long for the row-per-lane-group walk of hgin_aggregate_* (whose CSR the
 * caller passes with these rows emptied, so it writes their self term and zeros for the sum): items holds
 * n_items chunks of consecutive edges as (begin, end) pairs into `col`, grouped by row in edge order; row j
 * of `long_rows` owns items [item_ptr[j], item_ptr[j + 1]).  Each chunk is summed in edge order (fp32), the
 * chunk sums of a row are added in chunk order, then (ADD) the self term (1 + eps[0]) * x_dst; the result
 * overwrites out[row, 0:f_src] (CONCAT's self columns stay as hgin_aggregate_* wrote them).  Deterministic
 * run to run; re-associated against the sequential sum (tolerance).  partial: n_items * f_src floats.
 * f_src, ld_src, ld_out multiples of 4. */
int hgin_aggregate_long_f32(const int32_t* col, const int32_t* items, int64_t n_items, const int32_t* long_rows,
                            const int32_t* item_ptr, int64_t n_long, const float* x_src, int64_t ld_src,
                            int64_t f_src, const float* x_dst, int64_t ld_dst, int64_t f_dst, const float* eps,
                            int combine, float* out, int64_t ld_out, float* partial, size_t partial_bytes,
                            void* stream);
int hgin_aggregate_long_bf16(const int32_t* col, const int32_t* items, int64_t n_items, const int32_t* long_rows,
                             const int32_t* item_ptr, int64_t n_long, const uint16_t* x_src, int64_t ld_src,
                             int64_t f_src, const uint16_t* x_dst, int64_t ld_dst, int64_t f_dst, const float* eps,
                             int combine, uint16_t* out, int64_t ld_out, float* partial, size_t partial_bytes,
                             void* stream);

/* ---- A9: PReLU + bias backward -------------------------------------------------------------------
 *   g_z = z > 0 ? g_y : prelu[0] * g_y;  g_prelu[0] = sum (z > 0 ? 0 : z * g_y);  g_bias[n] = sum_m g_z[m, n]
 * Deterministic (fixed-shape two-level reductions).  workspace: hgin_prelu_bwd_workspace_size. */
int hgin_prelu_bwd_workspace_size(int64_t M, int64_t N, size_t* bytes);
int hgin_prelu_bwd_f32(const float* g_y, int64_t ld_gy, const float* z, int64_t M, int64_t N, const float* prelu,
                       float* g_z, float* g_prelu, float* g_bias, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ---- plain GEMM on MFMA (backward of Linear) --------------------------------------------------------
 * c[M, N] = a[M, K] @ b[N, K]^T   ("NT", both operands K-contiguous), fp32 MFMA. */
int hgin_gemm_nt_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
                     int64_t M, int64_t N, int64_t K, const void* b_planes, void* stream);

/* ---- NT GEMM operand planes (ABI 2) --------------------------------------------------------------------
 * Every NT GEMM entry point (hgin_gin_mlp_fwd_*, hgin_linear_fwd_*, hgin_gemm_nt_*, hgin_gemm_nt_combine_*)
 * takes `w_planes` / `b_planes`: NULL, or the B operand ([N, K], the weight) pre-converted by
 * hgin_nt_planes_* — fp32: its three bf16 split planes, bf16: a copy — in the per-K-stage, XOR-swizzled
 * layout of the LDS-DMA GEMM kernel (k_nt2 in hgin_gemm_nt.hip).  With planes, shapes the kernel takes
 * (K and the A split column multiples of 32 (fp32) / 64 (bf16), 16-B aligned A rows, N a multiple of 128) run
 * on it; everything else runs on the register-staged kernel.  Results are bit-identical either way.
 * Size: hgin_nt_planes_size (elem_bytes 4 or 2) = N * K * 6 (fp32) or N * K * 2 (bf16) bytes. */
int hgin_nt_planes_size(int64_t N, int64_t K, int elem_bytes, size_t* bytes);
int hgin_nt_planes_f32(const float* b, int64_t ldb, int64_t N, int64_t K, void* out, void* stream);
int hgin_nt_planes_bf16(const uint16_t* b, int64_t ldb, int64_t N, int64_t K, void* out, void* stream);

/* ---- A9: dX GEMM with the self term's backward fused --------------------------------------------------
 * Replaces hgin_gemm_nt_* followed by hgin_combine_bwd_* in a GINConv backward (models.py:210-217 reached
 * from train.py:43): c[M, N] = a[M, K] @ b[N, K]^T (= g_comb = g_z W) and, over the self columns [cs, N)
 * (cs = F_src for concat, 0 for add; a multiple of 4), with C as stored:
 *   g_dst[m, j] = (1 + eps[0]) * c[m, cs + j]   (g_dst may be NULL)
 *   g_eps[0]    = sum_{m, j} c[m, cs + j] * x_dst[m, j]      (fixed-order per-workgroup partials + final)
 * so g_comb is not read back.  g_prev (may be NULL; may alias g_dst; row stride ld_gp): another relation's
 * gradient of the same node type, which g_dst accumulates onto (g_dst = g_prev + (1 + eps) c, one rounding
 * more) — autograd's gradient sum over the relations sharing x_dst, fused (hgin/ops.py hetero layer).
 * workspace: hgin_gemm_nt_combine_workspace_size.  Deterministic. */
int hgin_gemm_nt_combine_workspace_size(int64_t M, int64_t N, size_t* bytes);
int hgin_gemm_nt_combine_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc,
                             int64_t M, int64_t N, int64_t K, const float* x_dst, int64_t ld_xd, float* g_dst,
                             int64_t ld_gd, const float* g_prev, int64_t ld_gp, int64_t cs, const float* eps,
                             float* g_eps, void* workspace, size_t workspace_bytes, const void* b_planes,
                             void* stream);
int hgin_gemm_nt_combine_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, uint16_t* c,
                              int64_t ldc, int64_t M, int64_t N, int64_t K, const uint16_t* x_dst, int64_t ld_xd,
                              uint16_t* g_dst, int64_t ld_gd, const uint16_t* g_prev, int64_t ld_gp, int64_t cs,
                              const float* eps, float* g_eps, void* workspace, size_t workspace_bytes,
                              const void* b_planes, void* stream);

/* ---- weight-gradient GEMM (backward of Linear: dW = g_z^T X) ----------------------------------------
 * out[N, K] = a[M, N]^T @ [b1 | b2],  b1 = columns [0, k1) ([M, k1], ldb1), b2 = columns [k1, K) ([M, K-k1],
 * ldb2; may be NULL when k1 == K).  Reduction over M split across workgroups into fp32 slabs summed in a
 * fixed order (deterministic).  workspace: hgin_gemm_tn_workspace_size. */
int hgin_gemm_tn_workspace_size(int64_t M, int64_t N, int64_t K, size_t* bytes);
int hgin_gemm_tn_f32(const float* a, int64_t lda, const float* b1, int64_t ldb1, int64_t k1, const float* b2,
                     int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out, int64_t ldo, void* workspace,
                     size_t workspace_bytes, void* stream);

/* ---- A9 fused: PReLU + bias backward folded into the weight-gradient GEMM ------------------------------
 * Replaces autograd of GINLayer.mlp = Sequential(Linear, PReLU) (models.py:236-239) and of the readout's
 * Linear + PReLU (models.py:300-330) at train.py:43 — hgin_prelu_bwd_* followed by hgin_gemm_tn_*:
 *   g_z = z > 0 ? g_y : prelu[0] * g_y
 *   g_w[N, K] = g_z^T @ [b1 | b2]                          (operand conventions of hgin_gemm_tn_f32)
 *   g_bias[n] = sum_m g_z[m, n];  g_prelu[0] = sum (z > 0 ? 0 : z * g_y)
 * fp32 with N, K >= 16 and g_z == NULL: one pass — g_z is formed while the A operand is staged and never
 * stored; bias / slope gradients come from per-split partials.  Otherwise (bf16, narrow shapes, or g_z
 * requested: g_z != NULL, dense, ld_gz == N) the two passes run, g_z in the caller's buffer or workspace.
 * Deterministic.  workspace: hgin_gin_mlp_bwd_w_workspace_size(M, N, K, element bytes 4 | 2, g_z != NULL).
 *
 * (A dX GEMM applying the same prologue to its A operand measured slower than the separate passes — the
 * z stream under the dX tile costs more than the g_z stream it saves — so dX reads a materialised g_z.) */
int hgin_gin_mlp_bwd_w_workspace_size(int64_t M, int64_t N, int64_t K, int elem_bytes, int have_gz, size_t* bytes);
int hgin_gin_mlp_bwd_w_f32(const float* g_y, int64_t ld_gy, const float* z, int64_t ldz, const float* prelu,
                           const float* b1, int64_t ldb1, int64_t k1, const float* b2, int64_t ldb2,
                           int64_t M, int64_t N, int64_t K, float* g_w, int64_t ldw, float* g_prelu, float* g_bias,
                           float* g_z, int64_t ld_gz, void* workspace, size_t workspace_bytes, void* stream);

/* ---- A9: self-term weight gradient of a first-layer GINConv (inputs are data) ---------------------------
 * Given G[N, KG] = g_z^T [aggregate | x_dst] (hgin_gin_mlp_bwd_w_* over both blocks; f = aggregate width):
 *   g_w[:, :f] = G[:, :f];  concat != 0: g_w[:, f:KG] = (1 + eps[0]) G[:, f:KG]
 *   g_eps[0] = sum_{n, j < KG - f} W[n, w0 + j] G[n, f + j]    (w0 = f for concat, 0 for add; W = the Linear weight)
 * i.e. d loss / d W and d loss / d eps of (1 + eps) * x_dst (models.py:210-215) without forming the [N_dst, K]
 * input gradient.  Replaces torch's scale / cat / product / sum (3-5 launches) with two.  Deterministic.
 * workspace: hgin_self_wgrad_workspace_size. */
int hgin_self_wgrad_workspace_size(int64_t N, int64_t KG, size_t* bytes);
int hgin_self_wgrad_f32(const float* G, int64_t ldg, const float* W, int64_t ldw, int64_t N, int64_t KG, int64_t f,
                        int concat, const float* eps, float* g_w, int64_t ld_gw, float* g_eps, void* workspace,
                        size_t workspace_bytes, void* stream);

/* ---- cfg5: bf16 storage + bf16 MFMA, fp32 accumulate (BASELINE.json configs[4]) ---------------------
 * Same operations and operand conventions as the fp32 entry points above; `uint16_t` = a bfloat16 bit
 * pattern.  Every sum / product is formed in fp32 and each stored bf16 value is rounded once
 * (round-to-nearest-even, NaN -> 0x7FC0 — torch's float->bfloat16 conversion).  Parameters (eps, bias,
 * prelu) stay fp32; GEMM weights are bf16 copies of the fp32 masters; weight gradients come out fp32.
 *   hgin_aggregate_bf16     fp32 sequential edge-order sum of bf16 rows, then (1+eps)*x_dst, one rounding:
 *                           bit-exact vs CPU scatter_add_ over the fp32-widened inputs + .bfloat16().
 *   hgin_gin_mlp_fwd_bf16   z, y (and accum) bf16; v_mfma_f32_32x32x16_bf16.
 *   hgin_linear_fwd_bf16    the readout head: bf16 operands, fp32 output.
 *   hgin_gemm_nt_bf16       c (bf16) = a @ b^T.
 *   hgin_gemm_tn_bf16       out (fp32) = a^T [b1 | b2]; workspace: hgin_gemm_tn_workspace_size.
 *   hgin_prelu_bwd_bf16     g_z bf16; g_prelu / g_bias fp32 sums of the unrounded fp32 g_z.
 *   hgin_combine_bwd_bf16   g_x_dst bf16; g_eps fp32. */
int hgin_aggregate_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                        const uint16_t* x_src, int64_t ld_src, int64_t f_src,
                        const uint16_t* x_dst, int64_t ld_dst, int64_t f_dst,
                        const float* eps, int combine, uint16_t* out, int64_t ld_out, void* stream);
int hgin_gin_mlp_fwd_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                          const float* a2_eps, const uint16_t* w, const float* bias, const float* prelu,
                          const uint16_t* accum, uint16_t* z, uint16_t* y, int64_t M, int64_t N, int64_t K,
                          const void* w_planes, void* stream);
int hgin_linear_fwd_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                         const uint16_t* w, const float* bias, float* y, int64_t M, int64_t N, int64_t K,
                         const void* w_planes, void* stream);
int hgin_gemm_nt_bf16(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, uint16_t* c, int64_t ldc,
                      int64_t M, int64_t N, int64_t K, const void* b_planes, void* stream);
int hgin_gemm_tn_bf16(const uint16_t* a, int64_t lda, const uint16_t* b1, int64_t ldb1, int64_t k1,
                      const uint16_t* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K, float* out, int64_t ldo,
                      void* workspace, size_t workspace_bytes, void* stream);
int hgin_prelu_bwd_bf16(const uint16_t* g_y, int64_t ld_gy, const uint16_t* z, int64_t M, int64_t N,
                        const float* prelu, uint16_t* g_z, float* g_prelu, float* g_bias, void* workspace,
                        size_t workspace_bytes, void* stream);
int hgin_gin_mlp_bwd_w_bf16(const uint16_t* g_y, int64_t ld_gy, const uint16_t* z, int64_t ldz, const float* prelu,
                            const uint16_t* b1, int64_t ldb1, int64_t k1, const uint16_t* b2, int64_t ldb2,
                            int64_t M, int64_t N, int64_t K, float* g_w, int64_t ldw, float* g_prelu,
                            float* g_bias, uint16_t* g_z, int64_t ld_gz, void* workspace, size_t workspace_bytes,
                            void* stream);
int hgin_combine_bwd_bf16(const uint16_t* g, int64_t ld_g, const uint16_t* x_dst, int64_t ld_dst,
                          int64_t n_rows, int64_t f_dst, const float* eps, uint16_t* g_x_dst, int64_t ld_gx,
                          float* g_eps, void* workspace, size_t workspace_bytes, void* stream);

/* z from y (ABI 8, round 6): a GINLayer MLP forward with no accum has y = prelu(z) exactly, so with a positive slope
 * z > 0 <=> y > 0 and z = y / slope.  hgin_gin_mlp_fwd_zy_bf16 = hgin_gin_mlp_fwd_bf16 (accum NULL) that may leave z
 * unwritten — it skips the z stores on the device when prelu[0] > 0 (the weight-stationary kernel; elsewhere it writes
 * z); hgin_gin_mlp_bwd_w_zy_bf16 = hgin_gin_mlp_bwd_w_bf16 for that layer (z / y / g_z dense [M, N], g_z required):
 * when prelu[0] > 0 it reads y in place of z (the PReLU-fused weight-stationary dW; other shapes restore z from y
 * in place first).  g_z, g_w and g_bias equal the plain pair's bit for bit; g_prelu = sum(y g_y | y <= 0) / slope,
 * the same sum up to the bf16 rounding of z.  Replaces, for the relations whose output starts a type's sum
 * (models.py:286-298 HeteroConv, the first relation into each type) and the readout's PReLU Linears, one of the
 * layer's three row streams (the z write: a third of the forward GEMM's HBM bytes). */
int hgin_gin_mlp_fwd_zy_bf16(const uint16_t* a1, int64_t lda1, int64_t k1, const uint16_t* a2, int64_t lda2,
                             const float* a2_eps, const uint16_t* w, const float* bias, const float* prelu,
                             uint16_t* z, uint16_t* y, int64_t M, int64_t N, int64_t K, void* stream);
int hgin_gin_mlp_bwd_w_zy_bf16(const uint16_t* g_y, int64_t ld_gy, uint16_t* z, const uint16_t* y,
                               const float* prelu, const uint16_t* b1, int64_t ldb1, int64_t k1,
                               const uint16_t* b2, int64_t ldb2, int64_t M, int64_t N, int64_t K, float* g_w,
                               int64_t ldw, float* g_prelu, float* g_bias, uint16_t* g_z, int64_t ld_gz,
                               void* workspace, size_t workspace_bytes, void* stream);

/* ---- F3: fused readout head + MAPE loss ------------------------------------------------------------
 * Replaces the head Linear(K, 1) (models.py:326-330, :373-374) and train.py:38-42:
 *   out[m] = sum_k h[m, k] w[k] + b[0];   *loss_value = 100 * mean_m |(out[m] - y[m]) / y[m]|   (train.py:12-13)
 * written to device memory (no host sync).  Backward, given g_loss = d J / d loss_value (device float[1]):
 *   g_out[m] = ((100 g_loss / M) * sgn(q[m])) / y[m],  q = (out - y) / y   (torch's autograd of mape)
 *   g_h[m, k] = g_out[m] w[k] (g_h may be NULL);  g_w[k] = sum_m g_out[m] h[m, k];  g_b[0] = sum_m g_out[m]
 * Fixed-order reductions (deterministic).  h: fp32 or bf16 [M, K] (ldh); w [K], b [1], y [M], out [M] fp32.
 * m_valid: NULL, or a device int32 — only rows < *m_valid are labelled: the mean runs over them and the other
 * rows get zero gradient (padded static-shape batches replayed from a hipGraph).
 * workspace: hgin_head_mape_workspace_size(M, K). */
int hgin_head_mape_workspace_size(int64_t M, int64_t K, size_t* bytes);
int hgin_head_mape_fwd_f32(const float* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* b,
                           const float* y, const int32_t* m_valid, float* out, float* loss_value, void* workspace,
                           size_t workspace_bytes, void* stream);
int hgin_head_mape_fwd_bf16(const uint16_t* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* b,
                            const float* y, const int32_t* m_valid, float* out, float* loss_value, void* workspace,
                            size_t workspace_bytes, void* stream);
int hgin_head_mape_bwd_f32(const float* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* y,
                           const float* out, const float* g_loss, const int32_t* m_valid, float* g_h, int64_t ldg,
                           float* g_w, float* g_b, void* workspace, size_t workspace_bytes, void* stream);
int hgin_head_mape_bwd_bf16(const uint16_t* h, int64_t ldh, int64_t M, int64_t K, const float* w, const float* y,
                            const float* out, const float* g_loss, const int32_t* m_valid, uint16_t* g_h,
                            int64_t ldg, float* g_w, float* g_b, void* workspace, size_t workspace_bytes,
                            void* stream);

/* ---- F4: queueing-theory baseline (replaces QTBaseline.forward, models.py:54-158, run on the CPU) ----
 * Inputs prepared once per sample graph (hgin/qt.py): the path<->link edges (edge_type 0) as source runs
 * (run_ptr int32 [n_runs + 1], run_src [n_runs], dst [E0]) and a CSR by destination over all vertices
 * whose rows list edge ids by (position in run, edge id) (rowptr [N + 1], col [E0]; pos [E0]).
 *   hgin_qt_traffic   val[e] = a[src] * prod_{earlier edges e' of the run} (1 - bp[dst[e']])   (models.py:103-121)
 *   hgin_qt_link_sum  t[v] = sum over positions k (in order) of the in-order sum of val over row v's edges
 *                     at position k  — the reference's `T += scatter(...)` per position, same rounding
 *   hgin_qt_links     per link i (vertex link_ids[i]): rho = t / cap, bp = (1-rho) rho^B / ((1 - rho^(B+1))
 *                     + 1e-8), pi_0 and the 32-term occupancy series, x[v] = occ * 32000 / cap_raw
 *                     (models.py:125-145, :153); bp must be 0 at non-link vertices on entry
 *   hgin_qt_delay     out[src] = in-order sum of x[dst] over the run (models.py:154-156) */
int hgin_qt_traffic(const int32_t* run_ptr, int64_t n_runs, const int32_t* run_src, const int32_t* dst,
                    const float* a, const float* bp, float* val, void* stream);
int hgin_qt_link_sum(const int32_t* rowptr, const int32_t* col, const int32_t* pos, const float* val,
                     int64_t n_rows, float* t_out, void* stream);
int hgin_qt_links(const int32_t* link_ids, int64_t n_links, const float* t_sum, const float* cap,
                  const float* cap_raw, int buffer, float* bp, float* rho, float* pi0, float* occ, float* x,
                  void* stream);
int hgin_qt_delay(const int32_t* run_ptr, int64_t n_runs, const int32_t* run_src, const int32_t* dst,
                  const float* x, float* out, void* stream);

/* ---- F1: device-side batch collation (replaces PyG's host Collater, dataset.py:239-244) -------------
 * Executes n_desc "segment copy with an integer shift" descriptors in one launch (device array `descs`);
 * max_count = the largest descriptor count (sizes the grid).  Kinds:
 *   HGIN_COPY_F32     dst[i] = src[i]            (float, count elements)
 *   HGIN_COPY_I32_ADD dst[i] = src[i] + add      (int32)
 *   HGIN_COPY_I64_ADD dst[i] = src[i] + add      (int64)
 *   HGIN_FILL_I64     dst[i] = add               (int64)
 *   HGIN_FILL_I32     dst[i] = (int32)add        (int32)
 *   HGIN_COPY_B16     dst[i] = src[i]            (16-bit elements: bf16 features, cfg5) */
#define HGIN_COPY_F32 0
#define HGIN_COPY_I32_ADD 1
#define HGIN_COPY_I64_ADD 2
#define HGIN_FILL_I64 3
#define HGIN_FILL_I32 4
#define HGIN_COPY_B16 5
typedef struct hgin_copy_desc {
  const void* src;
  void* dst;
  int64_t count;
  int64_t add;
  int32_t kind;
  int32_t reserved;
} hgin_copy_desc;
int hgin_batched_copy(const hgin_copy_desc* descs, int64_t n_desc, int64_t max_count, void* stream);
/* Host memory the device reads in place (F1 collation, no reference counterpart): page-locked, mapped and coherent
 * (hipHostMallocCoherent: not cached on the device, so a buffer refilled by the host between launches is never read
 * stale).  hgin_batched_copy takes its descriptor table from such a buffer directly, without a host -> device copy
 * ahead of it.  The caller owns the buffer and must not refill it before the launch reading it has finished. */
int hgin_host_alloc(size_t bytes, void** ptr);
int hgin_host_free(void* ptr);

/* ---- A10: negative-edge sampler (NOT IN REFERENCE; build-defined) --------------
 * out[i] = hi32( philox4x32_10(counter = {lo32(offset+i), hi32(offset+i), 0, 0},
 *                              key = {lo32(seed), hi32(seed)}).x  *  n_dst ),  i in [0, n)
 * (Lemire multiply-shift range reduction).  int32 output. */
int hgin_neg_sample(uint64_t seed, uint64_t offset, int64_t n, int64_t n_dst, int32_t* out,
                    void* stream);

/* ---- A11: dot-product link decoder (NOT IN REFERENCE; build-defined) ------------
 * score[e] = sum_f z_src[src[e], f] * z_dst[dst[e], f]   (fp32)
 * Backward: g_z_src[s] = sum_{e: src[e]=s} g[e] * z_dst[dst[e]] over a CSR of the pairs by src
 * (rowptr/col/perm from hgin_csr_build with key_row = 0), and symmetrically for g_z_dst. */
int hgin_dot_decode_fwd_f32(const int32_t* src, const int32_t* dst, int64_t n_pairs,
                            const float* z_src, int64_t ld_src, const float* z_dst, int64_t ld_dst,
                            int64_t F, float* score, void* stream);
int hgin_dot_decode_bwd_f32(const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                            int64_t n_rows, const float* g_score, const float* z_other,
                            int64_t ld_other, int64_t F, float* g_z, int64_t ld_g, void* stream);

/* ---- F4 widening: HetroGAT's graph attention (models.py:380-506, PyG 2.0.2 GATConv) ---------------------------
 * x_s / x_d: projected source / destination features [N, H * C] (row stride ld*), edges = the relation after
 * GATConv's self-loop handling, as CSR by destination (rowptr, col) and CSC by source (cptr, cdst, cpos = the CSR
 * position of each CSC entry).  fp32; one thread per (row, head); every sum in a fixed order (deterministic).
 *   hgin_gat_logits_f32:  a[n, h] = sum_c x[n, h, c] att[h, c]
 *   hgin_gat_fwd_f32:     alpha[k, h] (CSR order) = softmax over the row of leaky_relu(a_s[j_k, h] + a_d[i, h], slope)
 *                         (exp(e - max) / (sum + 1e-16), PyG's softmax); out[i, h, :] = sum_k alpha x_s[j_k, h, :]
 *                         + bias [+ accum].  a_d, bias, accum may be NULL.
 *   hgin_gat_bwd_dst_f32: g_pre[k, h] = d loss / d (a_s[j_k, h] + a_d[i, h]) (softmax + leaky_relu backward),
 *                         g_ad[i, h] = sum_k g_pre, g_xd[i, h, :] = g_ad[i, h] att_dst[h, :] (g_ad / g_xd may be NULL)
 *   hgin_gat_bwd_src_f32: g_as[j, h] = sum_k g_pre, g_xs[j, h, :] = sum_k alpha g_out[i_k, h, :] + g_as att_src[h, :]
 *   hgin_gat_wsum_f32:    out[h * C + c] = sum_n w[n, h] x[n, h * C + c] (w NULL: 1), fixed 256-row blocks in order;
 *                         workspace: hgin_gat_wsum_workspace_size. */
int hgin_gat_logits_f32(const float* x, int64_t ldx, int64_t n, int64_t H, int64_t C, const float* att, float* a,
                        void* stream);
int hgin_gat_fwd_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C, const float* xs,
                     int64_t ldxs, const float* as, const float* ad, float slope, const float* bias, const float* accum,
                     int64_t ld_acc, float* alpha, float* out, int64_t ldo, void* stream);
/* Round 5 (ABI 5): the forward attention in one pass, a_s formed from the gathered x_s rows (no a_s table):
 *   hgin_gat_attn_fwd_f32:  alpha / out as hgin_gat_fwd_f32 with a_s[j, h] = x_s[j, h, :] . att_src[h, :] (the same
 *                           per-lane arithmetic as hgin_gat_logits_f32's group form), the weighted sum divided once by
 *                           the softmax denominator at the end (online max / sum); needs the wave-group shape —
 *   hgin_gat_attn_supported: 1 when (H, C) and HGIN_GAT_WAVE allow it (C a multiple of 4 with C / 4 a power of two,
 *                           H * C <= 256; rows must also be 16-B aligned: HGIN_E_ARG otherwise).
 *   Replaces hgin_gat_logits_f32 (for a_s) + hgin_gat_fwd_f32 at models.py:413-418's GATConv.forward. */
int hgin_gat_attn_fwd_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                          const float* xs, int64_t ldxs, const float* att_src, const float* ad, float slope,
                          const float* bias, const float* accum, int64_t ld_acc, float* alpha, float* out, int64_t ldo,
                          void* stream);
int hgin_gat_attn_supported(int64_t H, int64_t C);
int hgin_gat_bwd_dst_f32(const int32_t* rowptr, const int32_t* col, int64_t n_dst, int64_t H, int64_t C,
                         const float* xs, int64_t ldxs, const float* g_out, int64_t ldg, const float* alpha,
                         const float* as, const float* ad, float slope, const float* att_dst, float* g_pre, float* g_ad,
                         float* g_xd, int64_t ldgxd, void* stream);
int hgin_gat_bwd_src_f32(const int32_t* cptr, const int32_t* cdst, const int32_t* cpos, int64_t n_src, int64_t H,
                         int64_t C, const float* g_out, int64_t ldg, const float* alpha, const float* g_pre,
                         const float* att_src, float* g_as, float* g_xs, int64_t ldgxs, void* stream);
int hgin_gat_wsum_workspace_size(int64_t n, int64_t H, int64_t C, size_t* bytes);
int hgin_gat_wsum_f32(const float* x, int64_t ldx, int64_t n, int64_t H, int64_t C, const float* w, float* out,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ---- F1: the fused small-batch train step (the reference's real loop: batches of small graphs) -------------------
 * hgin_sb_step: a HetroGIN forward + sqrt-MAPE backward over a padded batch in 3 L + 1 launches, or (SbArgs.gat,
 * ABI 7) a one-layer HetroGAT's (models.py:380-506: k_sb_gat_fwd, the readout, k_sb_gat_bwd, the final sum) — replaces
 * the reference's train_one_epoch body (train.py:31-44) over DataLoader batches (dataset.py:239-244)
 * (csrc/hgin_smallbatch.hip); args points to the host-filled SbArgs struct (hgin/smallbatch.py mirrors its layout;
 * hgin_sb_args_size() = its size), readout_lds = hgin_sb_readout_lds_bytes(..., with_weights = args' ro_wlds, ...):
 * the readout tile's dynamic LDS, with the hidden readout weights staged or not.  Writes every parameter gradient
 * into the flat gradient buffer and loss_value.  Deterministic. */
size_t hgin_sb_args_size(void);
int hgin_sb_args_offsets(int64_t* out, int64_t n);   /* offsetof of 19 field groups, for the host mirror's check */
int hgin_sb_readout_lds_bytes(int64_t H, int64_t f_path, int concat_path, int nhid, const int32_t* widths,
                              int with_weights, size_t* bytes);
int hgin_sb_step(const void* args, size_t args_bytes, size_t readout_lds, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HGIN_H_ */

// F1 — device-side hetero batch collation.
//
// Reference: PyG's Collater via torch_geometric.loader.DataLoader (dataset.py:239-244, consumed at
// train.py:25-28): on the host, per node type concatenate x, build the batch vector, offset every
// relation's edge_index by the running node counts; then sample.cuda() copies the batch to the device and
// the scatter kernels start from unsorted COO again.
//
// Here the whole dataset stays resident in HBM as ONE collated store (hgin/store.py) whose per-relation
// CSR / CSC were built once.  Because a graph's edges occupy a contiguous block of the store's stable
// sorted order, a batch's CSR is the concatenation of store slices shifted by (batch offset - store
// offset).  Every array of the batch — x rows, labels, batch vectors, edge_index, rowptr / col / perm of
// both directions — is one "segment copy with an integer shift" descriptor, and one launch executes them
// all: no sort, no host round trip.
#include "hgin_common.h"

namespace hgin {
namespace {

__global__ __launch_bounds__(256) void k_batched_copy(const hgin_copy_desc* __restrict__ descs, int64_t n_desc) {
  for (int64_t d = blockIdx.y; d < n_desc; d += gridDim.y) {
    const hgin_copy_desc ds = descs[d];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    switch (ds.kind) {
      case HGIN_COPY_F32: {
        const float* s = static_cast<const float*>(ds.src);
        float* o = static_cast<float*>(ds.dst);
        if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 15u) == 0) {
          const int64_t n4 = ds.count >> 2;
          for (int64_t i = t0; i < n4; i += stride)
            reinterpret_cast<float4*>(o)[i] = reinterpret_cast<const float4*>(s)[i];
          for (int64_t i = (n4 << 2) + t0; i < ds.count; i += stride) o[i] = s[i];
        } else {
          for (int64_t i = t0; i < ds.count; i += stride) o[i] = s[i];
        }
        break;
      }
      case HGIN_COPY_I32_ADD: {
        const int32_t* s = static_cast<const int32_t*>(ds.src);
        int32_t* o = static_cast<int32_t*>(ds.dst);
        for (int64_t i = t0; i < ds.count; i += stride) o[i] = (int32_t)((int64_t)s[i] + ds.add);
        break;
      }
      case HGIN_COPY_I64_ADD: {
        const int64_t* s = static_cast<const int64_t*>(ds.src);
        int64_t* o = static_cast<int64_t*>(ds.dst);
        for (int64_t i = t0; i < ds.count; i += stride) o[i] = s[i] + ds.add;
        break;
      }
      case HGIN_FILL_I64: {
        int64_t* o = static_cast<int64_t*>(ds.dst);
        for (int64_t i = t0; i < ds.count; i += stride) o[i] = ds.add;
        break;
      }
      case HGIN_FILL_I32: {
        int32_t* o = static_cast<int32_t*>(ds.dst);
        for (int64_t i = t0; i < ds.count; i += stride) o[i] = (int32_t)ds.add;
        break;
      }
      case HGIN_COPY_B16: {
        const uint16_t* s = static_cast<const uint16_t*>(ds.src);
        uint16_t* o = static_cast<uint16_t*>(ds.dst);
        if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 15u) == 0) {
          const int64_t n8 = ds.count >> 3;
          for (int64_t i = t0; i < n8; i += stride)
            reinterpret_cast<uint4*>(o)[i] = reinterpret_cast<const uint4*>(s)[i];
          for (int64_t i = (n8 << 3) + t0; i < ds.count; i += stride) o[i] = s[i];
        } else {
          for (int64_t i = t0; i < ds.count; i += stride) o[i] = s[i];
        }
        break;
      }
      default:
        break;
    }
  }
}

}  // namespace
}  // namespace hgin

using namespace hgin;

extern "C" int hgin_batched_copy(const hgin_copy_desc* descs, int64_t n_desc, int64_t max_count, void* stream) {
  HGIN_ARG_CHECK(n_desc >= 0 && max_count >= 0, "hgin_batched_copy: negative size");
  if (n_desc == 0 || max_count == 0) return HGIN_OK;
  HGIN_ARG_CHECK(descs != nullptr, "hgin_batched_copy: descs NULL");
  int64_t gx = ceil_div(max_count, 256 * 4);
  if (gx > 512) gx = 512;
  const int64_t gy = n_desc < 65535 ? n_desc : 65535;
  k_batched_copy<<<dim3((unsigned)gx, (unsigned)gy), 256, 0, as_stream(stream)>>>(descs, n_desc);
  return check_launch("hgin_batched_copy");
}

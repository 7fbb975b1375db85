// Compare gfx950's v_cvt_pk_bf16_f32 (RNE) with hgin_common.h's manual f2bf (RNE, NaN -> 0x7FC0, = torch) over
// special values and 2^24 strided bit patterns; prints the mismatches (diagnostic tool, not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../gnn-link-prediction_amd/csrc/hgin_common.h"

__global__ void k_cmp(const uint32_t* in, int n, uint32_t* hw, uint32_t* sw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float f = __uint_as_float(in[i]);
  hw[i] = hgin::cvt_pk_bf16(f, 0.0f) & 0xffffu;
  sw[i] = hgin::f2bf(f);
}

int main() {
  std::vector<uint32_t> v = {0x7fc00000u, 0x7f800001u, 0x7fbfffffu, 0xffc00000u, 0xff800001u, 0x7fffffffu, 0x7f800000u,
                             0xff800000u, 0x7f7fffffu, 0x7f7f8000u, 0x00000001u, 0x80000001u, 0x00008000u, 0x00018000u,
                             0x3f808000u, 0x3f818000u, 0x3f80ffffu, 0x7fa00000u, 0x7fd00001u};
  for (uint64_t u = 0; u < (1ull << 32); u += 4093) v.push_back((uint32_t)u);
  const int n = (int)v.size();
  uint32_t *d_in, *d_hw, *d_sw;
  hipMalloc(&d_in, n * 4); hipMalloc(&d_hw, n * 4); hipMalloc(&d_sw, n * 4);
  hipMemcpy(d_in, v.data(), n * 4, hipMemcpyHostToDevice);
  k_cmp<<<(n + 255) / 256, 256>>>(d_in, n, d_hw, d_sw);
  std::vector<uint32_t> hw(n), sw(n);
  hipMemcpy(hw.data(), d_hw, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(sw.data(), d_sw, n * 4, hipMemcpyDeviceToHost);
  long bad = 0, bad_nan = 0;
  for (int i = 0; i < n; ++i) {
    if (hw[i] == sw[i]) continue;
    const bool isnan = (v[i] & 0x7fffffffu) > 0x7f800000u;
    ++bad; bad_nan += isnan;
    if (bad <= 12) printf("in %08x: hw %04x manual %04x%s\n", v[i], hw[i], sw[i], isnan ? " (NaN)" : "");
  }
  printf("checked %d values: %ld mismatches (%ld NaN)\n", n, bad, bad_nan);
  return 0;
}

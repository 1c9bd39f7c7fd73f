// calib_gather.hip — known-byte calibration of rocprofv3 FETCH_SIZE for random 16-B gathers
// (the access pattern of K1's request rows after the coherence sort).
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced streaming reads (it reports
// half their bytes).  This program gathers n random 16-B records from a 1 GiB table (4x the
// 256 MiB Infinity Cache, so re-reads are rare and reach HBM), once per lane, and prints the
// distinct 64-B and 128-B lines those gathers touch (computed on the host from the same
// indices) next to the index stream (16 B per lane: FETCH_SIZE counts half of it) and the
// output bytes.  Run it under
//   rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gather -- tools/calib_gather
// and divide the known bytes by FETCH_SIZE (KiB x 1024): the factor tools/pmc_traffic.py
// applies to gather-dominated kernels.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/calib_gather.hip -o tools/calib_gather
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// Each lane reads 4 indices as one 16-B load (a wide coalesced stream: FETCH_SIZE counts half
// of it, the calibrated case) and gathers 4 random 16-B records.
__global__ void gather16(const uint4* __restrict__ table, const uint4* __restrict__ idx4, uint32_t n4,
                         uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const uint4 k = idx4[i];
  const uint4 a = table[k.x], b = table[k.y], c = table[k.z], d = table[k.w];
  out[i] = a.x ^ b.y ^ c.z ^ d.w;
}

int main() {
  const size_t table_bytes = size_t(1) << 30;
  const size_t records = table_bytes / 16;
  const uint32_t runs[] = {1u << 18, 1u << 20, 1u << 22};
  uint4* table = nullptr;
  CK(hipMalloc(&table, table_bytes));
  CK(hipMemset(table, 0x5A, table_bytes));
  std::mt19937_64 rng(12345);
  for (uint32_t n : runs) {
    std::vector<uint32_t> idx(n);
    std::uniform_int_distribution<uint64_t> d(0, records - 1);
    for (auto& x : idx) x = (uint32_t)d(rng);
    std::vector<uint64_t> l64(n), l128(n);
    for (uint32_t k = 0; k < n; ++k) {
      l64[k] = (uint64_t)idx[k] * 16 / 64;
      l128[k] = (uint64_t)idx[k] * 16 / 128;
    }
    std::sort(l64.begin(), l64.end());
    std::sort(l128.begin(), l128.end());
    const size_t u64 = std::unique(l64.begin(), l64.end()) - l64.begin();
    const size_t u128 = std::unique(l128.begin(), l128.end()) - l128.begin();
    uint32_t *didx = nullptr, *dout = nullptr;
    CK(hipMalloc(&didx, n * 4ull));
    CK(hipMalloc(&dout, n * 4ull));
    CK(hipMemcpy(didx, idx.data(), n * 4ull, hipMemcpyHostToDevice));
    const uint32_t n4 = n / 4;
    hipLaunchKernelGGL(gather16, dim3((n4 + 255) / 256), dim3(256), 0, 0, table, (const uint4*)didx, n4, dout);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("{\"n\": %u, \"record_bytes\": %llu, \"lines64\": %zu, \"lines128\": %zu, \"idx_bytes\": %llu, "
           "\"out_bytes\": %llu}\n",
           n, 16ull * n, u64, u128, 4ull * n, 1ull * n);
    CK(hipFree(didx));
    CK(hipFree(dout));
  }
  CK(hipFree(table));
  return 0;
}

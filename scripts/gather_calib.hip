// gather_calib.hip -- FETCH_SIZE calibration for the duplication's record gather.
//
// The duplication reads 48 B (float4 parts 0, 1 and 3) of each visible Gaussian's 64-B splat
// record in depth order, i.e. a random permutation of the record array; rocprofv3's FETCH_SIZE
// reported ~1.9x the 48 B.  MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for wide streaming
// reads (where it reads half the bytes); other access shapes must be calibrated on a known byte
// count.  This program gathers N records of a 64-MB-per-million table in a random order with the
// duplication's access shape and a few others, one kernel each, so a `rocprofv3 --pmc FETCH_SIZE`
// pass gives the bytes per record of every shape:
//   linear64    : every record, in order, all 4 parts (64 B/record)       -- the streaming reference
//   gather16    : random order, part 0 only (16 B)
//   gather32    : random order, parts 0-1 (32 B, one 32-B half of the line)
//   gather48    : random order, parts 0, 1, 3 (the duplication's 48 B)
//   gather64    : random order, all 4 parts (64 B)
// usage: gather_calib [records (default 3000000)]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

template <int MASK, bool LINEAR>
__global__ __launch_bounds__(256) void gather_kernel(const float4* __restrict__ rec,
                                                     const unsigned* __restrict__ order, size_t n,
                                                     float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const size_t g = LINEAR ? i : order[i];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (MASK & (1 << k)) {
      const float4 q = rec[4 * g + k];
      s += q.x + q.y + q.z + q.w;
    }
  out[i] = s;  // 4 B written per record (WRITE_SIZE), same for every shape
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 3000000ull;
  std::vector<unsigned> h(n);
  for (size_t i = 0; i < n; i++) h[i] = (unsigned)i;
  srand(12345);
  for (size_t i = n - 1; i > 0; i--) {  // Fisher-Yates with a 2^30-range LCG draw
    const size_t j = (((size_t)rand() << 15) ^ (size_t)rand()) % (i + 1);
    const unsigned t = h[i]; h[i] = h[j]; h[j] = t;
  }
  float4* rec = nullptr;
  unsigned* order = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&rec, n * 64));
  CHECK(hipMalloc(&order, n * 4));
  CHECK(hipMalloc(&out, n * 4));
  CHECK(hipMemset(rec, 0, n * 64));
  CHECK(hipMemcpy(order, h.data(), n * 4, hipMemcpyHostToDevice));
  const dim3 grid((unsigned)((n + 255) / 256));
  // a flush of the caches between the shapes: one 512-MB streaming pass
  void* big = nullptr;
  const size_t bigb = 512ull << 20;
  CHECK(hipMalloc(&big, bigb));
  auto flush = [&]() { return hipMemset(big, 1, bigb); };
  for (int rep = 0; rep < 2; rep++) {
    CHECK(flush());
    hipLaunchKernelGGL((gather_kernel<15, true>), grid, dim3(256), 0, 0, rec, order, n, out);
    CHECK(flush());
    hipLaunchKernelGGL((gather_kernel<1, false>), grid, dim3(256), 0, 0, rec, order, n, out);
    CHECK(flush());
    hipLaunchKernelGGL((gather_kernel<3, false>), grid, dim3(256), 0, 0, rec, order, n, out);
    CHECK(flush());
    hipLaunchKernelGGL((gather_kernel<11, false>), grid, dim3(256), 0, 0, rec, order, n, out);
    CHECK(flush());
    hipLaunchKernelGGL((gather_kernel<15, false>), grid, dim3(256), 0, 0, rec, order, n, out);
  }
  CHECK(hipDeviceSynchronize());
  printf("records %zu: linear64 gather16 gather32 gather48 gather64 (order reads 4 B/record in the "
         "gathers)\n", n);
  CHECK(hipFree(big));
  CHECK(hipFree(rec));
  CHECK(hipFree(order));
  CHECK(hipFree(out));
  return 0;
}

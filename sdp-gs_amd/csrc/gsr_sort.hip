// gsr_sort.hip -- device-wide prefix sum and stable LSD radix sort for gfx950 (wave64).
//
// Replaces the reference's CUB calls (cub::DeviceScan::InclusiveSum at
// cuda_rasterizer/rasterizer_impl.cu:277 and cub::DeviceRadixSort::SortPairs at :303-308, CUDA
// toolkit 11.6 per environment.yml:6).  The sort must be STABLE: the reference breaks equal-depth
// ties by emission order, i.e. by Gaussian index.
//
// Design: reduce-then-scan (3 launches, no inter-workgroup hand-off, hence no agent-scope
// release/acquire protocol to get wrong), and a 3-launch radix pass (histogram -> scan ->
// scatter) whose in-workgroup ranking uses wave64 ballots ("match" of the 8-bit digit) instead of
// shared-memory per-thread counters.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kScanItems = kScanTile / kThreads;   // 8
constexpr int kSortRounds = kSortTile / kThreads;  // 16

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Inclusive wave64 scan.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan across a workgroup of NW waves; lds must hold NW u32.  Returns the exclusive
// prefix of v and the workgroup total.  Contains two __syncthreads().
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  uint32_t incl = wave_incl_scan(v);
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    uint32_t c = lds[w];
    pre += (w < wid) ? c : 0u;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return pre + incl - v;
}

template <bool GATHER>
__global__ __launch_bounds__(kThreads) void scan_reduce_kernel(const uint32_t* __restrict__ in,
                                                               const uint32_t* __restrict__ gather,
                                                               size_t n,
                                                               uint32_t* __restrict__ parts) {
  __shared__ uint32_t lds[kThreads / 64];
  const size_t base = (size_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    size_t i = base + (size_t)k * kThreads + threadIdx.x;
    if (i < n) s += GATHER ? in[gather[i]] : in[i];
  }
  uint32_t total;
  block_excl_scan<kThreads / 64>(s, lds, total);
  if (threadIdx.x == 0) parts[blockIdx.x] = total;
}

// One workgroup of 1024 threads: exclusive scan of the partials in place (<= kScanMaxParts).
__global__ __launch_bounds__(1024) void scan_parts_kernel(uint32_t* __restrict__ parts, int n) {
  __shared__ uint32_t lds[16];
  constexpr int kPer = kScanMaxParts / 1024;
  uint32_t v[kPer];
  uint32_t s = 0;
  const int base = (int)threadIdx.x * kPer;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    v[k] = (base + k < n) ? parts[base + k] : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan<16>(s, lds, total);
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    if (base + k < n) parts[base + k] = pre;
    pre += v[k];
  }
}

template <bool GATHER, bool INCLUSIVE>
__global__ __launch_bounds__(kThreads) void scan_final_kernel(const uint32_t* __restrict__ in,
                                                              const uint32_t* __restrict__ gather,
                                                              size_t n,
                                                              const uint32_t* __restrict__ parts,
                                                              uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[kThreads / 64];
  const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    size_t i = base + k;
    v[k] = (i < n) ? (GATHER ? in[gather[i]] : in[i]) : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan<kThreads / 64>(s, lds, total) + parts[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    size_t i = base + k;
    uint32_t incl = pre + v[k];
    if (i < n) out[i] = INCLUSIVE ? incl : pre;
    pre = incl;
  }
}

// Lanes of this wave whose digit equals mine (among lanes with valid == true).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int bits) {
  uint64_t m = __ballot(valid);
  for (int b = 0; b < bits; b++) {
    const bool set = (d >> b) & 1u;
    const uint64_t bal = __ballot(set);
    m &= set ? bal : ~bal;
  }
  return valid ? m : 0ull;
}

__global__ __launch_bounds__(kThreads) void radix_hist_kernel(const uint32_t* __restrict__ keys,
                                                              size_t n, int shift, int bits,
                                                              uint32_t* __restrict__ hist,
                                                              uint32_t nblocks) {
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t mask = (1u << bits) - 1u;
  const int lane = lane_id();
  const size_t base = (size_t)blockIdx.x * kSortTile;
  for (int r = 0; r < kSortRounds; r++) {
    const size_t i = base + (size_t)r * kThreads + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? (keys[i] >> shift) & mask : 0u;
    const uint64_t peers = match_digit(d, valid, bits);
    if (valid && (__ffsll((long long)peers) - 1) == lane) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(kThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, size_t n, int shift,
    int bits, const uint32_t* __restrict__ hist_scanned, uint32_t nblocks,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint32_t running[256];
  __shared__ uint32_t cnt[4][256];
  __shared__ uint32_t wbase[4][256];
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  const uint32_t mask = (1u << bits) - 1u;
  running[threadIdx.x] = hist_scanned[(size_t)threadIdx.x * nblocks + blockIdx.x];
  const size_t base = (size_t)blockIdx.x * kSortTile;
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  for (int r = 0; r < kSortRounds; r++) {
    const size_t i = base + (size_t)r * kThreads + threadIdx.x;
    if (base + (size_t)r * kThreads >= n) break;  // workgroup-uniform
    const bool valid = i < n;
    const uint32_t k = valid ? kin[i] : 0u;
    const uint32_t v = valid ? vin[i] : 0u;
    const uint32_t d = (k >> shift) & mask;
    cnt[0][threadIdx.x] = 0;
    cnt[1][threadIdx.x] = 0;
    cnt[2][threadIdx.x] = 0;
    cnt[3][threadIdx.x] = 0;
    __syncthreads();
    const uint64_t peers = match_digit(d, valid, bits);
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (valid && (__ffsll((long long)peers) - 1) == lane) cnt[wid][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    {
      const uint32_t dd = threadIdx.x;
      const uint32_t c0 = cnt[0][dd], c1 = cnt[1][dd], c2 = cnt[2][dd], c3 = cnt[3][dd];
      const uint32_t b0 = running[dd];
      wbase[0][dd] = b0;
      wbase[1][dd] = b0 + c0;
      wbase[2][dd] = b0 + c0 + c1;
      wbase[3][dd] = b0 + c0 + c1 + c2;
      running[dd] = b0 + c0 + c1 + c2 + c3;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = wbase[wid][d] + rank;
      kout[pos] = k;
      vout[pos] = v;
    }
  }
}

}  // namespace

hipError_t scan_u32(const uint32_t* in, const uint32_t* gather, uint32_t* out, size_t n,
                    bool inclusive, uint32_t* parts, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const size_t np = scan_parts(n);
  if (np > (size_t)kScanMaxParts) return hipErrorInvalidValue;
  const dim3 grid((unsigned)np);
  if (gather) hipLaunchKernelGGL(scan_reduce_kernel<true>, grid, dim3(kThreads), 0, s, in, gather, n, parts);
  else hipLaunchKernelGGL(scan_reduce_kernel<false>, grid, dim3(kThreads), 0, s, in, gather, n, parts);
  hipLaunchKernelGGL(scan_parts_kernel, dim3(1), dim3(1024), 0, s, parts, (int)np);
  if (gather) {
    if (inclusive) hipLaunchKernelGGL((scan_final_kernel<true, true>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
    else hipLaunchKernelGGL((scan_final_kernel<true, false>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
  } else {
    if (inclusive) hipLaunchKernelGGL((scan_final_kernel<false, true>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
    else hipLaunchKernelGGL((scan_final_kernel<false, false>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
  }
  return hipGetLastError();
}

hipError_t radix_sort_pairs(uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb, size_t n,
                            int bits, SortScratch scratch, bool* result_in_b, hipStream_t s) {
  *result_in_b = false;
  if (n == 0 || bits <= 0) return hipSuccess;
  const uint32_t nb = (uint32_t)sort_blocks(n);
  const size_t hl = sort_hist_len(n);
  uint32_t *kin = ka, *vin = va, *kout = kb, *vout = vb;
  bool in_b = false;
  for (int shift = 0; shift < bits; shift += 8) {
    const int dbits = (bits - shift) < 8 ? (bits - shift) : 8;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(kThreads), 0, s, kin, n, shift, dbits,
                       scratch.hist, nb);
    hipError_t e = scan_u32(scratch.hist, nullptr, scratch.hist, hl, false, scratch.parts, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(nb), dim3(kThreads), 0, s, kin, vin, n, shift,
                       dbits, scratch.hist, nb, kout, vout);
    uint32_t* t;
    t = kin; kin = kout; kout = t;
    t = vin; vin = vout; vout = t;
    in_b = !in_b;
  }
  *result_in_b = in_b;
  return hipGetLastError();
}

}  // namespace gsr

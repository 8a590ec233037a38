// gsr_binning.hip -- tile binning: key duplication and per-tile ranges.
//
// Reference behaviour: duplicateWithKeys (cuda_rasterizer/rasterizer_impl.cu:70-111) emits one
// (tile << 32 | depth_bits, gaussian_id) pair per overlapped tile, SortPairs sorts them stably over
// 32 + bit bits (:300-308) and identifyTileRanges (:116-138) finds each tile's [start, end).
//
// gfx950 design: the order (tile, depth_bits, gaussian_id) is produced by a
// depth-first two-stage sort instead of one 45-bit sort of R 12-byte pairs:
//   1. stable 32-bit radix sort of the P depth keys (ties keep Gaussian order),
//   2. duplication in depth order (this file), emitting 4-byte tile ids,
//   3. stable radix sort of the R tile ids over `bit` bits (2 passes at 1080p instead of 6).
// Stage 3 is stable, so instances with equal tile keep the depth-sorted emission order; the
// resulting point_list is identical to the reference's.
#include "gsr_device.h"
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;

// wave-scope ordering of LDS stores before other lanes' loads of the same wave
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One lane per depth-sorted Gaussian, enumerating its kept tiles row-major over its tile
// rectangle (the reference's emission order inside one Gaussian, rasterizer_impl.cu:98-109).  A
// wave's 64 depth-consecutive Gaussians own one contiguous range of instances: every lane writes
// its tile ids into a per-wave LDS window, then the wave copies the window out with coalesced
// stores (each lane storing at its own offsets puts 64 scattered lines in every store
// instruction).  Each Gaussian's kept range per tile row comes from the preprocess's packed
// ranges (rectangles of at most 4 rows x 15 tiles), else from band_row_range itself.  The packed
// case reads only the Gaussian's 8-B binning word (bword), the rest its record.
// With hist (the multi-view forward): every instance's tile digits of the tile sort's passes are
// counted in the workgroup's LDS histogram hist[tpasses][256] (duplicate_body flushes it), so the
// tile sort needs no digit-totals launch re-reading the R keys.
// One chunk of kThreads depth-sorted Gaussians: s0 = its first.
constexpr int kWin = 256;  // instances per wave window
__device__ __forceinline__ void duplicate_chunk(int P, int s0, const uint32_t* __restrict__ order,
                                                const uint32_t* __restrict__ offsets,
                                                const float4* __restrict__ rec, uint32_t gx,
                                                uint32_t gy, uint32_t* __restrict__ tkey,
                                                uint32_t* __restrict__ tval, uint32_t R,
                                                uint32_t* __restrict__ egid,
                                                uint32_t* __restrict__ ebeg, uint32_t pack,
                                                const uint2* __restrict__ bword,
                                                uint32_t (*s_key)[kWin], uint32_t (*s_val)[kWin],
                                                uint32_t (*s_eg)[kWin], uint32_t* hist, int tdw,
                                                int tpasses) {
  const int s = s0 + (int)threadIdx.x;
  const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
  const int sw0 = s - lane;
  if (sw0 >= P) return;  // wave-uniform
  const bool valid = s < P;
  uint32_t off = valid ? ((s == 0) ? 0u : offsets[s - 1]) : 0u;
  const uint32_t end = valid ? min(offsets[s], R) : 0u;
  // the wave's instance range: offsets are a prefix sum, so it runs from lane 0's first to the
  // last valid lane's end
  const uint32_t obase = (uint32_t)__shfl((int)off, 0, 64);
  const uint32_t oend = (uint32_t)__shfl((int)end, min(P - 1 - sw0, 63), 64);
  uint32_t gid = 0, y = 0, y0 = 0, y1 = 0, x0 = 0, x1 = 0, x = 0, xe = 0;
  uint32_t rows = kNoRowPack;  // the preprocess's packed per-row ranges (rec[3].w)
  BandCut cut{};
  // the kept tiles of row y: from the packed ranges, else the cut itself (band_row_range)
  auto row_range = [&](uint32_t yy) {
    if (rows != kNoRowPack) {
      const uint32_t b = (rows >> (8 * (yy - y0))) & 0xffu;
      x = x0 + (b & 15u);
      xe = x + (b >> 4);
    } else {
      band_row_range(cut, yy, x0, x1, x, xe);
    }
  };
  if (off < end) {
    gid = min(order[s], (uint32_t)P - 1u);  // in range unless a sort gave up (reported)
    const uint2 bw = bword ? bword[gid] : make_uint2(0u, kNoRowPack);
    if (bw.y != kNoRowPack) {  // the same x0, y0, y1 and ranges the record path derives
      x0 = bw.x & 0x3fffu;
      y0 = (bw.x >> 14) & 0x3fffu;
      y1 = y0 + (bw.x >> 28);
      rows = bw.y;
    } else {
      const float4 r0 = rec[4 * (size_t)gid];
      const float4 r3 = rec[4 * (size_t)gid + 3];  // {f2, radius, q_cut, rows}
      rows = __float_as_uint(r3.w);
      tile_rect(r0.x, r0.y, (int)r3.y, gx, gy, x0, y0, x1, y1);
      if (rows == kNoRowPack)  // conic.c only for the cut itself
        cut = make_band_cut(r0.x, r0.y, r0.z, r0.w, rec[4 * (size_t)gid + 1].x, r3.z);
    }
    if (egid) ebeg[gid] = off;
    y = y0;
    if (y < y1) row_range(y);
    else off = end;
  }
  for (uint32_t wbeg = obase; wbeg < oend; wbeg += kWin) {
    const uint32_t wend = min(wbeg + (uint32_t)kWin, oend);
    const uint32_t lim = min(end, wend);
    while (off < lim) {
      if (x >= xe) {  // next row of the rectangle (rows may be empty after the cut)
        if (++y >= y1) {
          off = end;
          break;
        }
        row_range(y);
        continue;
      }
      s_key[wid][off - wbeg] = pack ? (((y * gx + x) << pack) | gid) : y * gx + x;
      if (!pack) s_val[wid][off - wbeg] = egid ? off : gid;
      if (egid) s_eg[wid][off - wbeg] = gid;
      x++;
      off++;
    }
    wave_sync();
    for (uint32_t i = (uint32_t)lane; i < wend - wbeg; i += 64) {
      const uint32_t kk = s_key[wid][i];
      tkey[wbeg + i] = kk;
      if (!pack) tval[wbeg + i] = s_val[wid][i];
      if (egid) egid[wbeg + i] = s_eg[wid][i];
      if (hist) {  // the tile's digits (radix_totals_body's, gsr_sort.hip)
        const uint32_t t = pack ? kk >> pack : kk, dm = (1u << tdw) - 1u;
        atomicAdd(&hist[t & dm], 1u);
        if (tpasses > 1) atomicAdd(&hist[256 + ((t >> tdw) & dm)], 1u);
      }
    }
    wave_sync();
  }
}

// Gaussians per duplication workgroup: kDupChunks chunks of kThreads, one after the other (fewer
// workgroups: fewer histogram flushes, each a set of device-scope atomics on shared lines)
constexpr int kDupChunks = 4;
constexpr int kDupPerBlock = kThreads * kDupChunks;
// (body shared by the one-view kernel and the several-views kernel: blk / nblk = this
// workgroup's index and the workgroup count of its view)
__device__ __forceinline__ void duplicate_body(int P, const uint32_t* __restrict__ order,
                                               const uint32_t* __restrict__ offsets,
                                               const float4* __restrict__ rec, uint32_t gx,
                                               uint32_t gy, uint32_t* __restrict__ tkey,
                                               uint32_t* __restrict__ tval, uint32_t R,
                                               SideClear clear0, SideClear clear1,
                                               uint32_t* __restrict__ egid,
                                               uint32_t* __restrict__ ebeg, uint32_t blk,
                                               uint32_t nblk, uint32_t pack,
                                               const uint2* __restrict__ bword,
                                               uint32_t* __restrict__ ttot, int tbits) {
  __shared__ uint32_t s_key[kThreads / 64][kWin];
  __shared__ uint32_t s_val[kThreads / 64][kWin];
  __shared__ uint32_t s_eg[kThreads / 64][kWin];
  __shared__ uint32_t s_hist[2 * 256];
  const size_t tid = (size_t)blk * kThreads + threadIdx.x, nth = (size_t)nblk * kThreads;
  side_clear(clear0.p, clear0.bytes, tid, nth);
  side_clear(clear1.p, clear1.bytes, tid, nth);
  // kernel-argument (grid-uniform) branch; tbits <= 16 (launch_duplicate_views)
  const int tpasses = ttot ? sort_passes(tbits) : 0, tdw = ttot ? sort_digit_bits(tbits) : 0;
  if (ttot) {
    s_hist[threadIdx.x] = 0u;
    s_hist[256 + threadIdx.x] = 0u;
    __syncthreads();
  }
  for (int c = 0; c < kDupChunks; c++)
    duplicate_chunk(P, (int)(blk * kDupPerBlock + c * kThreads), order, offsets, rec, gx, gy, tkey,
                    tval, R, egid, ebeg, pack, bword, s_key, s_val, s_eg, ttot ? s_hist : nullptr,
                    tdw, tpasses);
  if (ttot) {
    __syncthreads();
    // this workgroup's partial copy of the totals (radix_totals_body's shards)
    uint32_t* tot = ttot + (size_t)(blk % (uint32_t)kSortTotShards) * kSortMaxPasses * 256;
    for (int p = 0; p < tpasses; p++) {
      const uint32_t c = s_hist[p * 256 + threadIdx.x];
      if (c) atomicAdd(&tot[p * 256 + threadIdx.x], c);
    }
  }
}

__global__ __launch_bounds__(kThreads) void duplicate_kernel(int P,
                                                             const uint32_t* __restrict__ order,
                                                             const uint32_t* __restrict__ offsets,
                                                             const float4* __restrict__ rec,
                                                             uint32_t gx, uint32_t gy,
                                                             uint32_t* __restrict__ tkey,
                                                             uint32_t* __restrict__ tval,
                                                             uint32_t R, SideClear clear0,
                                                             SideClear clear1,
                                                             uint32_t* __restrict__ egid,
                                                             uint32_t* __restrict__ ebeg,
                                                             const uint2* __restrict__ bword) {
  duplicate_body(P, order, offsets, rec, gx, gy, tkey, tval, R, clear0, clear1, egid, ebeg,
                 blockIdx.x, gridDim.x, 0u, bword, nullptr, 0);
}

// Instances per lane of the ranges kernel: consecutive keys, one 16-B load when aligned (one
// key per lane made the launch ~4x more workgroups than its 4-byte loads can keep busy).
constexpr int kRangesKPT = 4;

__device__ __forceinline__ void tile_ranges_body(size_t R, const uint32_t* __restrict__ tiles,
                                                 uint2* __restrict__ ranges, uint32_t ntiles,
                                                 const uint32_t* __restrict__ derr,
                                                 const uint32_t* __restrict__ terr,
                                                 uint32_t* __restrict__ status,
                                                 uint32_t* host_status, uint32_t* fault,
                                                 uint32_t blk) {
  const size_t base = ((size_t)blk * kThreads + threadIdx.x) * kRangesKPT;
  if (base >= (R ? R : 1)) return;
  // the call's status: both sorts have finished (stream order); a timed-out look-back of either
  // fails this call (render_fwd poisons the outputs, the backward the gradients)
  if (base == 0) {
    const uint32_t st =
        ((derr && *derr) ? kStatusDepthSort : 0u) | ((terr && *terr) ? kStatusTileSort : 0u);
    *status = st;
    if (host_status) *host_status = st;  // pinned mailbox the host checks (gsr_api.cpp)
    if (st && fault) atomicOr(fault, st);  // sticky: the fused Adam step skips while set
  }
  if (R == 0) return;
  // tile ids are < ntiles by construction; the bounds tests only keep the output of a sort whose
  // look-back gave up (reported by the next read-back) from writing outside the table
  uint32_t t[kRangesKPT];
  if (kRangesKPT == 4 && base + 4 <= R && ((uintptr_t)(tiles + base) & 15u) == 0) {
    const uint4 q = *reinterpret_cast<const uint4*>(tiles + base);
    t[0] = q.x;
    t[kRangesKPT > 1 ? 1 : 0] = q.y;
    t[kRangesKPT > 2 ? 2 : 0] = q.z;
    t[kRangesKPT > 3 ? 3 : 0] = q.w;
  } else {
#pragma unroll
    for (int k = 0; k < kRangesKPT; k++) t[k] = base + k < R ? tiles[base + k] : 0u;
  }
  uint32_t prev = base ? tiles[base - 1] : 0u;
#pragma unroll
  for (int k = 0; k < kRangesKPT; k++) {
    const size_t idx = base + k;
    if (idx >= R) break;
    const uint32_t cur = t[k];
    const bool cur_ok = cur < ntiles;
    if (idx == 0) {
      if (cur_ok) ranges[cur].x = 0;
    } else if (cur != prev) {
      if (prev < ntiles) ranges[prev].y = (uint32_t)idx;
      if (cur_ok) ranges[cur].x = (uint32_t)idx;
    }
    if (idx == R - 1 && cur_ok) ranges[cur].y = (uint32_t)R;
    prev = cur;
  }
}

__global__ __launch_bounds__(kThreads) void tile_ranges_kernel(size_t R,
                                                               const uint32_t* __restrict__ tiles,
                                                               uint2* __restrict__ ranges,
                                                               uint32_t ntiles,
                                                               const uint32_t* __restrict__ derr,
                                                               const uint32_t* __restrict__ terr,
                                                               uint32_t* __restrict__ status,
                                                               uint32_t* host_status,
                                                               uint32_t* fault) {
  tile_ranges_body(R, tiles, ranges, ntiles, derr, terr, status, host_status, fault, blockIdx.x);
}

// ---- several views per launch (the multi-view forward's batched binning, gsr_api.cpp) ----------
struct DupViews {
  DupSpec j[kMaxBatchViews];
  uint32_t first[kMaxBatchViews + 1];
  int V;
};
struct RangesViews {
  RangesSpec j[kMaxBatchViews];
  uint32_t first[kMaxBatchViews + 1];
  int V;
};

__device__ __forceinline__ int batch_view(const uint32_t* first, int V, uint32_t b) {
  int k = 0;
  while (k + 1 < V && b >= first[k + 1]) k++;
  return k;
}

__global__ __launch_bounds__(kThreads) void duplicate_views_kernel(DupViews m) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const DupSpec& j = m.j[k];
  if (j.tag && blockIdx.x == m.first[k] && threadIdx.x == 0) *j.tag = j.tag_val;
  duplicate_body(j.P, j.order, j.offsets, j.rec, j.gx, j.gy, j.tkey, j.tval, j.R, j.clear0,
                 j.clear1, j.egid, j.ebeg, blockIdx.x - m.first[k], m.first[k + 1] - m.first[k],
                 j.pack, j.bword, j.ttot, j.tbits);
}

__global__ __launch_bounds__(kThreads) void tile_ranges_views_kernel(RangesViews m) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const RangesSpec& j = m.j[k];
  tile_ranges_body(j.R, j.tiles, j.ranges, j.ntiles, j.depth_err, j.tile_err, j.status,
                   j.host_status, j.fault, blockIdx.x - m.first[k]);
}

__global__ __launch_bounds__(kThreads) void det_gather_kernel(size_t R,
                                                              const uint32_t* __restrict__ einst,
                                                              const uint32_t* __restrict__ egid,
                                                              uint32_t* __restrict__ point_list) {
  const size_t q = (size_t)blockIdx.x * kThreads + threadIdx.x;
  if (q < R) point_list[q] = egid[min(einst[q], (uint32_t)(R - 1))];
}

}  // namespace

hipError_t launch_det_gather(size_t R, const uint32_t* einst, const uint32_t* egid,
                             uint32_t* point_list, hipStream_t s) {
  if (R == 0) return hipSuccess;
  hipLaunchKernelGGL(det_gather_kernel, dim3((unsigned)((R + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, R, einst, egid, point_list);
  return hipGetLastError();
}

hipError_t launch_duplicate(int P, const uint32_t* order, const uint32_t* offsets,
                            const int32_t* radii, const float4* rec, uint32_t gx, uint32_t gy,
                            uint32_t* tkey, uint32_t* tval, uint32_t R, SideClear clear0,
                            SideClear clear1, hipStream_t s, uint32_t* egid, uint32_t* ebeg,
                            const uint2* bword) {
  if (P == 0) return hipSuccess;
  hipLaunchKernelGGL(duplicate_kernel, dim3((P + kDupPerBlock - 1) / kDupPerBlock), dim3(kThreads), 0, s,
                     P, order, offsets, rec, gx, gy, tkey, tval, R, clear0, clear1, egid, ebeg,
                     bword);
  return hipGetLastError();
}

hipError_t launch_duplicate_views(const DupSpec* v, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  DupViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    const DupSpec& d = v[k];
    if (d.pack && (d.egid || d.pack >= 32u || (uint64_t)d.P > (1ull << d.pack) ||
                   (uint64_t)d.gx * d.gy > (1ull << (32u - d.pack))))
      return hipErrorInvalidValue;  // tile << pack | gid must fit 32 bits
    if (d.ttot && (d.tbits <= 0 || d.tbits > 16 || (uint64_t)d.gx * d.gy > (1ull << d.tbits)))
      return hipErrorInvalidValue;  // two digit passes at most (the LDS histogram's)
    m.j[k] = v[k];
    m.first[k + 1] = m.first[k] + (uint32_t)((v[k].P + kDupPerBlock - 1) / kDupPerBlock);
  }
  if (m.first[V] == 0) return hipSuccess;
  hipLaunchKernelGGL(duplicate_views_kernel, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t launch_tile_ranges_views(const RangesSpec* v, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  RangesViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    m.j[k] = v[k];
    if (!v[k].R) m.j[k].tile_err = nullptr;  // no instances: nothing tile-sorted
    const size_t n = v[k].R ? v[k].R : 1;  // R == 0: one lane still publishes the status
    const size_t per = (size_t)kThreads * kRangesKPT;
    m.first[k + 1] = m.first[k] + (uint32_t)((n + per - 1) / per);
  }
  hipLaunchKernelGGL(tile_ranges_views_kernel, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t launch_tile_ranges(size_t R, const uint32_t* sorted_tiles, uint2* ranges,
                              uint32_t ntiles, const uint32_t* depth_err, const uint32_t* tile_err,
                              uint32_t* status, uint32_t* host_status, uint32_t* fault,
                              hipStream_t s, bool ranges_cleared) {
  if (!ranges_cleared) {
    hipError_t e = hipMemsetAsync(ranges, 0, sizeof(uint2) * ntiles, s);
    if (e != hipSuccess) return e;
  }
  // R == 0: no instances, nothing tile-sorted; one lane still publishes the depth sort's word
  const size_t n = R ? R : 1;
  const size_t per = (size_t)kThreads * kRangesKPT;
  hipLaunchKernelGGL(tile_ranges_kernel, dim3((unsigned)((n + per - 1) / per)),
                     dim3(kThreads), 0, s, R, sorted_tiles, ranges, ntiles, depth_err,
                     R ? tile_err : nullptr, status, host_status, fault);
  return hipGetLastError();
}

}  // namespace gsr

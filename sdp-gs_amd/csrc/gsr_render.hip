// gsr_render.hip -- per-tile alpha blending, forward and backward, for gfx950.
//
// Reference behaviour: renderCUDA forward (cuda_rasterizer/forward.cu:261-374) and backward
// (cuda_rasterizer/backward.cu:399-557), extended with depth / alpha / 3-channel feature outputs
// (SURVEY.md row A12).
//
// gfx950 design:
//  * one 256-lane workgroup (4 waves of 64) per 16x16 tile; wave w owns the 8x8 quadrant
//    (w & 1, w >> 1) -- squares hug splat footprints better than 4x16 strips (-10% blend time);
//  * tile schedule: workgroups take tiles heaviest first (tile_schedule_kernel, LPT order), so
//    the centre-heavy tiles start early instead of forming the tail (GSR_TILE_ORDER=natural|xcd
//    select the natural order or contiguous per-XCD bands, both measured slower);
//  * per-wave culling: each wave compacts the batch to the splats that can reach alpha >= 1/255
//    in its 8x8 quadrant (same conservative test as the binning);
//  * batches of 256 splat records (64 B each, packed by the preprocess) staged in LDS and read
//    by all lanes as broadcasts;
//  * backward: the tile is replayed back to front starting at the tile's largest n_contrib (no
//    lane can use anything behind it), per-splat gradients are summed over the wave with a
//    halving butterfly (16 values -> 17 shuffles instead of 96), accumulated per batch in LDS with
//    ds_add_f32, and flushed once per (splat, tile) as 64-byte rows of global float atomics
//    (MI355X_MICROARCH.md: 4 x 64-B row segments per wave instruction) instead of the
//    reference's 9 atomics per contributing (splat, pixel) pair.
#include "gsr_device.h"
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = kTilePix;  // 256
constexpr int kAccPad = kAccFloats + 1;  // LDS accumulator row stride (odd: conflict-free columns)

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles) {
  const uint32_t q = ntiles >> 3, r = ntiles & 7u;
  const uint32_t xcd = b & 7u, local = b >> 3;
  const uint32_t start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + local;
}

// Tile schedule: 0 = natural order (round-robin over XCDs by the dispatcher), 1 = contiguous
// band per XCD (L2 locality), 2 = heaviest tiles first (order[] computed on device by
// tile_schedule_kernel; a schedule only, results do not depend on it).
__device__ __forceinline__ uint32_t sched_tile(uint32_t b, uint32_t ntiles, int mode,
                                               const uint32_t* order) {
  if (mode == 2 && order) return order[b];
  if (mode == 1) return xcd_tile(b, ntiles);
  return b;
}

// One workgroup: bucket the tiles by log2 of their work (list length) and write them heaviest
// bucket first.  Order inside a bucket is whatever the LDS atomics produce -- only a schedule.
constexpr int kSchedThreads = 1024;
__device__ __forceinline__ void tile_schedule_body(const uint2* __restrict__ ranges,
                                                   const uint32_t* __restrict__ work,
                                                   uint32_t ntiles, uint32_t* __restrict__ order) {
  __shared__ uint32_t cnt[33];
  __shared__ uint32_t off[33];
  if (threadIdx.x < 33) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ntiles; t += kSchedThreads) {
    const uint32_t w = work ? work[t] : ranges[t].y - ranges[t].x;
    const uint32_t bkt = 32u - (uint32_t)__clz((int)w);  // 0 for empty, 32 for >= 2^31
    atomicAdd(&cnt[32 - bkt], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int i = 0; i < 33; i++) { off[i] = s; s += cnt[i]; }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ntiles; t += kSchedThreads) {
    const uint32_t w = work ? work[t] : ranges[t].y - ranges[t].x;
    const uint32_t bkt = 32u - (uint32_t)__clz((int)w);
    order[atomicAdd(&off[32 - bkt], 1u)] = t;
  }
}

__global__ __launch_bounds__(kSchedThreads) void tile_schedule_kernel(const uint2* __restrict__ ranges,
                                                                      const uint32_t* __restrict__ work,
                                                                      uint32_t ntiles,
                                                                      uint32_t* __restrict__ order) {
  tile_schedule_body(ranges, work, ntiles, order);
}

struct SchedViews {
  const uint2* ranges[kMaxBatchViews];
  uint32_t* order[kMaxBatchViews];
  uint32_t ntiles[kMaxBatchViews];
};
__global__ __launch_bounds__(kSchedThreads) void tile_schedule_views_kernel(SchedViews m) {
  const int k = (int)blockIdx.x;  // one workgroup per view
  tile_schedule_body(m.ranges[k], nullptr, m.ntiles[k], m.order[k]);
}

// Lane -> pixel map.  GSR_QUAD_WAVES: wave w owns the 8x8 quadrant (w & 1, w >> 1) of the tile
// (lane l -> (l & 7, l >> 3)); otherwise wave w owns pixel rows 4w..4w+3 (lane l -> (l & 15,
// l >> 4)).  Squares hug the (mostly round) splat footprints better than 4x16 strips.
#ifndef GSR_QUAD_WAVES
#define GSR_QUAD_WAVES 1
#endif
// diagnostic builds (wrong gradients, timing only): 1 = no wave reduction of the pair terms,
// 2 = the flush's global atomics as plain stores, 3 = no pair update / reduction at all
#ifndef GSR_BWD_DIAG
#define GSR_BWD_DIAG 0
#endif
// backward Gaussian weight: 1 = hardware exp2 with an exact splat_exp at the alpha >= 1/255
// threshold (see render_bwd_kernel), 0 = splat_exp everywhere (the forward's sequence)
#ifndef GSR_BWD_FAST_EXP
#define GSR_BWD_FAST_EXP 1
#endif
// backward group replay: 1 = every entry of a group is replayed straight-line (no wave-uniform
// skip of entries without a contributing lane), 0 = such entries are skipped.  Round 3, after the
// hoisted loads: 0.2115 -> 0.235 ms with 1 (profiles/r03_bwd_flush_noskip_ab.txt), not kept
#ifndef GSR_BWD_NOSKIP
#define GSR_BWD_NOSKIP 0
#endif
// backward batch order: 1 = the next batch is staged before this batch's flush (its loads not
// queued behind the flush's atomics), 0 = after it.  Measured 0.2115 -> 0.2185 ms with 1 (the
// workgroup then waits for the staged loads before it can flush), not kept
#ifndef GSR_BWD_FLUSH_LATE
#define GSR_BWD_FLUSH_LATE 0
#endif
// backward colour dot product: 1 = formed in the group's test phase for every entry (the colour
// registers die early), 0 = where the compiler places it
#ifndef GSR_BWD_CDOT_EARLY
#define GSR_BWD_CDOT_EARLY 1
#endif
// backward LDS accumulator rows: 1 = 13 floats (the gradient values; the flush supplies the row's
// three zero slots), 0 = 17 (16 + 1 pad).  13 is odd as well, so the column accesses stay
// conflict-free, and the workgroup's LDS drops 34.3 -> 30.2 KB (5 workgroups per CU instead of 4)
#ifndef GSR_BWD_ACC13
#define GSR_BWD_ACC13 1
#endif
// backward minimum waves per SIMD requested from the register allocator (amdgpu_waves_per_eu; the
// default-mode kernels).  5 with the 13-float rows and the colour dot product in the test phase:
// 96 VGPRs, 12 spilled (all outside the entry loop), 5 workgroups per CU -- render_bwd 1.012 /
// 1.011 -> 0.998 / 0.995 ms per 6-view launch (profiles/r04_bwd_occ_ab.txt); 5 without the early
// dot product spills 23 and is slower (1.017 / 1.020)
#ifndef GSR_BWD_MIN_WAVES
#define GSR_BWD_MIN_WAVES 5
#endif
// backward transmittance recovery T / (1 - alpha): 0 = IEEE division, 1 = rcp + Newton step
#ifndef GSR_BWD_FAST_DIV
#define GSR_BWD_FAST_DIV 1
#endif
// instrumentation build (-DGSR_BLEND_STATS=1): per-wave work counters of both blends, read with
// gsr_test_blend_stats (scripts/blend_stats.py); off in the product build
#ifndef GSR_BLEND_STATS
#define GSR_BLEND_STATS 0
#endif
#if GSR_BLEND_STATS
// [0] fwd list entries, [1] fwd entries evaluated, [2] fwd entries with a contributing lane,
// [3] fwd contributing (lane, entry) pairs, [4] bwd list entries, [5] bwd groups evaluated,
// [6] bwd entries with a contributing lane, [7] bwd contributing pairs, [8] waves
__device__ unsigned long long g_blend_stats[16];
#define BLEND_STAT(k, v) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_blend_stats[k], (unsigned long long)(v)); } while (0)
#else
#define BLEND_STAT(k, v) do { } while (0)
#endif
// block-list forward: 1 = the group's four alpha tests run ahead of the replay as four
// interleaved exp chains (splat_exp_n), 0 = where the compiler puts them (inside the replay's
// per-lane branches).  Round 3: render_fwd 0.1140 vs 0.1141 ms (3 alternating pairs at 1 stream,
// profiles/r03_fwd_testfirst_ab.txt) -- the forward is not latency-bound on these chains; off
#ifndef GSR_FWD_TEST_FIRST
#define GSR_FWD_TEST_FIRST 0
#endif
// forward: 1 = blend weight alpha * T formed once per pair, 0 = col * alpha * T per channel
#ifndef GSR_FWD_WEIGHT
#define GSR_FWD_WEIGHT 1
#endif
__device__ __forceinline__ void pixel_of(uint32_t tx, uint32_t ty, uint32_t t, uint32_t& px,
                                         uint32_t& py) {
  const uint32_t w = t >> 6, l = t & 63u;
  if (GSR_QUAD_WAVES) {
    px = tx * kTile + (w & 1u) * 8u + (l & 7u);
    py = ty * kTile + (w >> 1) * 8u + (l >> 3);
  } else {
    px = tx * kTile + (t & (kTile - 1));
    py = ty * kTile + (t >> 4);
  }
}

// Which of the 4 waves a splat can reach: bit w set unless the conservative test of
// gsr_device.h proves alpha < 1/255 on all 64 pixels of wave w.
__device__ __forceinline__ uint32_t wave_mask(float4 r0, float4 r1, float qc, uint32_t tx,
                                              uint32_t ty) {
  // qc: the record's q_cut (rec[3].z, computed once by the preprocess)
  if (qc == -1.0f) return 0xfu;
  if (qc == -2.0f) return 0u;
  const SplatCut cut = make_cut(r0.x, r0.y, r0.z, r0.w, r1.x, qc);
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    float x0, x1, y0, y1;
    if (GSR_QUAD_WAVES) {
      x0 = (float)(tx * kTile + (w & 1) * 8); x1 = x0 + 7.0f;
      y0 = (float)(ty * kTile + (w >> 1) * 8); y1 = y0 + 7.0f;
    } else {
      x0 = (float)(tx * kTile); x1 = (float)(tx * kTile + kTile - 1);
      y0 = (float)(ty * kTile + 4 * w); y1 = y0 + 3.0f;
    }
    m |= cut_touches_rect(cut, x0, x1, y0, y1) ? (1u << w) : 0u;
  }
  return m;
}

// Per-wave compaction of the batch: the wave's list holds, in batch order, the entries whose
// mask has this wave's bit.  Returns the list length (wave-uniform).
__device__ __forceinline__ uint32_t build_wave_list(const uint8_t* s_mask, uint8_t* list,
                                                    uint32_t cnt, int wid, int lane) {
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t n = 0;
#pragma unroll
  for (int c = 0; c < kThreads / 64; c++) {
    const uint32_t j = (uint32_t)(c * 64 + lane);
    const bool bit = j < cnt && ((s_mask[j] >> wid) & 1u);
    const uint64_t b = __ballot(bit);
    if (bit) list[n + (uint32_t)__popcll(b & lt)] = (uint8_t)j;
    n += (uint32_t)__popcll(b);
  }
  return n;
}

template <bool FEAT>
__global__ __launch_bounds__(kThreads) void render_fwd_kernel(RenderArgs a) {
  __shared__ float4 s_r0[kThreads];
  __shared__ float4 s_r1[kThreads];
  __shared__ float4 s_r2[kThreads];
  __shared__ float s_f2[FEAT ? kThreads : 1];  // rec[3].x (feature 2) only
  __shared__ uint8_t s_mask[kThreads];
  __shared__ uint8_t s_list[kThreads / 64][kThreads];
  __shared__ uint32_t s_max;
  side_clear(a.clear.p, a.clear.bytes, (size_t)blockIdx.x * kThreads + threadIdx.x,
             (size_t)gridDim.x * kThreads);
  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);

  const uint32_t ntiles = a.gx * a.gy;
  const uint32_t tile = sched_tile(blockIdx.x, ntiles, a.sched, a.order);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  uint32_t px, py;
  pixel_of(tx, ty, threadIdx.x, px, py);
  const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
  const float pfx = (float)px, pfy = (float)py;
  bool done = !inside;
  if (threadIdx.x == 0) s_max = 0;

  // a sort of this call gave up (look-back timeout): the lists are not the reference's, so the
  // call's outputs are NaN and its backward fails (gsr_api.cpp) instead of training on them
  if (*a.status & (kStatusDepthSort | kStatusTileSort)) {
    if (threadIdx.x == 0) a.tile_last[tile] = 0;
    if (inside) {
      const size_t pix = (size_t)py * a.W + px, HW = (size_t)a.W * a.H;
      const float nan = __builtin_nanf("");
      a.final_T[pix] = nan;
      a.n_contrib[pix] = 0;
      for (int c = 0; c < 3; c++) a.out_color[c * HW + pix] = nan;
      if (a.out_depth) a.out_depth[pix] = nan;
      if (a.out_alpha) a.out_alpha[pix] = nan;
      if (a.out_feature)
        for (int c = 0; c < 3; c++) a.out_feature[c * HW + pix] = nan;
    }
    return;
  }

  const uint2 range = a.ranges[tile];
  float T = 1.0f;
  uint32_t last_contributor = 0;
  constexpr int NC = FEAT ? 8 : 5;
  float C[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) C[c] = 0.0f;

  for (uint32_t base = range.x; base < range.y; base += kThreads) {
    // forward.cu:309-311: stop when every pixel of the tile is saturated
    if (__syncthreads_count(done) == kThreads) break;
    const uint32_t i = base + threadIdx.x;
    if (i < range.y) {
      const uint32_t pid = a.point_list[i];
      if (pid >= a.P) {  // memory-safe clamp, reported to this call's status check
        atomicOr(a.status, kStatusClamp);
        if (a.host_status) *a.host_status = kStatusClamp;  // sort bits are 0 on this path
        if (a.fault) atomicOr(a.fault, kStatusClamp);
      }
      const uint32_t gid = min(pid, a.P - 1u);
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1], q3 = rec[3];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = q1;
      s_r2[threadIdx.x] = rec[2];
      if (FEAT) s_f2[threadIdx.x] = q3.x;
      s_mask[threadIdx.x] = (uint8_t)wave_mask(q0, q1, q3.z, tx, ty);
    }
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, range.y - base);
    const uint32_t nlist = build_wave_list(s_mask, s_list[wid], cnt, wid, lane);
    BLEND_STAT(0, nlist);
    const uint32_t rel0 = base - range.x;
    // Four list entries per iteration: their (independent) Gaussian weights are evaluated
    // together, then composited in list order exactly as the reference's per-splat loop
    // (forward.cu:325-362) -- same operations, same order, per pixel.
    for (uint32_t k = 0; k < nlist; k += 4) {
      if (__ballot(!done) == 0ull) break;  // wave-uniform
      BLEND_STAT(1, min(4u, nlist - k));
      const uint32_t packed = *reinterpret_cast<const uint32_t*>(&s_list[wid][k]);
      uint32_t jj[4];
      float pw[4], al[4];
      float4 r1v[4], r2v[4];
      float f2v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        jj[u] = (packed >> (8 * u)) & 0xffu;
        const float4 r0 = s_r0[jj[u]];
        r1v[u] = s_r1[jj[u]];
        r2v[u] = s_r2[jj[u]];
        f2v[u] = FEAT ? s_f2[jj[u]] : 0.0f;
        const float dx = r0.x - pfx, dy = r0.y - pfy;
        const float power = -0.5f * (r0.z * dx * dx + r1v[u].x * dy * dy) - r0.w * dx * dy;
        // entries past the list end get power = +1 and are skipped like any power > 0 pair
        pw[u] = (k + u < nlist) ? power : 1.0f;
        al[u] = fminf(0.99f, r1v[u].y * splat_exp(pw[u]));
      }
#if GSR_BLEND_STATS
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint64_t cb = __ballot(!done && !(pw[u] > 0.0f) && !(al[u] < 1.0f / 255.0f));
        if (cb) { BLEND_STAT(2, 1); BLEND_STAT(3, __popcll(cb)); }
      }
#endif
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (done) continue;
        if (pw[u] > 0.0f) continue;
        const float alpha = al[u];
        if (alpha < 1.0f / 255.0f) continue;
        const float test_T = T * (1 - alpha);
        if (test_T < 0.0001f) {
          done = true;
          continue;
        }
#if GSR_FWD_WEIGHT
        // blend weight alpha * T formed once (the reference forms col * alpha * T per channel,
        // forward.cu:341-343: same value up to the rounding of one product)
        const float wgt = alpha * T;
        C[0] += r1v[u].w * wgt;
        C[1] += r2v[u].x * wgt;
        C[2] += r2v[u].y * wgt;
        C[3] += r1v[u].z * wgt;
        C[4] += wgt;
        if (FEAT) {
          C[5 % NC] += r2v[u].z * wgt;
          C[6 % NC] += r2v[u].w * wgt;
          C[7 % NC] += f2v[u] * wgt;
        }
#else
        C[0] += r1v[u].w * alpha * T;
        C[1] += r2v[u].x * alpha * T;
        C[2] += r2v[u].y * alpha * T;
        C[3] += r1v[u].z * alpha * T;
        C[4] += alpha * T;
        if (FEAT) {
          C[5 % NC] += r2v[u].z * alpha * T;
          C[6 % NC] += r2v[u].w * alpha * T;
          C[7 % NC] += f2v[u] * alpha * T;
        }
#endif
        T = test_T;
        // the reference counts every list position (forward.cu:328); skipped entries cannot blend
        last_contributor = rel0 + jj[u] + 1;
      }
    }
  }

  // tile-wide max of n_contrib: the backward starts its replay there
  uint32_t m = last_contributor;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) atomicMax(&s_max, m);
  __syncthreads();
  if (threadIdx.x == 0) a.tile_last[tile] = s_max;

  if (inside) {
    const size_t pix = (size_t)py * a.W + px;
    const size_t HW = (size_t)a.W * a.H;
    a.final_T[pix] = T;
    a.n_contrib[pix] = last_contributor;
    a.out_color[pix] = C[0] + T * a.bg[0];
    a.out_color[HW + pix] = C[1] + T * a.bg[1];
    a.out_color[2 * HW + pix] = C[2] + T * a.bg[2];
    if (a.out_depth) a.out_depth[pix] = C[3];
    if (a.out_alpha) a.out_alpha[pix] = C[4];
    if (a.out_feature) {
      a.out_feature[pix] = FEAT ? C[FEAT ? 5 : 0] : 0.0f;
      a.out_feature[HW + pix] = FEAT ? C[FEAT ? 6 : 0] : 0.0f;
      a.out_feature[2 * HW + pix] = FEAT ? C[FEAT ? 7 : 0] : 0.0f;
    }
  }
}

// Two floats in one 64-bit register pair: gfx950's packed FP32 VALU (v_pk_mul_f32, v_pk_add_f32,
// v_pk_fma_f32) does both halves in one issue slot.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 mk2(float x, float y) { return f2{x, y}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// DPP move with bound_ctrl and full masks (every source lane of the patterns used here exists), in
// the form the backend folds into the consuming v_add_f32 as a DPP operand
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, true));
}

// Orientation of gfx950's v_permlane32_swap / v_permlane16_swap (which half of the pair keeps
// the first operand), probed once per kernel so the value->lane map below does not rest on an
// assumption about the ISA description.
struct SwapOrient {
  uint32_t flip32, flip16;  // 1 if the low half ends up holding the second operand's pair
};
__device__ __forceinline__ SwapOrient probe_swaps(int lane) {
  const uint32_t a = (uint32_t)lane, b = (uint32_t)lane + 64u;
  const auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  const auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  SwapOrient o;
  o.flip32 = (__builtin_amdgcn_readfirstlane(r32[0]) == 0u) ? 0u : 1u;
  o.flip16 = (__builtin_amdgcn_readfirstlane(r16[0]) == 0u) ? 0u : 1u;
  return o;
}

__device__ __forceinline__ f2 swap32_add(f2 p, f2 q) {
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(p.x), __float_as_uint(q.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(p.y), __float_as_uint(q.y), false, false);
  return mk2(__uint_as_float(rx[0]), __uint_as_float(ry[0])) +
         mk2(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
}
__device__ __forceinline__ f2 swap16_add(f2 p, f2 q) {
  const auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(p.x), __float_as_uint(q.x), false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(p.y), __float_as_uint(q.y), false, false);
  return mk2(__uint_as_float(rx[0]), __uint_as_float(ry[0])) +
         mk2(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
}

// Halving butterfly on VALU only: on entry every lane holds 16 partial values as 8 pairs
// (v[i] = values 2i, 2i+1); on exit every lane holds the full wave sum of ONE value, index
// k = 8*b5' + 4*b4' + 2*b3 + b2 (b = lane bits, b5'/b4' corrected by the probed swap
// orientation), 4 lanes per value.  Steps: permlane32_swap (pairs lane l with l^32: values k and
// k+8, 4 packed adds), permlane16_swap (l^16: k and k+4, 2 packed adds), DPP row_mirror (l^15
// within a row: k and k+2, one packed add), DPP row_half_mirror (l^7), quad_perm xor 2, xor 1.
// The partner maps {^15, ^7, ^2, ^1} are linearly independent over the low 4 lane bits, so every
// lane of the 16-lane row is summed exactly once; no LDS traffic.
__device__ __forceinline__ float wave_reduce16_dpp(f2 (&v)[8], int lane) {
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = swap32_add(v[i], v[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; i++) v[i] = swap16_add(v[i], v[i + 2]);
  f2 w;
  {
    const bool hi = lane & 8;
    const f2 send = hi ? v[0] : v[1];
    const f2 keep = hi ? v[1] : v[0];
    w = keep + mk2(dpp<0x140>(send.x), dpp<0x140>(send.y));  // row_mirror
  }
  float x;
  {
    const bool hi = lane & 4;
    const float send = hi ? w.x : w.y;
    const float keep = hi ? w.y : w.x;
    x = keep + dpp<0x141>(send);  // row_half_mirror
  }
  x += dpp<0x4E>(x);  // quad_perm [2,3,0,1]
  x += dpp<0xB1>(x);  // quad_perm [1,0,3,2]
  return x;
}

__device__ __forceinline__ int reduce16_slot(int lane, SwapOrient o) {
  const int b5 = ((lane >> 5) & 1) ^ (int)o.flip32;
  const int b4 = ((lane >> 4) & 1) ^ (int)o.flip16;
  return b5 * 8 + b4 * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
}

// Joint halving butterfly of FOUR entries' 16 values (GSR_BWD_PIPE=2): 64 values per lane, one
// fully reduced value per lane on exit -- entry e = 2 b5' + b4' (the probed swap orientation, as
// reduce16_slot), slot k = lane & 15.  permlane32_swap pairs entries (0, 2) and (1, 3),
// permlane16_swap then (0|2, 1|3); the rest is the 16-lane row's four halving DPP stages (l^15,
// l^7, l^2, l^1: linearly independent over the low lane bits, so every lane of the row is summed
// once).  Same instruction count per entry as wave_reduce16_dpp, four times the independent work
// per stage, and one LDS add per lane for the four entries.
__device__ __forceinline__ float wave_reduce_joint4(f2 (&v)[4][8], int lane) {
  f2 r0[8], r1[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r0[i] = swap32_add(v[0][i], v[2][i]);
    r1[i] = swap32_add(v[1][i], v[3][i]);
  }
  f2 s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = swap16_add(r0[i], r1[i]);
  f2 w[4];
  {
    const bool hi = lane & 8;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const f2 send = hi ? s[i] : s[i + 4];
      const f2 keep = hi ? s[i + 4] : s[i];
      w[i] = keep + mk2(dpp<0x140>(send.x), dpp<0x140>(send.y));  // row_mirror
    }
  }
  f2 x[2];
  {
    const bool hi = lane & 4;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const f2 send = hi ? w[i] : w[i + 2];
      const f2 keep = hi ? w[i + 2] : w[i];
      x[i] = keep + mk2(dpp<0x141>(send.x), dpp<0x141>(send.y));  // row_half_mirror
    }
  }
  f2 y;
  {
    const bool hi = lane & 2;
    const f2 send = hi ? x[0] : x[1];
    const f2 keep = hi ? x[1] : x[0];
    y = keep + mk2(dpp<0x4E>(send.x), dpp<0x4E>(send.y));  // quad_perm [2,3,0,1]
  }
  const bool hi = lane & 1;
  const float send = hi ? y.x : y.y;
  const float keep = hi ? y.y : y.x;
  return keep + dpp<0xB1>(send);  // quad_perm [1,0,3,2]
}

__device__ __forceinline__ int joint4_entry(int lane, SwapOrient o) {
  return (((lane >> 5) & 1) ^ (int)o.flip32) * 2 + (((lane >> 4) & 1) ^ (int)o.flip16);
}

// Deterministic variant (DET, gsr.h debug bit 1): no float atomics.  Every wave stores its
// butterfly sums into its OWN accumulator rows (each batch entry is in a wave's list at most
// once), the four waves' rows are added in wave order, and each (splat, tile) row is stored to
// partial[emission index of the instance]; det_reduce_kernel then sums every Gaussian's rows in
// emission order.  13-float rows (the gradient values; slots 13-15 are always zero), 2
// workgroups per CU.
constexpr int kAccDet = 13;

// ROWS (rows layout, gsr_internal.h bwd_rows_mode): the flush STORES every (splat, tile) row to
// partial[emission index] -- one coalesced 64-B row per instance, no global float atomics (they
// execute at the memory side at ~1.3 TB/s chip-wide, MI355X_MICROARCH.md "Global float atomics")
// -- and the backward preprocess sums each Gaussian's rows.  DET implies ROWS.
// One tile of the backward blend: workgroup `blk` of the view described by `a` (render_bwd_kernel:
// one view per launch; render_bwd_views_kernel: the tiles of several views in one launch).
// 4 waves per SIMD (128 VGPRs): the pipelined variants hold pending entries
#define GSR_BWD_WAVES(PIPE, DET) \
  __attribute__((amdgpu_waves_per_eu((PIPE) ? 4 : ((DET) ? 1 : GSR_BWD_MIN_WAVES))))
// PIPE (GSR_BWD_PIPE, round 4): the wave reduction of a contributing entry is issued together
// with the next contributing entry's recurrence, in one basic block -- the two are independent
// (the reduction needs only the entry's u = G dL/dalpha, w = alpha T and (dx, dy)), so the
// butterfly's six dependent permlane / DPP stages overlap the recurrence's T-recovery chain
// instead of serialising behind it.  The last entry of a batch is reduced before the batch's
// barrier.  Same values, same LDS adds: results equal to the unpipelined kernel up to the order
// of the LDS float adds (as between waves already).
// PIPE == 2 (GSR_BWD_PIPE=2, round 4): the group's contributing entries keep their (u, w, d) and
// the group ends in ONE joint reduction of its four entries (wave_reduce_joint4; entries without
// a contributing lane are zeros) -- the butterfly's dependent stages carry four entries' work.
template <bool EXTRA, bool FEAT, int GROUP, bool DET, bool ROWS, int PIPE>
__device__ __forceinline__ void render_bwd_tile(const RenderBwdArgs& a, uint32_t blk) {
  static_assert(!DET || ROWS, "the deterministic backward stores per-instance rows");
  static_assert(!(PIPE && DET), "the pipelined reduction is a default-mode kernel");
  static_assert(PIPE != 2 || GROUP == 4, "the joint reduction takes a group of four entries");
  // the batch's records in LDS, regrouped so that the colour dot product's packed FMAs read
  // register pairs straight from the loads: s_r0 = {x, y, conic.a, conic.b}, s_r1 = {conic.c,
  // opacity}, s_c0 = {r, g, b, depth}, s_c1 = {f0, f1, f2, 1} (alpha channel)
  __shared__ float4 s_r0[kThreads];
  __shared__ float2 s_r1[kThreads];
  __shared__ float4 s_c0[kThreads];
  __shared__ float4 s_c1[FEAT ? kThreads : 1];
  // double-buffered under GSR_BWD_FLUSH_LATE: the flush of batch k reads its ids after batch k + 1
  // has been staged
  __shared__ uint32_t s_gid[GSR_BWD_FLUSH_LATE ? 2 : 1][kThreads];
  // accumulator rows of an odd stride (13 floats, the gradient values; 17 without
  // GSR_BWD_ACC13): the per-splat moments pass (lane t -> row t) and the zero-fill are
  // bank-conflict-free; the butterfly's adds (one row's slots) and the flush (4 rows x 16 slots
  // per wave, slots >= 13 supplied as zeros) stay conflict-free as well
  constexpr int kRow = (DET || GSR_BWD_ACC13) ? kAccDet : kAccPad;
  __shared__ float s_acc[(DET ? 4 : 1) * kThreads * kRow];
  __shared__ uint8_t s_mask[kThreads];
  __shared__ uint8_t s_list[kThreads / 64][kThreads];

  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);
  const SwapOrient swap_orient = probe_swaps(lane);
  // the lanes that hold a reduced gradient value (one of the four per value, value < kAccDet)
  const int red_slot = reduce16_slot(lane, swap_orient);
  const bool red_lane = (lane & 3) == 0 && red_slot < kAccDet;
  const int j4_shift = 8 * joint4_entry(lane, swap_orient);  // PIPE == 2: this lane's entry's byte
  const uint32_t ntiles = a.gx * a.gy;
  const uint32_t tile = sched_tile(blk, ntiles, a.sched, a.order);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  uint32_t px, py;
  pixel_of(tx, ty, threadIdx.x, px, py);
  const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
  const float pfx = (float)px, pfy = (float)py;
  const size_t pix = (size_t)py * a.W + px;
  const size_t HW = (size_t)a.W * a.H;

  // a failed forward (a sort gave up): its lists are not valid and the backward preprocess
  // NaN-poisons every gradient; nothing is read from them here (grid-uniform)
  if (ROWS && a.status && (*a.status & (kStatusDepthSort | kStatusTileSort))) return;
  const uint2 range = a.ranges[tile];
  const uint32_t tile_last = a.tile_last[tile];
  BLEND_STAT(8, 1);
  const float T_final = inside ? a.final_T[pix] : 0.0f;
  float T = T_final;
  const uint32_t last_contributor = inside ? a.n_contrib[pix] : 0u;
  uint32_t wave_last = last_contributor;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) wave_last = max(wave_last, (uint32_t)__shfl_xor((int)wave_last, d, 64));

  constexpr int NC = FEAT ? 8 : (EXTRA ? 5 : 3);
  float dpix[NC];
  if (inside) {
    dpix[0] = a.dL_dcolor[pix];
    dpix[1] = a.dL_dcolor[HW + pix];
    dpix[2] = a.dL_dcolor[2 * HW + pix];
    if (NC > 3) {
      dpix[3 % NC] = a.dL_ddepth ? a.dL_ddepth[pix] : 0.0f;
      dpix[4 % NC] = a.dL_dalpha ? a.dL_dalpha[pix] : 0.0f;
    }
    if (FEAT) {
      dpix[5 % NC] = a.dL_dfeature[pix];
      dpix[6 % NC] = a.dL_dfeature[HW + pix];
      dpix[7 % NC] = a.dL_dfeature[2 * HW + pix];
    }
  } else {
#pragma unroll
    for (int c = 0; c < NC; c++) dpix[c] = 0.0f;
  }
  // backward.cu:531-533: only the colour channels see the background
  const float bg_dot = a.bg[0] * dpix[0] + a.bg[1] * dpix[1] + a.bg[2] * dpix[2];
  // the bg term of dL/dalpha is -T_final / (1 - alpha) * bg_dot: with a zero background it is a
  // signed zero, so its division is skipped (bit-identical) -- workgroup-uniform test
  const bool has_bg = a.bg[0] != 0.0f || a.bg[1] != 0.0f || a.bg[2] != 0.0f;
  // backward.cu:502-520 keeps one accum_rec per channel and forms
  //   dL_dalpha = sum_c (col_c - accum_rec_c) * dpix_c.
  // By linearity only the projection onto dpix is needed:
  //   acc_dot' = last_alpha * last_cdot + (1 - last_alpha) * acc_dot,  cdot = sum_c col_c dpix_c,
  //   dL_dalpha = cdot - acc_dot'
  // (the same recurrence on one scalar instead of NC channels; equal up to float rounding)
  // upstream gradients as the pairs the packed math uses: A = (r, g), B = (b, depth),
  // C = (f0, f1), D = (f2, alpha) -- absent channels are zero
  const f2 dpA = mk2(dpix[0], dpix[1]);
  const f2 dpB = mk2(dpix[2], NC > 3 ? dpix[3 % NC] : 0.f);
  const f2 dpC = mk2(FEAT ? dpix[5 % NC] : 0.f, FEAT ? dpix[6 % NC] : 0.f);
  const f2 dpD = mk2(FEAT ? dpix[7 % NC] : 0.f, NC > 3 ? dpix[4 % NC] : 0.f);
  static_assert(kAccMx == 0 && kAccMy == 1 && kAccCa == 2 && kAccCb == 3 && kAccCc == 4 &&
                kAccOp == 5 && kAccR == 6 && kAccG == 7 && kAccB == 8 && kAccDepth == 9 &&
                kAccF0 == 10 && kAccF1 == 11 && kAccF2 == 12, "pair layout of the gradient row");
  // the upstream gradients' loads are waited for here: left to their first use inside the pair
  // loop, that wait (vmcnt is in-order) would also cover the previous batch's flush atomics
  asm volatile("" ::"v"(dpA.x), "v"(dpA.y), "v"(dpB.x), "v"(dpB.y), "v"(dpC.x), "v"(dpC.y),
               "v"(dpD.x), "v"(dpD.y));
  float acc_dot = 0.0f, last_cdot = 0.0f;
  float last_alpha = 0.0f;
  // PIPE: the contributing entry whose wave reduction is still to be issued (u, w, (dx, dy), its
  // batch slot); zeros reduce to zeros, so an empty pending entry needs no branch
  float p_uu = 0.0f, p_w = 0.0f;
  uint32_t p_j = 0;
  // (dx, dy) of a batch slot, re-read from LDS (one broadcast read instead of two live registers)
  auto slot_dxy = [&](uint32_t j) {
    const float4 r0 = s_r0[j];
    return mk2(r0.x - pfx, r0.y - pfy);
  };
  // the moments and colour terms of one (u, w, d) as the butterfly's 8 pairs (slot order of the
  // accumulator row: kAccMx.. kAccF2; slots 14, 15 never reach the accumulator)
  auto pair_terms = [&](float uu, float w, f2 dxy, f2 (&g)[8]) {
    g[0] = uu * dxy;                               // kAccMx, kAccMy   <- sum u dx, sum u dy
    g[1] = (uu * dxy.x) * dxy;                     // kAccCa, kAccCb   <- sum u dx dx, sum u dx dy
    g[2] = mk2((uu * dxy.y) * dxy.y, uu);          // kAccCc, kAccOp   <- sum u dy dy, sum u
    g[3] = w * dpA;                                // kAccR, kAccG
    g[4] = w * dpB;                                // kAccB, kAccDepth
    g[5] = FEAT ? w * dpC : mk2(0.f, 0.f);         // kAccF0, kAccF1
    g[6] = mk2(FEAT ? w * dpD.x : 0.f, 0.f);       // kAccF2, (13)
    g[7] = dxy;                                    // (14, 15), ignored
  };
  auto reduce_add = [&](f2 (&g)[8], uint32_t j) {
    const float sum = wave_reduce16_dpp(g, lane);
    if (red_lane && sum != 0.0f) atomicAdd(&s_acc[j * kRow + red_slot], sum);
  };
  const float ddelx_dx = (float)(0.5 * a.W);
  const float ddely_dy = (float)(0.5 * a.H);

  for (int k = (int)threadIdx.x; k < (DET ? 4 : 1) * kThreads * kRow; k += kThreads) s_acc[k] = 0.0f;

  // stage the batch starting at list position dc (back to front) into LDS, ids into s_gid[buf]
  auto stage_batch = [&](uint32_t dc, int buf) {
    const uint32_t n = min((uint32_t)kThreads, tile_last - dc);
    if (threadIdx.x < n) {
      const uint32_t rel = tile_last - 1 - dc - threadIdx.x;
      const uint32_t gid = min(a.point_list[range.x + rel], a.P - 1u);
      s_gid[buf][threadIdx.x] = gid;
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2], q3 = rec[3];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = make_float2(q1.x, q1.y);
      s_mask[threadIdx.x] = (uint8_t)wave_mask(q0, q1, q3.z, tx, ty);
      s_c0[threadIdx.x] = make_float4(q1.w, q2.x, q2.y, q1.z);
      if (FEAT) s_c1[threadIdx.x] = make_float4(q2.z, q2.w, q3.x, 1.0f);
    }
  };
#if GSR_BWD_FLUSH_LATE
  if (tile_last > 0) stage_batch(0, 0);
#endif
  // rel = position inside the tile's list; every pixel only uses rel < its n_contrib <= tile_last
  for (uint32_t done_cnt = 0; done_cnt < tile_last; done_cnt += kThreads) {
    const int buf = GSR_BWD_FLUSH_LATE ? (int)((done_cnt / kThreads) & 1u) : 0;
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, tile_last - done_cnt);
#if !GSR_BWD_FLUSH_LATE
    stage_batch(done_cnt, buf);
    __syncthreads();
#endif
    const uint32_t nlist = build_wave_list(s_mask, s_list[wid], cnt, wid, lane);
    BLEND_STAT(4, nlist);
#if GSR_BLEND_STATS
    uint32_t ncw = 0;  // this wave's contributing entries in the batch (imbalance statistic)
    __shared__ uint32_t s_maxc;
    if (threadIdx.x == 0) s_maxc = 0;
#endif
    // Four list entries per group: the cheap per-pair test (power, G, alpha) of all four is
    // evaluated first (independent work), then the entries are replayed in list order.
    for (uint32_t k0 = 0; k0 < nlist; k0 += GROUP) {
    const uint32_t packed = GROUP == 4 ? *reinterpret_cast<const uint32_t*>(&s_list[wid][k0])
                                       : (uint32_t)s_list[wid][k0];
    {
      // list order is back to front: if even the group's front-most entry lies behind every
      // pixel's last contributor in this wave, nothing in the group can contribute
      const uint32_t ulast = min((uint32_t)GROUP - 1u, nlist - 1 - k0);
      const uint32_t jl = (packed >> (8 * ulast)) & 0xffu;
      if (tile_last - 1 - done_cnt - jl >= wave_last) continue;  // wave-uniform
    }
    BLEND_STAT(5, 1);
    // Every LDS read of the group's entries is issued here, before any arithmetic (one wait per
    // group instead of one per entry and phase); the colours are consumed at once by the colour
    // dot product, so the pair phase below reads no LDS and keeps only per-entry scalars.
    float Gv[GROUP], av[GROUP], pw[GROUP], cdv[GROUP];
    f2 dxyv[GROUP];
    bool cv[GROUP];
    {
      float4 r0v[GROUP], c0v[GROUP], c1v[GROUP];
      float2 r1v[GROUP];
#pragma unroll
      for (int u = 0; u < GROUP; u++) {
        const uint32_t j = (packed >> (8 * u)) & 0xffu;
        r0v[u] = s_r0[j];
        r1v[u] = s_r1[j];
        c0v[u] = s_c0[j];
        if (FEAT) c1v[u] = s_c1[j];
      }
      float tdist = 1.0f;  // min over the group of |op * G - 1/255| (the exact-path test)
#pragma unroll
      for (int u = 0; u < GROUP; u++) {
        const float4 r0 = r0v[u];
        const float dx = r0.x - pfx, dy = r0.y - pfy;
        dxyv[u] = mk2(dx, dy);
        pw[u] = -0.5f * (r0.z * dx * dx + r1v[u].x * dy * dy) - r0.w * dx * dy;
#if GSR_BWD_FAST_EXP
        // The backward needs the forward's alpha >= 1/255 DECISION exactly, its G only to
        // gradient precision: G by the hardware exp2 (v_exp_f32, ~1 ulp; 3 instructions instead
        // of the 17 of splat_exp), and splat_exp -- the forward's and the oracle's sequence --
        // wherever op * G lies within 2e-6 (relative) of 1/255, so the decision is the forward's
        // at every pixel.  The exact path is one wave-uniform branch per group (rarely taken).
        Gv[u] = __builtin_amdgcn_exp2f(pw[u] * 1.44269504088896341f);
        {
          const float d = fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f));
          tdist = d < tdist ? d : tdist;
        }
#else
        Gv[u] = splat_exp(pw[u]);
#endif
        // cdot = sum_c col_c * dpix_c as packed FMAs over the colour pairs (gradient-only
        // arithmetic: the forward-consistent quantities G, alpha, T are computed unfused)
        const float4 c0 = c0v[u];
        f2 c2 = mk2(c0.x, c0.y) * dpA;
        c2 = fma2(mk2(c0.z, NC > 3 ? c0.w : 0.f), dpB, c2);
        if (FEAT) c2 = fma2(mk2(c1v[u].x, c1v[u].y), dpC, c2);
        if (NC > 3) c2 = fma2(mk2(FEAT ? c1v[u].z : 0.f, 1.0f), dpD, c2);
        cdv[u] = c2.x + c2.y;
#if GSR_BWD_CDOT_EARLY
        // keep the dot product here (the compiler would sink it into the contributing branch and
        // hold the colours live across the test phase)
        asm volatile("" ::"v"(cdv[u]));
#endif
      }
#if GSR_BWD_FAST_EXP
      if (__ballot(tdist <= 2e-6f * (1.0f / 255.0f))) {
#pragma unroll
        for (int u = 0; u < GROUP; u++) {
          if (fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f))
            Gv[u] = splat_exp(pw[u]);
        }
      }
#endif
#pragma unroll
      for (int u = 0; u < GROUP; u++) {
        const uint32_t j = (packed >> (8 * u)) & 0xffu;
        const uint32_t rel = tile_last - 1 - done_cnt - j;
        av[u] = fminf(0.99f, r1v[u].y * Gv[u]);
        cv[u] = (k0 + u < nlist) && rel < last_contributor && !(pw[u] > 0.0f) &&
                !(av[u] < 1.0f / 255.0f);
      }
    }
    // PIPE == 2: the group's entries for the joint reduction (zeros unless contributing)
    float q_uu[GROUP], q_w[GROUP];
    f2 q_d[GROUP];
    bool q_any = false;
#pragma unroll
    for (int u = 0; u < GROUP; u++) {
      q_uu[u] = 0.0f;
      q_w[u] = 0.0f;
      q_d[u] = mk2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < GROUP; u++) {
      const bool contrib = cv[u];
      const uint64_t cmask = __ballot(contrib);
      // wave-uniform skip (always in DET: its rows are stored, not added, so an entry past the
      // list end must not write)
      if ((DET || !GSR_BWD_NOSKIP) && cmask == 0ull) continue;
#if GSR_BWD_DIAG == 3
      // diagnostic build only (wrong gradients): no pair update / reduction -- what the batch
      // loads, lists, alpha tests, barriers and flush cost by themselves
      if (cmask != 0ull) continue;
#endif
      BLEND_STAT(6, 1);
      BLEND_STAT(7, __popcll(cmask));
      // contributing-lane histogram of the backward's entries: <= 2, <= 4, <= 8, <= 16 lanes
      BLEND_STAT(11, __popcll(cmask) <= 2);
      BLEND_STAT(12, __popcll(cmask) <= 4);
      BLEND_STAT(13, __popcll(cmask) <= 8);
      BLEND_STAT(14, __popcll(cmask) <= 16);
#if GSR_BLEND_STATS
      ncw++;
#endif
      const uint32_t j = (packed >> (8 * u)) & 0xffu;
      // Branch-free: a lane whose pixel does not take this splat runs the same arithmetic with
      // G = alpha = 0, which makes every gradient term exactly zero and T / (1 - 0) == T; its
      // recurrence state is kept by selects.  Contributing lanes compute exactly the operations
      // of the reference (backward.cu:486-555).
      const float G = contrib ? Gv[u] : 0.0f;
      const float alpha = contrib ? av[u] : 0.0f;
      const f2 dxy = dxyv[u];

#if GSR_BWD_FAST_DIV
      {
        // T / (1 - alpha) by v_rcp_f32 + one Newton correction on the exact residual (4 VALU
        // instead of the 10 of the scaled IEEE sequence): operands lie in [1e-4, 1] / [0.01, 1],
        // so the result is the correctly rounded quotient up to rare last-ulp ties; alpha = 0
        // (non-contributing lanes) gives T exactly
        const float d = 1.f - alpha;
        const float r = __builtin_amdgcn_rcpf(d);
        const float q = T * r;
        T = __builtin_fmaf(__builtin_fmaf(-q, d, T), r, q);
      }
#else
      T = T / (1.f - alpha);
#endif
      const float dchannel_dcolor = alpha * T;
      const float cdot = cdv[u];
      const float acc_new = last_alpha * last_cdot + (1.f - last_alpha) * acc_dot;
      float dL_dalpha = cdot - acc_new;
      acc_dot = contrib ? acc_new : acc_dot;
      last_cdot = contrib ? cdot : last_cdot;
      last_alpha = contrib ? alpha : last_alpha;
      dL_dalpha *= T;
      if (has_bg) dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
      // Per-pixel moments instead of the reference's per-pixel conic / mean2D terms: with
      // u = G * dL/dalpha, dL/dG = opacity * dL/dalpha, and d = (dx, dy) (backward.cu:536-554)
      //   dL/dmean2D.x = -(W/2) o (a sum u dx + b sum u dy),  dL/dmean2D.y = -(H/2) o (c sum u dy + b sum u dx)
      //   dL/dconic.{x,y,w} = -1/2 o sum u {dx dx, dx dy, dy dy},   dL/dopacity = sum u
      // The per-splat constants (a, b, c, o) are applied once per (splat, tile) at the flush.
      const float uu = G * dL_dalpha;
      if (PIPE == 2) {
        q_uu[u] = uu;
        q_w[u] = dchannel_dcolor;
        q_d[u] = dxy;
        q_any = true;
        continue;
      }
      if (PIPE == 1) {
        // the previous contributing entry's reduction, beside this entry's recurrence
        f2 g[8];
        pair_terms(p_uu, p_w, slot_dxy(p_j), g);
        reduce_add(g, p_j);
        p_uu = uu;
        p_w = dchannel_dcolor;
        p_j = j;
        continue;
      }
      f2 g[8];
      // slots 14, 15 are never read (only k < kAccDet reaches the accumulator): the dead dxy
      // pair rides along instead of two freshly zeroed registers for the butterfly's swaps
      pair_terms(uu, dchannel_dcolor, dxy, g);
#if GSR_BWD_DIAG == 1
      // diagnostic build only (wrong gradients): no wave reduction, one lane-local LDS add
      {
        f2 t = g[0] + g[1] + g[2] + g[3] + g[4] + g[5] + g[6];
        if (lane == 0 && t.x + t.y != 0.0f) atomicAdd(&s_acc[j * kRow], t.x + t.y);
      }
#else
      const float sum = wave_reduce16_dpp(g, lane);
      if (red_lane) {
        if (DET) s_acc[(wid * kThreads + j) * kRow + red_slot] = sum;
        else if (sum != 0.0f) atomicAdd(&s_acc[j * kRow + red_slot], sum);
      }
#endif
    }
    if constexpr (PIPE == 2) if (q_any) {  // wave-uniform
      f2 g[4][8];
#pragma unroll
      for (int u = 0; u < 4; u++) pair_terms(q_uu[u], q_w[u], q_d[u], g[u]);
      const float sum = wave_reduce_joint4(g, lane);
      const int k = lane & 15;
      if (k < kAccDet && sum != 0.0f)
        atomicAdd(&s_acc[((packed >> j4_shift) & 0xffu) * kRow + k], sum);
    }
    }
    if (PIPE == 1) {  // the batch's last contributing entry
      f2 g[8];
      pair_terms(p_uu, p_w, slot_dxy(p_j), g);
      reduce_add(g, p_j);
      p_uu = 0.0f;
      p_w = 0.0f;
    }
#if GSR_BLEND_STATS
    if ((threadIdx.x & 63) == 0) atomicMax(&s_maxc, ncw);
#endif
    __syncthreads();
#if GSR_BLEND_STATS
    // [9] sum over waves of contributing entries, [10] 4 x the batch's busiest wave's
    BLEND_STAT(9, ncw);
    if (threadIdx.x == 0) atomicAdd(&g_blend_stats[10], 4ull * s_maxc);
#endif
    // moments -> the reference's dL/dmean2D (NDC-scaled) and dL/dconic, once per (splat, tile)
    if (threadIdx.x < cnt) {
      const float4 r0 = s_r0[threadIdx.x];
      const float2 r1 = s_r1[threadIdx.x];
      float* row = s_acc + threadIdx.x * kRow;
      if (DET) {  // the four waves' rows, added in wave order, into wave 0's row
#pragma unroll
        for (int k = 0; k < kAccDet; k++)
          row[k] = ((row[k] + row[kThreads * kRow + k]) + row[2 * kThreads * kRow + k]) +
                   row[3 * kThreads * kRow + k];
      }
      const float sx = row[kAccMx], sy = row[kAccMy];
      const float o = r1.y;
      row[kAccMx] = -(o * (r0.z * sx + r0.w * sy)) * ddelx_dx;
      row[kAccMy] = -(o * (r1.x * sy + r0.w * sx)) * ddely_dy;
      row[kAccCa] = (-0.5f * o) * row[kAccCa];
      row[kAccCb] = (-0.5f * o) * row[kAccCb];
      row[kAccCc] = (-0.5f * o) * row[kAccCc];
    }
    __syncthreads();
#if GSR_BWD_FLUSH_LATE
    // the next batch is staged BEFORE this batch's flush: its loads are not queued behind the
    // flush's atomics (vmcnt is in-order), and those atomics retire during the next pair phase
    if (done_cnt + kThreads < tile_last) stage_batch(done_cnt + kThreads, buf ^ 1);
#endif
    // flush: lane l of wave-instruction `it` handles splat (it*16 + tid/16), slot tid%16
#pragma unroll 4
    for (int it = 0; it < kThreads * kAccFloats / kThreads; it++) {
      const uint32_t jj = (uint32_t)it * (kThreads / kAccFloats) + (threadIdx.x >> 4);
      const int k = (int)(threadIdx.x & 15);
      if (jj < cnt) {
        if (DET) {  // every slot of the instance's row is stored (zeros too), then re-zeroed
          const uint32_t q = range.x + tile_last - 1 - done_cnt - jj;
          const float v = k < kAccDet ? s_acc[jj * kRow + k] : 0.0f;
          a.partial[(size_t)min(a.einst[q], a.nrows - 1u) * kAccFloats + k] = v;
          if (k < kAccDet)
#pragma unroll
            for (int w = 0; w < 4; w++) s_acc[(w * kThreads + jj) * kRow + k] = 0.0f;
        } else if (ROWS) {  // every slot stored (16 lanes = one 64-B row), then re-zeroed
          const uint32_t q = range.x + tile_last - 1 - done_cnt - jj;
          const bool held = kRow > kAccDet || k < kAccDet;
          const float v = held ? s_acc[jj * kRow + k] : 0.0f;
          a.partial[(size_t)min(a.einst[q], a.nrows - 1u) * kAccFloats + k] = v;
          if (held) s_acc[jj * kRow + k] = 0.0f;
        } else {
          const float v = (kRow > kAccDet || k < kAccDet) ? s_acc[jj * kRow + k] : 0.0f;
          if (v != 0.0f) {
#if GSR_BWD_DIAG == 2
            // diagnostic build only (wrong gradients): the flush's traffic as plain stores
            a.acc[(size_t)s_gid[buf][jj] * kAccFloats + k] = v;
#else
            atomicAdd(&a.acc[(size_t)s_gid[buf][jj] * kAccFloats + k], v);
#endif
            s_acc[jj * kRow + k] = 0.0f;
          }
        }
      }
    }
  }
  if (ROWS) {  // instances behind the tile's last contributor: zero rows
    const uint32_t n = range.y - range.x - min(tile_last, range.y - range.x);
    for (uint32_t idx = threadIdx.x; idx < n * kAccFloats; idx += kThreads)
      a.partial[(size_t)min(a.einst[range.x + tile_last + idx / kAccFloats], a.nrows - 1u) *
                    kAccFloats + idx % kAccFloats] = 0.0f;
  }
}

template <bool EXTRA, bool FEAT, int GROUP, bool DET, bool ROWS, int PIPE>
__global__ __launch_bounds__(kThreads) GSR_BWD_WAVES(PIPE, DET) void render_bwd_kernel(RenderBwdArgs a) {
  render_bwd_tile<EXTRA, FEAT, GROUP, DET, ROWS, PIPE>(a, blockIdx.x);
}

// The backward blends of several views of a step in ONE launch: workgroup b belongs to the view k
// with first[k] <= b < first[k + 1] (view-major; inside a view the forward's heaviest-first tile
// order), so the views' launches do not each end in a tail of idle CUs, and one launch's duration
// is the time of all its views' blends.
template <bool EXTRA, bool FEAT, int GROUP, bool DET, bool ROWS, int PIPE>
__global__ __launch_bounds__(kThreads) GSR_BWD_WAVES(PIPE, DET) void render_bwd_views_kernel(RenderBwdViews m) {
  const uint32_t b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.V && b >= m.first[k + 1]) k++;  // workgroup-uniform
  render_bwd_tile<EXTRA, FEAT, GROUP, DET, ROWS, PIPE>(m.v[k], b - m.first[k]);
}

// ================================================================================================
// Backward with two pixels per lane (GSR_BWD_PIX2=1): 128-lane workgroups, wave
// w owns the 8x16 column half w of the tile, lane l the pixels (8w + l % 8, l / 8) and the one 8
// rows below.  Per list entry both pixels' recurrences run side by side (two independent chains
// per lane) and their terms are added in-lane before ONE wave reduction, which thus serves 128
// pixels instead of 64; a wave's list is the union of its two quadrants' lists.  Batches of 128
// records (one per lane), 17 KB of LDS per workgroup.  Same per-pixel arithmetic as
// render_bwd_tile, so the results agree with it up to the order of the float additions.
// ================================================================================================
constexpr int kThreads2 = 128;
template <bool EXTRA, bool FEAT, int GROUP>
__device__ __forceinline__ void render_bwd_tile2(const RenderBwdArgs& a, uint32_t blk) {
  __shared__ float4 s_r0[kThreads2];
  __shared__ float2 s_r1[kThreads2];
  __shared__ float4 s_c0[kThreads2];
  __shared__ float4 s_c1[FEAT ? kThreads2 : 1];
  __shared__ uint32_t s_gid[kThreads2];
  __shared__ float s_acc[kThreads2 * kAccPad];
  __shared__ uint8_t s_mask[kThreads2];
  __shared__ uint8_t s_list[kThreads2 / 64][kThreads2];

  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);
  const SwapOrient swap_orient = probe_swaps(lane);
  const int red_slot = reduce16_slot(lane, swap_orient);
  const bool red_lane = (lane & 3) == 0 && red_slot < kAccDet;
  const uint32_t ntiles = a.gx * a.gy;
  const uint32_t tile = sched_tile(blk, ntiles, a.sched, a.order);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  const uint32_t px = tx * kTile + (uint32_t)wid * 8u + (uint32_t)(lane & 7);
  const uint32_t py0 = ty * kTile + (uint32_t)(lane >> 3), py1 = py0 + 8u;
  const bool in0 = px < (uint32_t)a.W && py0 < (uint32_t)a.H;
  const bool in1 = px < (uint32_t)a.W && py1 < (uint32_t)a.H;
  const float pfx = (float)px, pfy0 = (float)py0, pfy1 = (float)py1;
  const size_t pix0 = (size_t)py0 * a.W + px, pix1 = (size_t)py1 * a.W + px;
  const size_t HW = (size_t)a.W * a.H;

  const uint2 range = a.ranges[tile];
  const uint32_t tile_last = a.tile_last[tile];
  const float Tf0 = in0 ? a.final_T[pix0] : 0.0f, Tf1 = in1 ? a.final_T[pix1] : 0.0f;
  float T0 = Tf0, T1 = Tf1;
  const uint32_t lc0 = in0 ? a.n_contrib[pix0] : 0u, lc1 = in1 ? a.n_contrib[pix1] : 0u;
  uint32_t wave_last = max(lc0, lc1);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) wave_last = max(wave_last, (uint32_t)__shfl_xor((int)wave_last, d, 64));

  // upstream gradients of both pixels as the packed pairs of render_bwd_tile
  auto load_dp = [&](bool in, size_t pix, f2& A, f2& B, f2& C, f2& D) {
    float d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (in) {
      d[0] = a.dL_dcolor[pix]; d[1] = a.dL_dcolor[HW + pix]; d[2] = a.dL_dcolor[2 * HW + pix];
      if (EXTRA) {
        d[3] = a.dL_ddepth ? a.dL_ddepth[pix] : 0.0f;
        d[4] = a.dL_dalpha ? a.dL_dalpha[pix] : 0.0f;
      }
      if (FEAT) {
        d[5] = a.dL_dfeature[pix]; d[6] = a.dL_dfeature[HW + pix]; d[7] = a.dL_dfeature[2 * HW + pix];
      }
    }
    A = mk2(d[0], d[1]);
    B = mk2(d[2], d[3]);
    C = mk2(d[5], d[6]);
    D = mk2(d[7], d[4]);
  };
  f2 dA0, dB0, dC0, dD0, dA1, dB1, dC1, dD1;
  load_dp(in0, pix0, dA0, dB0, dC0, dD0);
  load_dp(in1, pix1, dA1, dB1, dC1, dD1);
  const float bgd0 = a.bg[0] * dA0.x + a.bg[1] * dA0.y + a.bg[2] * dB0.x;
  const float bgd1 = a.bg[0] * dA1.x + a.bg[1] * dA1.y + a.bg[2] * dB1.x;
  const bool has_bg = a.bg[0] != 0.0f || a.bg[1] != 0.0f || a.bg[2] != 0.0f;
  asm volatile("" ::"v"(dA0.x), "v"(dA0.y), "v"(dB0.x), "v"(dB0.y), "v"(dC0.x), "v"(dC0.y),
               "v"(dD0.x), "v"(dD0.y));
  asm volatile("" ::"v"(dA1.x), "v"(dA1.y), "v"(dB1.x), "v"(dB1.y), "v"(dC1.x), "v"(dC1.y),
               "v"(dD1.x), "v"(dD1.y));
  float acc0 = 0.f, lcd0 = 0.f, la0 = 0.f, acc1 = 0.f, lcd1 = 0.f, la1 = 0.f;
  const float ddelx_dx = (float)(0.5 * a.W);
  const float ddely_dy = (float)(0.5 * a.H);
  for (int k = (int)threadIdx.x; k < kThreads2 * kAccPad; k += kThreads2) s_acc[k] = 0.0f;

  // one pixel's pair update: the recurrence and (u = G dL/dalpha, w = alpha T) of render_bwd_tile
  auto pair = [&](bool contrib, float Gv, float av, float cdot, float Tf, float bgd, float& T,
                  float& acc, float& lcd, float& la, float& uu, float& w) {
    const float G = contrib ? Gv : 0.0f;
    const float alpha = contrib ? av : 0.0f;
    {
      const float d = 1.f - alpha;
      const float r = __builtin_amdgcn_rcpf(d);
      const float q = T * r;
      T = __builtin_fmaf(__builtin_fmaf(-q, d, T), r, q);
    }
    w = alpha * T;
    const float acc_new = la * lcd + (1.f - la) * acc;
    float dL_dalpha = cdot - acc_new;
    acc = contrib ? acc_new : acc;
    lcd = contrib ? cdot : lcd;
    la = contrib ? alpha : la;
    dL_dalpha *= T;
    if (has_bg) dL_dalpha += (-Tf / (1.f - alpha)) * bgd;
    uu = G * dL_dalpha;
  };

  for (uint32_t done_cnt = 0; done_cnt < tile_last; done_cnt += kThreads2) {
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads2, tile_last - done_cnt);
    if (threadIdx.x < cnt) {
      const uint32_t rel = tile_last - 1 - done_cnt - threadIdx.x;
      const uint32_t gid = min(a.point_list[range.x + rel], a.P - 1u);
      s_gid[threadIdx.x] = gid;
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2], q3 = rec[3];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = make_float2(q1.x, q1.y);
      s_mask[threadIdx.x] = (uint8_t)wave_mask(q0, q1, q3.z, tx, ty);
      s_c0[threadIdx.x] = make_float4(q1.w, q2.x, q2.y, q1.z);
      if (FEAT) s_c1[threadIdx.x] = make_float4(q2.z, q2.w, q3.x, 1.0f);
    }
    __syncthreads();
    uint32_t nlist = 0;
    {  // the wave's list: entries reaching either of its quadrants (w top, w + 2 bottom)
      const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
#pragma unroll
      for (int c = 0; c < kThreads2 / 64; c++) {
        const uint32_t j = (uint32_t)(c * 64 + lane);
        const uint32_t m = j < cnt ? (uint32_t)s_mask[j] : 0u;
        const bool bit = ((m >> wid) | (m >> (wid + 2))) & 1u;
        const uint64_t b = __ballot(bit);
        if (bit) s_list[wid][nlist + (uint32_t)__popcll(b & lt)] = (uint8_t)j;
        nlist += (uint32_t)__popcll(b);
      }
    }
    for (uint32_t k0 = 0; k0 < nlist; k0 += GROUP) {
      const uint32_t packed = GROUP == 4 ? *reinterpret_cast<const uint32_t*>(&s_list[wid][k0])
                                         : GROUP == 2 ? (uint32_t)*reinterpret_cast<const uint16_t*>(&s_list[wid][k0])
                                                      : (uint32_t)s_list[wid][k0];
      {
        const uint32_t ulast = min((uint32_t)GROUP - 1u, nlist - 1 - k0);
        const uint32_t jl = (packed >> (8 * ulast)) & 0xffu;
        if (tile_last - 1 - done_cnt - jl >= wave_last) continue;  // wave-uniform
      }
      float G0[GROUP], G1[GROUP], a0v[GROUP], a1v[GROUP], cd0[GROUP], cd1[GROUP], dxv[GROUP];
      float dyv[GROUP], dy1v[GROUP];
      bool c0v[GROUP], c1v[GROUP];
      {
        float4 r0v[GROUP], cc0[GROUP], cc1[GROUP];
        float2 r1v[GROUP];
#pragma unroll
        for (int u = 0; u < GROUP; u++) {
          const uint32_t j = (packed >> (8 * u)) & 0xffu;
          r0v[u] = s_r0[j];
          r1v[u] = s_r1[j];
          cc0[u] = s_c0[j];
          if (FEAT) cc1[u] = s_c1[j];
        }
        float tdist = 1.0f;
        float pw0[GROUP], pw1[GROUP];
#pragma unroll
        for (int u = 0; u < GROUP; u++) {
          const float4 r0 = r0v[u];
          // each pixel's offsets exactly as the forward forms them (same power, same decisions)
          const float dx = r0.x - pfx, dy = r0.y - pfy0, dy1 = r0.y - pfy1;
          dxv[u] = dx;
          dyv[u] = dy;
          dy1v[u] = dy1;
          pw0[u] = -0.5f * (r0.z * dx * dx + r1v[u].x * dy * dy) - r0.w * dx * dy;
          pw1[u] = -0.5f * (r0.z * dx * dx + r1v[u].x * dy1 * dy1) - r0.w * dx * dy1;
          G0[u] = __builtin_amdgcn_exp2f(pw0[u] * 1.44269504088896341f);
          G1[u] = __builtin_amdgcn_exp2f(pw1[u] * 1.44269504088896341f);
          const float e0 = fabsf(r1v[u].y * G0[u] - (1.0f / 255.0f));
          const float e1 = fabsf(r1v[u].y * G1[u] - (1.0f / 255.0f));
          tdist = fminf(tdist, fminf(e0, e1));
          const float4 c0 = cc0[u];
          f2 x0 = mk2(c0.x, c0.y) * dA0, x1 = mk2(c0.x, c0.y) * dA1;
          x0 = fma2(mk2(c0.z, EXTRA ? c0.w : 0.f), dB0, x0);
          x1 = fma2(mk2(c0.z, EXTRA ? c0.w : 0.f), dB1, x1);
          if (FEAT) {
            x0 = fma2(mk2(cc1[u].x, cc1[u].y), dC0, x0);
            x1 = fma2(mk2(cc1[u].x, cc1[u].y), dC1, x1);
          }
          if (EXTRA) {
            x0 = fma2(mk2(FEAT ? cc1[u].z : 0.f, 1.0f), dD0, x0);
            x1 = fma2(mk2(FEAT ? cc1[u].z : 0.f, 1.0f), dD1, x1);
          }
          cd0[u] = x0.x + x0.y;
          cd1[u] = x1.x + x1.y;
        }
        if (__ballot(tdist <= 2e-6f * (1.0f / 255.0f))) {
#pragma unroll
          for (int u = 0; u < GROUP; u++) {
            if (fabsf(r1v[u].y * G0[u] - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f)) G0[u] = splat_exp(pw0[u]);
            if (fabsf(r1v[u].y * G1[u] - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f)) G1[u] = splat_exp(pw1[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < GROUP; u++) {
          const uint32_t j = (packed >> (8 * u)) & 0xffu;
          const uint32_t rel = tile_last - 1 - done_cnt - j;
          a0v[u] = fminf(0.99f, r1v[u].y * G0[u]);
          a1v[u] = fminf(0.99f, r1v[u].y * G1[u]);
          const bool live = k0 + u < nlist;
          c0v[u] = live && rel < lc0 && !(pw0[u] > 0.0f) && !(a0v[u] < 1.0f / 255.0f);
          c1v[u] = live && rel < lc1 && !(pw1[u] > 0.0f) && !(a1v[u] < 1.0f / 255.0f);
        }
      }
#pragma unroll
      for (int u = 0; u < GROUP; u++) {
        if (__ballot(c0v[u] || c1v[u]) == 0ull) continue;  // wave-uniform
        const uint32_t j = (packed >> (8 * u)) & 0xffu;
        float u0, w0, u1, w1;
        pair(c0v[u], G0[u], a0v[u], cd0[u], Tf0, bgd0, T0, acc0, lcd0, la0, u0, w0);
        pair(c1v[u], G1[u], a1v[u], cd1[u], Tf1, bgd1, T1, acc1, lcd1, la1, u1, w1);
        const float dx = dxv[u], dy0 = dyv[u], dy1 = dy1v[u];
        // both pixels' terms, added in-lane, then one reduction over the wave's 128 pixels
        const float usum = u0 + u1;
        const float ux = u0 * dx + u1 * dx;
        f2 g[8];
        g[0] = mk2(ux, u0 * dy0 + u1 * dy1);
        g[1] = mk2(ux * dx, (u0 * dx) * dy0 + (u1 * dx) * dy1);
        g[2] = mk2((u0 * dy0) * dy0 + (u1 * dy1) * dy1, usum);
        g[3] = w0 * dA0 + w1 * dA1;
        g[4] = w0 * dB0 + w1 * dB1;
        g[5] = FEAT ? w0 * dC0 + w1 * dC1 : mk2(0.f, 0.f);
        g[6] = mk2(FEAT ? w0 * dD0.x + w1 * dD1.x : 0.f, 0.f);
        g[7] = mk2(dx, dy0);
        const float sum = wave_reduce16_dpp(g, lane);
        if (red_lane && sum != 0.0f) atomicAdd(&s_acc[j * kAccPad + red_slot], sum);
      }
    }
    __syncthreads();
    if (threadIdx.x < cnt) {
      const float4 r0 = s_r0[threadIdx.x];
      const float2 r1 = s_r1[threadIdx.x];
      float* row = s_acc + threadIdx.x * kAccPad;
      const float sx = row[kAccMx], sy = row[kAccMy];
      const float o = r1.y;
      row[kAccMx] = -(o * (r0.z * sx + r0.w * sy)) * ddelx_dx;
      row[kAccMy] = -(o * (r1.x * sy + r0.w * sx)) * ddely_dy;
      row[kAccCa] = (-0.5f * o) * row[kAccCa];
      row[kAccCb] = (-0.5f * o) * row[kAccCb];
      row[kAccCc] = (-0.5f * o) * row[kAccCc];
    }
    __syncthreads();
#pragma unroll 4
    for (int it = 0; it < kThreads2 * kAccFloats / kThreads2; it++) {
      const uint32_t jj = (uint32_t)it * (kThreads2 / kAccFloats) + (threadIdx.x >> 4);
      const int k = (int)(threadIdx.x & 15);
      if (jj < cnt) {
        const float v = s_acc[jj * kAccPad + k];
        if (v != 0.0f) {
          atomicAdd(&a.acc[(size_t)s_gid[jj] * kAccFloats + k], v);
          s_acc[jj * kAccPad + k] = 0.0f;
        }
      }
    }
  }
}

template <bool EXTRA, bool FEAT, int GROUP>
__global__ __launch_bounds__(kThreads2) void render_bwd2_views_kernel(RenderBwdViews m) {
  const uint32_t b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.V && b >= m.first[k + 1]) k++;  // workgroup-uniform
  render_bwd_tile2<EXTRA, FEAT, GROUP>(m.v[k], b - m.first[k]);
}

// GSR_BWD_PIX2 (default 0): the two-pixels-per-lane backward above; its list group size
static int bwd_pix2() {
  static const int g = [] {
    const char* e = getenv("GSR_BWD_PIX2");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  return g;
}

// GSR_BWD_PIPE (default 0): the pipelined wave reduction of render_bwd_tile (1), the joint
// reduction of a group's four entries (2), or neither (0)
static int bwd_pipe() {
  static const int mode = [] {
    const char* e = getenv("GSR_BWD_PIPE");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2) ? v : 0;
  }();
  return mode;
}

// ================================================================================================
// Forward with block lists: each wave's 64 lanes are four 16-lane groups, group g = lane bits
// (1, 2) owning a 4x4 pixel block of the wave's 8x8 quadrant, and every group walks its OWN
// compacted list of the batch, so a wave step evaluates four (block, splat) entries at once.  A
// (quadrant, splat) entry has only ~24 of its 64 lanes contributing (scripts/blend_stats.py, bench
// scene); per wave the longest block list is 78 entries against 100 in the quadrant list, and
// render_fwd drops 0.128 -> 0.116 ms at 1 stream.  Per pixel the blend's operations and their
// order are unchanged: outputs bit-identical to render_fwd_kernel (GSR_BLOCK_LISTS=0).
// The same structure in the backward (16-lane group reductions over lane bits {5, 4, 3, 0}) was
// measured slower, 0.236 -> 0.253 ms: its wave steps with a contributing lane fell only from 68 to
// 57 per wave while the 16-bit masks and four lists per batch cost more than that saved.
// ================================================================================================

// lane -> pixel: quadrant (w & 1, w >> 1); block g = blk_group(lane) at (g & 1, g >> 1) inside
// it.  GSR_FWD_GROUP_ROWS (default 1, round 4): block g is lanes 16 g .. 16 g + 15 (x = lane & 3,
// y = (lane >> 2) & 3), i.e. exactly one of ds_read_b128's 16-lane groups, so a group's record
// reads are one address (a broadcast) and never conflict across the four blocks' records (round 3
// 's map, g = lane bits 1-2 with x = bit0 + 2 bit3, y = bit4 + 2 bit5, put all four blocks in
// every 16-lane group: a 2-way bank conflict whenever two of the four records share an index mod
// 16).  Per pixel the blend is unchanged: outputs bit-identical either way.
#ifndef GSR_FWD_GROUP_ROWS
#define GSR_FWD_GROUP_ROWS 1
#endif
__device__ __forceinline__ uint32_t blk_group(uint32_t l) {
  return GSR_FWD_GROUP_ROWS ? (l >> 4) : ((l >> 1) & 3u);
}
__device__ __forceinline__ void pixel_of_blk(uint32_t tx, uint32_t ty, uint32_t t, uint32_t& px,
                                             uint32_t& py) {
  const uint32_t w = t >> 6, l = t & 63u, g = blk_group(l);
  const uint32_t bx = GSR_FWD_GROUP_ROWS ? (l & 3u) : ((l & 1u) | ((l >> 2) & 2u));
  const uint32_t by = GSR_FWD_GROUP_ROWS ? ((l >> 2) & 3u) : ((l >> 4) & 3u);
  px = tx * kTile + (w & 1u) * 8u + (g & 1u) * 4u + bx;
  py = ty * kTile + (w >> 1) * 8u + (g >> 1) * 4u + by;
}

// Which of the 16 4x4 blocks a splat can reach: bit 4w + g for block g of quadrant w.  The exact
// quadrant test (wave_mask) ANDed with the blocks met by the axis-aligned bounding box of the
// splat's cut ellipse q <= c, where c widens q_cut by cut_touches_rect's own margin
// (2e-2 + 1e-4 |terms|, with |terms| <= c * ta on the ellipse) -- a superset of the blocks where
// any pixel can reach alpha >= 1/255, like the quadrant test.
__device__ __forceinline__ uint32_t block_mask(float4 r0, float4 r1, float qc, uint32_t tx,
                                               uint32_t ty) {
  const uint32_t qm = wave_mask(r0, r1, qc, tx, ty);
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) m |= ((qm >> w) & 1u) ? (0xfu << (4 * w)) : 0u;
  if (qc < 0.0f || m == 0) return m;
  const float ca = r0.z, cb = r0.w, cc = r1.x;
  const float det = ca * cc - cb * cb;
  if (!(det > 0.0f)) return m;
  const float h2x = cc / det, h2y = ca / det;  // (half-extent)^2 per unit c
  const float ta = ca * h2x + cc * h2y + 2.0f * fabsf(cb) * sqrtf(h2x * h2y);
  if (!(1e-4f * ta < 0.5f)) return m;
  const float c = (qc + 2e-2f) / (1.0f - 1e-4f * ta) * 1.001f;
  const float hx = sqrtf(c * h2x) * 1.001f + 1e-3f, hy = sqrtf(c * h2y) * 1.001f + 1e-3f;
  // 4-pixel columns / rows of the tile met by [mx - hx, mx + hx] x [my - hy, my + hy]
  const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
  uint32_t cols = 0, rows = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float x0 = bx0 + 4.0f * i, y0 = by0 + 4.0f * i;
    cols |= (x0 <= r0.x + hx && x0 + 3.0f >= r0.x - hx) ? (1u << i) : 0u;
    rows |= (y0 <= r0.y + hy && y0 + 3.0f >= r0.y - hy) ? (1u << i) : 0u;
  }
  // block g of quadrant w covers tile column 2 (w & 1) + (g & 1), row 2 (w >> 1) + (g >> 1)
  uint32_t bb = 0;
#pragma unroll
  for (int w = 0; w < 4; w++)
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const int cx = 2 * (w & 1) + (g & 1), cy = 2 * (w >> 1) + (g >> 1);
      bb |= (((cols >> cx) & (rows >> cy)) & 1u) << (4 * w + g);
    }
  return m & bb;
}

// Per-group compaction: group g's list holds, in batch order, the entries whose mask has bit
// 4 wid + g.  Returns this lane's group's length; `nmax` gets the longest of the wave's four.
// The four lists of a wave sit kListRow bytes apart: a 4-byte pad puts the four groups' list
// reads (one ds_read_b32 per step, four addresses per wave) on four different banks instead of
// one (256-byte rows: a 4-way conflict on every step).
constexpr int kListRow = kThreads + 4;
__device__ __forceinline__ uint32_t build_group_lists(const uint16_t* s_mask, uint8_t (*list)[kListRow],
                                                      uint32_t cnt, int wid, int lane, uint32_t grp,
                                                      uint32_t& nmax, uint32_t& ntot) {
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t n[4] = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < kThreads / 64; c++) {
    const uint32_t j = (uint32_t)(c * 64 + lane);
    const uint32_t bits = j < cnt ? ((uint32_t)s_mask[j] >> (4 * wid)) & 0xfu : 0u;
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const bool bit = (bits >> g) & 1u;
      const uint64_t b = __ballot(bit);
      if (bit) list[g][n[g] + (uint32_t)__popcll(b & lt)] = (uint8_t)j;
      n[g] += (uint32_t)__popcll(b);
    }
  }
  nmax = max(max(n[0], n[1]), max(n[2], n[3]));
  ntot = n[0] + n[1] + n[2] + n[3];
  return grp == 0 ? n[0] : grp == 1 ? n[1] : grp == 2 ? n[2] : n[3];
}

// GSR_FWD_LAZY=1: the block-list forward reads a group's channel values (colour, depth,
// feature) after its four alpha tests instead of with the geometry, so they are not live in
// VGPRs through the tests (more waves per SIMD)
#ifndef GSR_FWD_LAZY
#define GSR_FWD_LAZY 0
#endif
// waves per SIMD the block-list forward is compiled for (VGPR budget 512 / n).  Round 2: 5
// measured slower (96 VGPRs with 16 spilled: 0.116 -> 0.122 ms per view).  Round 4, with the
// hardware-exp2 alpha test and the block-to-lane map: 5 (96 VGPRs, 4 spilled) 0.262 / 0.263
// against 0.275 / 0.276 ms per 3-view launch at the default 104 VGPRs (4 waves); the lazy
// channel reads at 5 / 6 waves 0.271 / 0.265 (profiles/r04_fwd_occ_ab.txt) -- 5, no lazy reads
#ifndef GSR_FWD_BLK_WAVES
#define GSR_FWD_BLK_WAVES 5
#endif
// FAST (GSR_FWD_FAST, default 1; round 4): G by the hardware exp2 (v_exp_f32, 3 instructions
// instead of the 17 of splat_exp) with splat_exp wherever op * G lies within 2e-6 (relative) of
// 1/255 -- the alpha >= 1/255 decision stays the oracle's exactly, G differs from splat_exp's by
// < 1e-6 relative (so the T < 1e-4 stop can flip only at pixels within ~1e-6 of it, inside the
// parity tests' threshold margin); the backward evaluates the same instruction sequence
// (GSR_BWD_FAST_EXP), so its alpha is the forward's bit for bit.  render_fwd 0.294 / 0.299 ->
// 0.279 / 0.284 ms per 3-view launch (profiles/r04_fwd_fast_ab.txt).  Fused multiply-adds for
// the channel sums (output-only arithmetic) measured slower, 0.313 ms, and were dropped.
template <bool FEAT, bool FAST>
__device__ __forceinline__ void render_fwd_blk_tile(const RenderArgs& a, uint32_t blk) {
  __shared__ float4 s_r0[kThreads];
  __shared__ float4 s_r1[kThreads];
  __shared__ float4 s_r2[kThreads];
  __shared__ float s_f2[FEAT ? kThreads : 1];  // rec[3].x (feature 2) only
  __shared__ uint16_t s_mask[kThreads];
  __shared__ uint8_t s_list[kThreads / 64][4][kListRow];
  __shared__ uint32_t s_max;
  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);
  const uint32_t grp = blk_group((uint32_t)lane);

  const uint32_t ntiles = a.gx * a.gy;
  side_clear(a.clear.p, a.clear.bytes, (size_t)blk * kThreads + threadIdx.x, (size_t)ntiles * kThreads);
  const uint32_t tile = sched_tile(blk, ntiles, a.sched, a.order);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  uint32_t px, py;
  pixel_of_blk(tx, ty, threadIdx.x, px, py);
  const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
  const float pfx = (float)px, pfy = (float)py;
  bool done = !inside;
  if (threadIdx.x == 0) s_max = 0;

  // a sort of this call gave up: NaN outputs, the backward fails (see render_fwd_kernel)
  if (*a.status & (kStatusDepthSort | kStatusTileSort)) {
    if (threadIdx.x == 0) a.tile_last[tile] = 0;
    if (inside) {
      const size_t pix = (size_t)py * a.W + px, HW = (size_t)a.W * a.H;
      const float nan = __builtin_nanf("");
      a.final_T[pix] = nan;
      a.n_contrib[pix] = 0;
      for (int c = 0; c < 3; c++) a.out_color[c * HW + pix] = nan;
      if (a.out_depth) a.out_depth[pix] = nan;
      if (a.out_alpha) a.out_alpha[pix] = nan;
      if (a.out_feature)
        for (int c = 0; c < 3; c++) a.out_feature[c * HW + pix] = nan;
    }
    return;
  }

  const uint2 range = a.ranges[tile];
  float T = 1.0f;
  uint32_t last_contributor = 0;
  constexpr int NC = FEAT ? 8 : 5;
  float C[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) C[c] = 0.0f;

  for (uint32_t base = range.x; base < range.y; base += kThreads) {
    // forward.cu:309-311: stop when every pixel of the tile is saturated
    if (__syncthreads_count(done) == kThreads) break;
    const uint32_t i = base + threadIdx.x;
    if (i < range.y) {
      const uint32_t pid = a.point_list[i];
      if (pid >= a.P) {  // memory-safe clamp, reported to this call's status check
        atomicOr(a.status, kStatusClamp);
        if (a.host_status) *a.host_status = kStatusClamp;
        if (a.fault) atomicOr(a.fault, kStatusClamp);
      }
      const uint32_t gid = min(pid, a.P - 1u);
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1], q3 = rec[3];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = q1;
      s_r2[threadIdx.x] = rec[2];
      if (FEAT) s_f2[threadIdx.x] = q3.x;
      s_mask[threadIdx.x] = (uint16_t)block_mask(q0, q1, q3.z, tx, ty);
    }
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, range.y - base);
    uint32_t nmax, ntot;
    const uint32_t nl = build_group_lists(s_mask, s_list[wid], cnt, wid, lane, grp, nmax, ntot);
    BLEND_STAT(0, nmax);
    BLEND_STAT(1, ntot);
    const uint32_t rel0 = base - range.x;
    // four entries of the group's list per iteration, as render_fwd_kernel
    for (uint32_t k = 0; k < nmax; k += 4) {
      if (__ballot(!done) == 0ull) break;  // wave-uniform
      BLEND_STAT(2, 4);
      const uint32_t packed = *reinterpret_cast<const uint32_t*>(&s_list[wid][grp][k]);
      uint32_t jj[4];
      float pw[4], al[4];
      float4 r1v[4], r2v[4];
      float f2v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        jj[u] = (packed >> (8 * u)) & 0xffu;
        const float4 r0 = s_r0[jj[u]];
        r1v[u] = s_r1[jj[u]];
        if (!GSR_FWD_LAZY) {
          r2v[u] = s_r2[jj[u]];
          f2v[u] = FEAT ? s_f2[jj[u]] : 0.0f;
        }
        const float dx = r0.x - pfx, dy = r0.y - pfy;
        const float power = -0.5f * (r0.z * dx * dx + r1v[u].x * dy * dy) - r0.w * dx * dy;
        // entries past the group's list end get power = +1 and are skipped
        pw[u] = (k + u < nl) ? power : 1.0f;
#if !GSR_FWD_TEST_FIRST
        if (FAST) {
          float G = __builtin_amdgcn_exp2f(pw[u] * 1.44269504088896341f);
          if (fabsf(r1v[u].y * G - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f)) G = splat_exp(pw[u]);
          al[u] = fminf(0.99f, r1v[u].y * G);
        } else {
          al[u] = fminf(0.99f, r1v[u].y * splat_exp(pw[u]));
        }
#endif
      }
#if GSR_FWD_TEST_FIRST
      {
        float G4[4];
        splat_exp_n<4>(pw, G4);
#pragma unroll
        for (int u = 0; u < 4; u++) al[u] = fminf(0.99f, r1v[u].y * G4[u]);
      }
      // the four entries' power / exp / alpha are evaluated here, for every lane, as four
      // independent chains: left alone, the compiler sinks each into the replay's per-lane
      // `done` branches below and serialises the exps
      asm volatile("" ::"v"(al[0]), "v"(al[1]), "v"(al[2]), "v"(al[3]), "v"(pw[0]), "v"(pw[1]),
                   "v"(pw[2]), "v"(pw[3]));
#endif
#if GSR_FWD_LAZY
      // the channel values of the four entries are read only now: no LDS access crosses this
      // point, so they are not live (and held in VGPRs) through the alpha tests above
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < 4; u++) {
        r1v[u] = s_r1[jj[u]];
        r2v[u] = s_r2[jj[u]];
        f2v[u] = FEAT ? s_f2[jj[u]] : 0.0f;
      }
#endif
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (done) continue;
        if (pw[u] > 0.0f) continue;
        const float alpha = al[u];
        if (alpha < 1.0f / 255.0f) continue;
        const float test_T = T * (1 - alpha);
        if (test_T < 0.0001f) {
          done = true;
          continue;
        }
        const float wgt = alpha * T;
        C[0] += r1v[u].w * wgt;
        C[1] += r2v[u].x * wgt;
        C[2] += r2v[u].y * wgt;
        C[3] += r1v[u].z * wgt;
        C[4] += wgt;
        if (FEAT) {
          C[5 % NC] += r2v[u].z * wgt;
          C[6 % NC] += r2v[u].w * wgt;
          C[7 % NC] += f2v[u] * wgt;
        }
        T = test_T;
        last_contributor = rel0 + jj[u] + 1;
      }
    }
  }

  uint32_t m = last_contributor;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) atomicMax(&s_max, m);
  __syncthreads();
  if (threadIdx.x == 0) a.tile_last[tile] = s_max;

  if (inside) {
    const size_t pix = (size_t)py * a.W + px;
    const size_t HW = (size_t)a.W * a.H;
    a.final_T[pix] = T;
    a.n_contrib[pix] = last_contributor;
    a.out_color[pix] = C[0] + T * a.bg[0];
    a.out_color[HW + pix] = C[1] + T * a.bg[1];
    a.out_color[2 * HW + pix] = C[2] + T * a.bg[2];
    if (a.out_depth) a.out_depth[pix] = C[3];
    if (a.out_alpha) a.out_alpha[pix] = C[4];
    if (a.out_feature) {
      a.out_feature[pix] = FEAT ? C[FEAT ? 5 : 0] : 0.0f;
      a.out_feature[HW + pix] = FEAT ? C[FEAT ? 6 : 0] : 0.0f;
      a.out_feature[2 * HW + pix] = FEAT ? C[FEAT ? 7 : 0] : 0.0f;
    }
  }
}

template <bool FEAT, bool FAST>
__global__ __launch_bounds__(kThreads, GSR_FWD_BLK_WAVES) void render_fwd_blk_kernel(RenderArgs a) {
  render_fwd_blk_tile<FEAT, FAST>(a, blockIdx.x);
}

// The forward blends of several views in ONE launch (view-major workgroups, as
// render_bwd_views_kernel): no per-view tail of idle CUs.
template <bool FEAT, bool FAST>
__global__ __launch_bounds__(kThreads, GSR_FWD_BLK_WAVES) void render_fwd_blk_views_kernel(
    RenderFwdViews m) {
  const uint32_t b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.V && b >= m.first[k + 1]) k++;  // workgroup-uniform
  render_fwd_blk_tile<FEAT, FAST>(m.v[k], b - m.first[k]);
}

__global__ void expf_pair_kernel(const float* __restrict__ x, float* __restrict__ ref,
                                 float* __restrict__ fast, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    ref[i] = expf(x[i]);
    fast[i] = splat_exp(x[i]);
  }
}

// The fused path's GaussianModel activations, exactly as the preprocess / backward kernels evaluate
// them (gsr_device.h): sigmoid(_opacity), exp(_scaling), normalize(_rotation).
__global__ void activations_kernel(const float* __restrict__ op_raw, const float* __restrict__ sc_raw,
                                   const float4* __restrict__ rot_raw, size_t P,
                                   float* __restrict__ op, float* __restrict__ sc,
                                   float4* __restrict__ rot) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  op[i] = sigmoid_f(op_raw[i]);
  sc[3 * i] = expf(sc_raw[3 * i]);
  sc[3 * i + 1] = expf(sc_raw[3 * i + 1]);
  sc[3 * i + 2] = expf(sc_raw[3 * i + 2]);
  rot[i] = normalize_quat(rot_raw[i]);
}

}  // namespace

hipError_t launch_activations(const float* op_raw, const float* sc_raw, const float* rot_raw,
                              size_t P, float* op, float* sc, float* rot, hipStream_t s) {
  if (P == 0) return hipSuccess;
  hipLaunchKernelGGL(activations_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s,
                     op_raw, sc_raw, reinterpret_cast<const float4*>(rot_raw), P, op, sc,
                     reinterpret_cast<float4*>(rot));
  return hipGetLastError();
}

#if GSR_BLEND_STATS
extern "C" int gsr_test_blend_stats(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blend_stats), sizeof(g_blend_stats)) != hipSuccess) return 2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_blend_stats), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif

hipError_t launch_expf_pair(const float* x, float* ref, float* fast, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(expf_pair_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ref,
                     fast, n);
  return hipGetLastError();
}

// GSR_BLOCK_LISTS=0 selects the quadrant-list kernels (one list per wave) for A/B runs
// GSR_FWD_FAST (default 1): render_fwd_blk_tile's hardware-exp2 alpha test; 0 = splat_exp
static bool fwd_fast() {
  static const bool v = [] {
    const char* e = getenv("GSR_FWD_FAST");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

static bool block_lists() {
  static const bool on = [] {
    const char* e = getenv("GSR_BLOCK_LISTS");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

hipError_t launch_render_schedule(const RenderArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0 || a.sched != 2) return hipSuccess;
  hipLaunchKernelGGL(tile_schedule_kernel, dim3(1), dim3(kSchedThreads), 0, s, a.ranges,
                     (const uint32_t*)nullptr, ntiles, a.order);
  return hipGetLastError();
}

hipError_t launch_render_schedule_views(const RenderArgs* views, int V, hipStream_t s) {
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  SchedViews m{};
  int n = 0;
  for (int k = 0; k < V; k++) {
    const RenderArgs& a = views[k];
    if (a.gx * a.gy == 0 || a.sched != 2) continue;
    m.ranges[n] = a.ranges;
    m.order[n] = a.order;
    m.ntiles[n] = a.gx * a.gy;
    n++;
  }
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_schedule_views_kernel, dim3((unsigned)n), dim3(kSchedThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t launch_render_forward_views(const RenderArgs* views, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxFwdViews) return hipErrorInvalidValue;
  if (!block_lists()) {  // the quadrant-list kernel: one launch per view
    for (int k = 0; k < V; k++) {
      const RenderArgs& a = views[k];
      if (a.gx * a.gy == 0) continue;
      if (a.include_feature)
        hipLaunchKernelGGL(render_fwd_kernel<true>, dim3(a.gx * a.gy), dim3(kThreads), 0, s, a);
      else
        hipLaunchKernelGGL(render_fwd_kernel<false>, dim3(a.gx * a.gy), dim3(kThreads), 0, s, a);
    }
    return hipGetLastError();
  }
  RenderFwdViews m{};
  m.V = V;
  m.first[0] = 0;
  const bool feat = views[0].include_feature != 0;
  for (int k = 0; k < V; k++) {
    if ((views[k].include_feature != 0) != feat) return hipErrorInvalidValue;
    m.v[k] = views[k];
    m.first[k + 1] = m.first[k] + views[k].gx * views[k].gy;
  }
  if (m.first[V] == 0) return hipSuccess;
#define GSR_FWDV(F)                                                                               \
  do {                                                                                           \
    if (fwd_fast())                                                                              \
      hipLaunchKernelGGL((render_fwd_blk_views_kernel<F, true>), dim3(m.first[V]), dim3(kThreads), 0, s, m); \
    else                                                                                         \
      hipLaunchKernelGGL((render_fwd_blk_views_kernel<F, false>), dim3(m.first[V]), dim3(kThreads), 0, s, m); \
  } while (0)
  if (feat) GSR_FWDV(true);
  else GSR_FWDV(false);
#undef GSR_FWDV
  return hipGetLastError();
}

hipError_t launch_render_forward(const RenderArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0) return hipSuccess;
  if (a.sched == 2)
    hipLaunchKernelGGL(tile_schedule_kernel, dim3(1), dim3(kSchedThreads), 0, s, a.ranges,
                       (const uint32_t*)nullptr, ntiles, a.order);
  if (block_lists()) {
#define GSR_FWD1(F)                                                                               \
  do {                                                                                           \
    if (fwd_fast())                                                                              \
      hipLaunchKernelGGL((render_fwd_blk_kernel<F, true>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else                                                                                         \
      hipLaunchKernelGGL((render_fwd_blk_kernel<F, false>), dim3(ntiles), dim3(kThreads), 0, s, a); \
  } while (0)
    if (a.include_feature) GSR_FWD1(true);
    else GSR_FWD1(false);
#undef GSR_FWD1
  } else if (a.include_feature)
    hipLaunchKernelGGL(render_fwd_kernel<true>, dim3(ntiles), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(render_fwd_kernel<false>, dim3(ntiles), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_render_backward_views(const RenderBwdArgs* views, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBwdViews) return hipErrorInvalidValue;
  const RenderBwdArgs& a = views[0];
  const bool extra = a.dL_ddepth != nullptr || a.dL_dalpha != nullptr;
  const bool feat = a.include_feature && a.dL_dfeature != nullptr;
  RenderBwdViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    const RenderBwdArgs& w = views[k];
    // one kernel instance for all: the views must agree on the template switches
    if ((w.dL_ddepth != nullptr || w.dL_dalpha != nullptr) != extra ||
        (w.include_feature && w.dL_dfeature != nullptr) != feat ||
        (w.partial != nullptr) != (a.partial != nullptr) || w.det != a.det ||
        (a.sched == 2) != (w.sched == 2))
      return hipErrorInvalidValue;
    m.v[k] = w;
    m.first[k + 1] = m.first[k] + w.gx * w.gy;
  }
  const uint32_t nblk = m.first[V];
  if (nblk == 0) return hipSuccess;
  if (bwd_pix2() && !a.partial && a.sched == 2) {  // the two-pixels-per-lane variant (A/B)
#define GSR_BWD2(E, F)                                                                            \
    do {                                                                                           \
      if (bwd_pix2() == 4)                                                                         \
        hipLaunchKernelGGL((render_bwd2_views_kernel<E, F, 4>), dim3(nblk), dim3(kThreads2), 0, s, m); \
      else if (bwd_pix2() == 2)                                                                    \
        hipLaunchKernelGGL((render_bwd2_views_kernel<E, F, 2>), dim3(nblk), dim3(kThreads2), 0, s, m); \
      else                                                                                         \
        hipLaunchKernelGGL((render_bwd2_views_kernel<E, F, 1>), dim3(nblk), dim3(kThreads2), 0, s, m); \
    } while (0)
    if (feat) GSR_BWD2(true, true);
    else if (extra) GSR_BWD2(true, false);
    else GSR_BWD2(false, false);
#undef GSR_BWD2
    return hipGetLastError();
  }
#define GSR_BWDV(E, F)                                                                            \
  do {                                                                                           \
    if (a.partial && a.det)                                                                      \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, 4, true, true, 0>), dim3(nblk), dim3(kThreads), 0, s, m); \
    else if (a.partial)                                                                          \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, 4, false, true, 0>), dim3(nblk), dim3(kThreads), 0, s, m); \
    else if (bwd_pipe() == 2)                                                                    \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, 4, false, false, 2>), dim3(nblk), dim3(kThreads), 0, s, m); \
    else if (bwd_pipe() == 1)                                                                    \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, 4, false, false, 1>), dim3(nblk), dim3(kThreads), 0, s, m); \
    else                                                                                         \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, 4, false, false, 0>), dim3(nblk), dim3(kThreads), 0, s, m); \
  } while (0)
  if (feat) GSR_BWDV(true, true);
  else if (extra) GSR_BWDV(true, false);
  else GSR_BWDV(false, false);
#undef GSR_BWDV
  return hipGetLastError();
}

hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0) return hipSuccess;
  const bool extra = a.dL_ddepth != nullptr || a.dL_dalpha != nullptr;
  const bool feat = a.include_feature && a.dL_dfeature != nullptr;
  static const int group = [] {
    const char* e = getenv("GSR_BWD_GROUP");
    return (e && atoi(e) == 1) ? 1 : 4;
  }();
  static const bool resched = [] {
    const char* e = getenv("GSR_BWD_RESCHED");
    return e && atoi(e) == 1;
  }();
  // The backward keeps the forward's heaviest-first order (by list length, still in a.order):
  // re-ranking by the replayed prefix (max n_contrib, GSR_BWD_RESCHED=1) costs a launch and was
  // measured slower, render_bwd 0.2361 vs 0.2324 ms at 1 stream, 3.408-3.427 vs 3.391-3.395 ms
  // per 3-stream step
  if (a.sched == 2 && resched)
    hipLaunchKernelGGL(tile_schedule_kernel, dim3(1), dim3(kSchedThreads), 0, s, a.ranges,
                       a.tile_last, ntiles, a.order);
#define GSR_BWD(E, F)                                                                             \
  do {                                                                                           \
    if (a.partial && a.det)                                                                      \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 4, true, true, 0>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else if (a.partial)                                                                          \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 4, false, true, 0>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else if (group == 1)                                                                         \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 1, false, false, 0>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else if (bwd_pipe() == 2)                                                                    \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 4, false, false, 2>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else if (bwd_pipe() == 1)                                                                    \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 4, false, false, 1>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else                                                                                         \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, 4, false, false, 0>), dim3(ntiles), dim3(kThreads), 0, s, a); \
  } while (0)
  if (feat) GSR_BWD(true, true);
  else if (extra) GSR_BWD(true, false);
  else GSR_BWD(false, false);
#undef GSR_BWD
  return hipGetLastError();
}

}  // namespace gsr

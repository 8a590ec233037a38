// gsr_render.hip -- per-tile alpha blending, forward and backward, for gfx950.
//
// Reference behaviour: renderCUDA forward (cuda_rasterizer/forward.cu:261-374) and backward
// (cuda_rasterizer/backward.cu:399-557), extended with depth / alpha / 3-channel feature outputs
// (SURVEY.md row A12).
//
// gfx950 design:
//  * one 256-lane workgroup (4 waves of 64) per 16x16 tile; tiles are taken heaviest first
//    (tile_schedule_kernel, LPT order) so the centre-heavy tiles do not form the tail;
//  * batches of splat records (64 B each, packed by the preprocess) staged in LDS and read by all
//    lanes as broadcasts; each wave compacts a batch to the splats that can reach alpha >= 1/255
//    in its pixels (the conservative test the binning uses);
//  * forward: each wave's 64 lanes are four 16-lane groups owning 4x4 pixel blocks, each walking
//    its own compacted list (block lists);
//  * backward (two phases per wave): the two halves of a wave's quadrant walk
//    their own lists; phase 1 replays the tile back to front with lanes = pixels (the reference's
//    per-pixel recurrence, backward.cu:482-534) and parks each contributing splat's per-pixel
//    pair (u = G dL/dalpha, w = alpha T) in LDS; phase 2 switches to lanes = (splat, pixel row),
//    sums the 13 gradient values over the pixels in registers, eight slots at a time, and flushes
//    them as global float atomics, each wave-instruction covering 4 whole accumulator rows --
//    instead of a 64-lane reduction per splat, or the reference's 9 atomics per contributing
//    (splat, pixel) pair.
//
// Two translation units: GSR_RENDER_PART 1 = the backward (this file, built with the SLP
// vectorizer), 2 = the forward, schedule and activation kernels (gsr_render_fwd.hip, built
// without it: its scalar code runs 6 % faster unpaired, profiles/r05_slp_ab.txt); 0 = both.
#ifndef GSR_RENDER_PART
#define GSR_RENDER_PART 0
#endif
#include "gsr_device.h"
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = kTilePix;  // 256

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
                                                   uint32_t ntiles, uint32_t* __restrict__ order) {
  __shared__ uint32_t cnt[33];
  __shared__ uint32_t off[33];
  if (threadIdx.x < 33) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ntiles; t += kSchedThreads) {
    const uint32_t w = ranges[t].y - ranges[t].x;
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
    const uint32_t w = ranges[t].y - ranges[t].x;
    const uint32_t bkt = 32u - (uint32_t)__clz((int)w);
    order[atomicAdd(&off[32 - bkt], 1u)] = t;
  }
}

__global__ __launch_bounds__(kSchedThreads) void tile_schedule_kernel(const uint2* __restrict__ ranges,
                                                                      uint32_t ntiles,
                                                                      uint32_t* __restrict__ order) {
  tile_schedule_body(ranges, ntiles, order);
}

struct SchedViews {
  const uint2* ranges[kMaxBatchViews];
  uint32_t* order[kMaxBatchViews];
  uint32_t ntiles[kMaxBatchViews];
};
__global__ __launch_bounds__(kSchedThreads) void tile_schedule_views_kernel(SchedViews m) {
  const int k = (int)blockIdx.x;  // one workgroup per view
  tile_schedule_body(m.ranges[k], m.ntiles[k], m.order[k]);
}

// Backward lane -> pixel map: wave w owns the 8x8 quadrant (w & 1, w >> 1), lane l the pixel
// (l & 7, l >> 3) of it (squares hug the mostly round splat footprints better than 4x16 strips).
__device__ __forceinline__ void pixel_of(uint32_t tx, uint32_t ty, uint32_t t, uint32_t& px,
                                         uint32_t& py) {
  const uint32_t w = t >> 6, l = t & 63u;
  px = tx * kTile + (w & 1u) * 8u + (l & 7u);
  py = ty * kTile + (w >> 1) * 8u + (l >> 3);
}

// Which of the 4 quadrants a splat can reach: bit w set unless the band form of the cut
// (gsr_device.h BandCut) proves alpha < 1/255 on all 64 pixels of quadrant w (the quadrants'
// 8-row bands, each quadrant an interval overlap).
__device__ __forceinline__ uint32_t wave_mask(float4 r0, float4 r1, float qc, uint32_t tx,
                                              uint32_t ty) {
  const BandCut s = make_band_cut_fast(r0.x, r0.y, r0.z, r0.w, r1.x, qc);
  if (s.mode == 0) return 0u;
  if (s.mode == 1) return 0xfu;
  const float xa = (float)(tx * kTile) - s.mx;
  uint32_t m = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const float y0 = (float)(ty * kTile + 8u * (uint32_t)h);
    float xl, xr;
    if (!band_extent(s, y0, y0 + 7.0f, xl, xr)) continue;
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const float x0 = xa + 8.0f * (float)c;
      m |= (xl <= x0 + 7.0f && xr >= x0) ? (1u << (2 * h + c)) : 0u;
    }
  }
  return m;
}

// The backward's finer form: bit 2 w + h for half h (pixel rows 4 h .. 4 h + 3) of quadrant w, for
// the quadrants w0, w0 + 1 (one row of quadrants: two 4-row bands of the tile); the ellipse's
// x-extent in each band is found once and each (quadrant, half) is an interval overlap.
__device__ __forceinline__ uint32_t half_mask_bands(float4 r0, float4 r1, float qc, uint32_t tx,
                                                    uint32_t ty, int w0) {
  const BandCut s = make_band_cut_fast(r0.x, r0.y, r0.z, r0.w, r1.x, qc);
  if (s.mode == 0) return 0u;
  if (s.mode == 1) return 0xffu;
  // the band rows and column starts are re-derived here for each batch: the backend would hoist
  // them out of the batch loop and spill them (the backward runs at its 128-VGPR cap)
  asm volatile("" : "+v"(tx), "+v"(ty));
  const float xa = (float)(tx * kTile) - s.mx;  // the tile's first pixel column, relative
  uint32_t m = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const float y0 = (float)(ty * kTile + (uint32_t)(w0 >> 1) * 8u + (uint32_t)h * 4u);
    float xl, xr;
    if (!band_extent(s, y0, y0 + 3.0f, xl, xr)) continue;
#pragma unroll
    for (int wi = 0; wi < 2; wi++) {
      const int w = w0 + wi;
      const float x0 = xa + (float)((w & 1) * 8);
      m |= (xl <= x0 + 7.0f && xr >= x0) ? (1u << (2 * w + h)) : 0u;
    }
  }
  return m;
}

// Per-wave compaction of the batch: the list holds, in batch order, the entries whose mask has
// bit `bit` and whose list position base - j lies before `lim` (the largest n_contrib of the
// pixels the list serves: entries behind it contribute nowhere).  Returns the list length
// (wave-uniform).
template <int N>
__device__ __forceinline__ uint32_t build_wave_list(const uint8_t* s_mask, uint8_t* list,
                                                    uint32_t cnt, int bit_idx, int lane,
                                                    uint32_t base = 0u, uint32_t lim = ~0u) {
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t n = 0;
#pragma unroll
  for (int c = 0; c < N / 64; c++) {
    const uint32_t j = (uint32_t)(c * 64 + lane);
    const bool bit = j < cnt && ((s_mask[j] >> bit_idx) & 1u) && base - j < lim;
    const uint64_t b = __ballot(bit);
    if (bit) list[n + (uint32_t)__popcll(b & lt)] = (uint8_t)j;
    n += (uint32_t)__popcll(b);
  }
  return n;
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
template <int CTRL>
__device__ __forceinline__ uint32_t dppu(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}
// DPP controls: quad_perm (lane i of each quad takes lane p_i), row_half_mirror (lane i of each
// 8-lane half row takes lane 7 - i), row_ror:8
constexpr int kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppHalfMirror = 0x141;
constexpr int kDppQuadBcast0 = 0x00, kDppQuadBcast1 = 0x55, kDppQuadBcast2 = 0xAA, kDppQuadBcast3 = 0xFF;

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

// p + partner: permlane32_swap pairs lane l with l ^ 32, permlane16_swap with l ^ 16 (inside each
// 32-lane half); afterwards one half holds the sum of the p's, the other the sum of the q's
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

#if GSR_RENDER_PART != 2
// ================================================================================================
// Backward blend.
//
// Per (pixel, contributing splat) pair the reference (backward.cu:482-555) recovers T, runs the
// dL/dalpha recurrence and adds nine per-pair terms to the splat's gradients.  The terms here are
// the moments of u = G dL/dalpha -- (u dx, u dy, u dx dx, u dx dy, u dy dy, u) with (dx, dy) the
// splat centre minus the pixel -- and w dpix_c for the channels c with w = alpha T; the per-splat
// constants (conic a, b, c, opacity o, W/2, H/2) turn the moments into the reference's dL/dmean2D
// and dL/dconic once per (splat, tile):
//   dL/dmean2D.x = -(W/2) o (a sum u dx + b sum u dy),  dL/dmean2D.y = -(H/2) o (c sum u dy + b sum u dx)
//   dL/dconic.{x,y,w} = -1/2 o sum u {dx dx, dx dy, dy dy},   dL/dopacity = sum u
// (linear, so exact up to float rounding).
//
// Phase 1, lanes = pixels.  The wave replays its quadrant list back to front; for each entry with
// a contributing lane every lane runs the recurrence (non-contributing lanes with G = alpha = 0,
// which leaves T and the state unchanged and makes u = w = 0) and stores its (u, w) into the next
// of kSlots LDS slots (64 pairs, 512 contiguous bytes).
// Phase 2, lanes = (slot j = l & 7, pixel row s = l >> 3), run whenever the slots are full and at
// the end of a batch: each lane sums its slot's 8 pixels of row s -- (u, w) from the slots, the
// pixels' upstream gradients from a per-wave LDS table -- into 13 registers (dy is constant along
// the row, so sum u dy = dy sum u etc.), then a 3-stage halving butterfly over the 8 rows (lane
// bits 5, 4, 3) leaves each lane one (value pair) of its slot, added into the batch's LDS row.
// Per contributing (wave, entry): ~40 VALU in phase 1 and ~12 in phase 2, against ~105 for the
// per-entry 64-lane butterfly this replaces.
// ================================================================================================
#ifndef GSR_BWD_HALF
#define GSR_BWD_HALF 1
#endif
// Batch (records staged per batch) and phase-2 width (slots summed per pass; phase-2 lanes
// j = l & 7): the default backward flushes each wave's sums straight to the accumulator rows
// (128 records, 8 slots); the deterministic one keeps wave-private LDS rows for the ordered
// per-instance store (64 records and 7 slots so that they fit 4 workgroups per CU)
template <bool DET> struct BwdShape {
  static constexpr int kBatch = DET ? 64 : 128;
  static constexpr int kSlots = DET ? 7 : 8;
};
constexpr int kAccRow = 13;          // LDS accumulator row: the 13 gradient values (odd: conflict-free)
// phase-2 slot stride in dwords: 64 (u, w) pairs + 2 pad dwords, so the eight slots of a phase-2
// read start on banks 2j (ds_read_b64: 32 lanes x 2 banks, all distinct)
constexpr int kUwStride = 130;
// per-wave table of the pixels' upstream gradients: 8 rows of 8 pixels x 8 floats
// {r, g, b, depth}, {f0, f1, f2, 0}; rows padded by 4 dwords so the rows read in one phase-2 step
// fall on different banks (ds_read_b128: row s at bank 4 s + 8 t, conflict-free)
constexpr int kDpRow = 68;

template <bool EXTRA, bool FEAT, bool DET>
__device__ __forceinline__ void render_bwd_tile(const RenderBwdArgs& a, uint32_t blk) {
  constexpr bool ROWS = DET;  // the deterministic backward stores per-instance rows
  // HALF: the two halves of a quadrant (pixel rows 0-3 = lanes 0-31, rows 4-7 = lanes 32-63) walk
  // their own lists, so one phase-1 step replays a splat for each half; the deterministic
  // backward keeps one list per quadrant (its per-(wave, entry) rows)
  constexpr bool HALF = !DET && GSR_BWD_HALF;
  constexpr int kBatch = BwdShape<DET>::kBatch, kSlots = BwdShape<DET>::kSlots;
  // list entries per test-phase group: 2 in the default backward (106 VGPRs instead of 126 for 4,
  // which pays for phase 2's four-pixel read batches), 4 in the deterministic one
  constexpr int kGrp = DET ? 4 : 2;
  // the batch's records, regrouped for the test phase: s_r0 = {x, y, conic.a, conic.c} (the
  // packed pairs of the power), s_r1 = {conic.b, opacity}, s_c0 = {r, g, b, depth},
  // s_c1 = {f0, f1, f2, 1} (alpha channel)
  __shared__ float4 s_r0[kBatch];
  __shared__ float2 s_r1[kBatch];
  __shared__ float4 s_c0[kBatch];
  __shared__ float4 s_c1[FEAT ? kBatch : 1];
  __shared__ uint32_t s_gid[kBatch];
  // DET: per batch entry and wave its 13 gradient values, stored and summed over the waves in
  // wave order (the default backward flushes from phase 2 and needs none: LDS float atomics cost
  // ~1 cycle per active lane, profiles/r05_bwd_ab.txt)
  __shared__ float s_acc[DET ? 4 * kBatch * kAccRow : 1];
  __shared__ uint8_t s_mask[kBatch];
  // HALF: the mask bits of quadrants 2 and 3, computed by the workgroup's upper half
  __shared__ uint8_t s_mask23[HALF ? kBatch : 1];
  __shared__ uint8_t s_list[kThreads / 64][HALF ? 2 : 1][kBatch];
  __shared__ __attribute__((aligned(16))) float s_uw[kThreads / 64][kSlots * kUwStride];
  __shared__ __attribute__((aligned(16))) float s_dp[kThreads / 64][8 * kDpRow];

  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);
  const int half = HALF ? (lane >> 5) : 0;
  const SwapOrient swap_orient = probe_swaps(lane);
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
  if (a.status && (*a.status & (kStatusDepthSort | kStatusTileSort))) return;
  const uint2 range = a.ranges[tile];
  // every loop trip count of this kernel is bounded by the tile's list: the
  // forward's largest n_contrib cannot exceed it, the min() makes that hold for any buffer
  const uint32_t tile_last = min(a.tile_last[tile], range.y - min(range.x, range.y));
  const float T_final = inside ? a.final_T[pix] : 0.0f;
  float T = T_final;
  const uint32_t last_contributor = inside ? a.n_contrib[pix] : 0u;
  // the largest n_contrib of the wave (HALF: of the lane's half)
  uint32_t wave_last = last_contributor;
#pragma unroll
  for (int d = HALF ? 16 : 32; d >= 1; d >>= 1)
    wave_last = max(wave_last, (uint32_t)__shfl_xor((int)wave_last, d, 64));

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
                kAccF0 == 10 && kAccF1 == 11 && kAccF2 == 12, "slot layout of the gradient row");
  // this wave's pixel table for phase 2: lane l = pixel (l & 7, l >> 3) of the quadrant
  {
    float* d = &s_dp[wid][(lane >> 3) * kDpRow + (lane & 7) * 8];
    *reinterpret_cast<float4*>(d) = make_float4(dpA.x, dpA.y, dpB.x, dpB.y);
    *reinterpret_cast<float4*>(d + 4) = make_float4(dpC.x, dpC.y, dpD.x, 0.0f);
  }
  float acc_dot = 0.0f, last_cdot = 0.0f;
  float last_alpha = 0.0f;
  const float ddelx_dx = (float)(0.5 * a.W);
  const float ddely_dy = (float)(0.5 * a.H);
  // the quadrant's first pixel: phase 2 forms each pixel's (dx, dy) as phase 1 does,
  // splat centre minus (float)pixel, so the two phases see the same offsets
  const uint32_t qx0 = tx * kTile + (uint32_t)(wid & 1) * 8u;
  const float pfy_row = (float)(ty * kTile + (uint32_t)(wid >> 1) * 8u + (uint32_t)(lane >> 3));

  if (DET)
    for (int k = (int)threadIdx.x; k < 4 * kBatch * kAccRow; k += kThreads) s_acc[k] = 0.0f;

  // Phase 2 over the first `ns` slots (wave-uniform, 1..kSlots).  slotv: lane l holds the batch
  // index of slot l & 7 (set in phase 1, no LDS round trip).
  auto phase2 = [&](uint32_t ns, uint32_t slotv) {
    const int j = lane & 7;
    const uint32_t bj = slotv & (uint32_t)(kBatch - 1);  // stale for j >= ns: kept in range
    const float4 r0 = s_r0[bj];
    const float dy = r0.y - pfy_row;
    const float* uw = &s_uw[wid][j * kUwStride + (lane >> 3) * 16];
    const float* dp = &s_dp[wid][(lane >> 3) * kDpRow];
    float su = 0.f, sux = 0.f, suxx = 0.f;
    f2 cA = mk2(0.f, 0.f), cB = mk2(0.f, 0.f), cC = mk2(0.f, 0.f), cD = mk2(0.f, 0.f);
    // The row's reads in batches of four pixels (two in the deterministic backward), each
    // batch's reads issued together before its arithmetic (sched_barrier: the backend otherwise
    // interleaves them one pixel at a time, one LDS round trip per pixel).  Batches of 4 fit the
    // 128-VGPR budget since the test phase groups 2 entries instead of 4 (round 6: 125 VGPRs,
    // render_bwd -1.3 %, profiles/r06_bwd_ablation.txt; with 4-entry groups they needed 142 VGPRs,
    // 3 waves per SIMD, profiles/r05_bwd_ab.txt)
    constexpr int kB = DET ? 2 : 4;
#pragma unroll
    for (int t0 = 0; t0 < 8; t0 += kB) {
      f2 p[kB];
      float4 d0[kB], d1[kB];
#pragma unroll
      for (int t = 0; t < kB; t++) {
        // one ds_read_b64 per pixel (2 LDS cycles, conflict-free at kUwStride): the opaque
        // offset keeps the backend from pairing two of them into a ds_read2_b64 (8 cycles)
        uint32_t off = (uint32_t)(2 * (t0 + t));
        asm volatile("" : "+v"(off));
        p[t] = *reinterpret_cast<const f2*>(uw + off);  // (u, w) of pixel (t0 + t, row)
        // both halves of the pixel's table entry as ds_read_b128 (4 cycles each; a 12-byte
        // read of the second half would be a ds_read_b96, 8 cycles)
        d0[t] = *reinterpret_cast<const float4*>(dp + 8 * (t0 + t));
        if (FEAT) d1[t] = *reinterpret_cast<const float4*>(dp + 8 * (t0 + t) + 4);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < kB; t++) {
        const float dx = r0.x - (float)(qx0 + (uint32_t)(t0 + t));
        su += p[t].x;
        const float ux = p[t].x * dx;
        sux += ux;
        suxx = __builtin_fmaf(ux, dx, suxx);
        cA = fma2(mk2(p[t].y, p[t].y), mk2(d0[t].x, d0[t].y), cA);
        cB = fma2(mk2(p[t].y, p[t].y), mk2(d0[t].z, NC > 3 ? d0[t].w : 0.f), cB);
        if (FEAT) {
          cC = fma2(mk2(p[t].y, p[t].y), mk2(d1[t].x, d1[t].y), cC);
          cD = fma2(mk2(p[t].y, p[t].y), mk2(d1[t].z, d1[t].w), cD);  // d1.w = 0
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the 16 slots of the row as 8 pairs (slot order of kAcc*): (sum u dx, sum u dy),
    // (sum u dx dx, sum u dx dy), (sum u dy dy, sum u), (r, g), (b, depth), (f0, f1), (f2, -), -
    f2 v[8];
    v[0] = mk2(sux, dy * su);
    v[1] = mk2(suxx, dy * sux);
    v[2] = mk2((dy * dy) * su, su);
    v[3] = cA;
    v[4] = cB;
    v[5] = cC;
    v[6] = cD;
    v[7] = mk2(0.f, 0.f);
    if (HALF) {
      // rows 0-3 and 4-7 (lane bit 5) are different splats: halving butterfly over the 4 rows of
      // each half, lane bit 4 (permlane16_swap), bit 3 (DPP row_ror:8); each lane is left with the
      // two pairs 2 m, 2 m + 1 of its slot and half, m = b3 + 2 b4' -- the 4 consecutive values
      // 4 m .. 4 m + 3 of the gradient row
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = swap16_add(v[i], v[i + 4]);
      f2 w2[2];
      const bool hi = lane & 8;
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const f2 send = hi ? v[i] : v[i + 2];
        const f2 keep = hi ? v[i + 2] : v[i];
        w2[i] = keep + mk2(dpp<0x128>(send.x), dpp<0x128>(send.y));  // row_ror:8
      }
      const int m = ((lane >> 3) & 1) + 2 * (((lane >> 4) & 1) ^ (int)swap_orient.flip16);
      // this wave-half's sums of the splat -> the reference's dL/dmean2D (NDC-scaled) and
      // dL/dconic (linear in the moments: partial sums convert exactly up to rounding)
      float g[4];
      {
        const float2 r1 = s_r1[bj];
        const float o = r1.y, nho = -0.5f * o;
        const f2 p0 = w2[0], p1 = w2[1];
        const bool m0 = m == 0;
        g[0] = m0 ? -(o * (r0.z * p0.x + r1.x * p0.y)) * ddelx_dx : (m == 1 ? nho * p0.x : p0.x);
        g[1] = m0 ? -(o * (r0.w * p0.y + r1.x * p0.x)) * ddely_dy : p0.y;
        g[2] = m0 ? nho * p1.x : p1.x;
        g[3] = m0 ? nho * p1.y : p1.y;
      }
      // one global float atomic per value into the splat's accumulator row.  Float atomics cost
      // per 64-B line a wave-instruction touches, so the values are first transposed inside each
      // quad (lanes q = slot bits 0-1): lane q's register k (slot q, value 4 m + k) moves to lane
      // k's register q, and atomic instruction r then covers 4 whole rows (slots 4 b + r of both
      // halves) instead of values of 16 rows
      uint32_t gid = ((uint32_t)j < ns && slotv < (uint32_t)kBatch) ? s_gid[bj] : 0xffffffffu;
      const int q = lane & 3;
#pragma unroll
      for (int i = 0; i < 2; i++) {  // lane bit 1 <-> register bit 1
        const bool b1 = q & 2;
        const float recv = dpp<kDppQuadXor2>(b1 ? g[i] : g[i + 2]);
        g[i] = b1 ? recv : g[i];
        g[i + 2] = b1 ? g[i + 2] : recv;
      }
#pragma unroll
      for (int i = 0; i < 4; i += 2) {  // lane bit 0 <-> register bit 0
        const bool b0 = q & 1;
        const float recv = dpp<kDppQuadXor1>(b0 ? g[i] : g[i + 1]);
        g[i] = b0 ? recv : g[i];
        g[i + 1] = b0 ? g[i + 1] : recv;
      }
      const int k = 4 * m + q;  // the value every register of this lane now holds
      // register r's row: slot r of the quad (DPP quad broadcast of lane r's id)
      const uint32_t gr[4] = {dppu<kDppQuadBcast0>(gid), dppu<kDppQuadBcast1>(gid),
                              dppu<kDppQuadBcast2>(gid), dppu<kDppQuadBcast3>(gid)};
      if (k < kAccRow) {
#pragma unroll
        for (int r = 0; r < 4; r++)
          if (gr[r] != 0xffffffffu && g[r] != 0.0f) {
            atomicAdd(a.acc + (size_t)gr[r] * kAccFloats + k, g[r]);
          }
      }
      return;
    }
    // halving butterfly over the 8 rows: lane bit 5 (permlane32_swap), bit 4 (permlane16_swap),
    // bit 3 (DPP row_ror:8 swaps the halves of a 16-lane row)
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = swap32_add(v[i], v[i + 4]);
#pragma unroll
    for (int i = 0; i < 2; i++) v[i] = swap16_add(v[i], v[i + 2]);
    f2 w;
    {
      const bool hi = lane & 8;
      const f2 send = hi ? v[0] : v[1];
      const f2 keep = hi ? v[1] : v[0];
      w = keep + mk2(dpp<0x128>(send.x), dpp<0x128>(send.y));  // row_ror:8
    }
    // pair index held: b3 + 2 b4' + 4 b5' (b4', b5' corrected by the probed swap orientation)
    const int pr = ((lane >> 3) & 1) + 2 * (((lane >> 4) & 1) ^ (int)swap_orient.flip16) +
                   4 * (((lane >> 5) & 1) ^ (int)swap_orient.flip32);
    if (DET) {
      if ((uint32_t)j < ns) {
        // a batch entry is in a wave's list at most once: its row of this wave is written once
        const int k0 = 2 * pr;
        float* row = &s_acc[(wid * kBatch + bj) * kAccRow];
        if (k0 < kAccRow) row[k0] = w.x;
        if (k0 + 1 < kAccRow) row[k0 + 1] = w.y;
      }
    } else {
      // this wave's sums of the splat -> the reference's dL/dmean2D (NDC-scaled), dL/dconic
      // (linear in the moments, so per-wave partial sums convert exactly up to rounding), then
      // one global float atomic per value into the splat's accumulator row
      const float2 r1 = s_r1[bj];
      const float o = r1.y, nho = -0.5f * o;
      f2 g;
      g.x = pr == 0 ? -(o * (r0.z * w.x + r1.x * w.y)) * ddelx_dx : (pr <= 2 ? nho * w.x : w.x);
      g.y = pr == 0 ? -(o * (r0.w * w.y + r1.x * w.x)) * ddely_dy : (pr == 1 ? nho * w.y : w.y);
      // float atomics cost per 64-B line a wave-instruction touches: slots j and 7 - j swap one
      // value (DPP row_half_mirror), so each of the two atomic instructions covers 4 whole rows
      // (slots 0-3 / 4-7) instead of one value pair of all 8
      const uint32_t gid = (uint32_t)j < ns ? s_gid[bj] : 0xffffffffu;
      const bool lo = j < 4;
      const float recv = dpp<kDppHalfMirror>(lo ? g.y : g.x);
      const uint32_t gp = dppu<kDppHalfMirror>(gid);
      const int k = 2 * pr + (lo ? 0 : 1);
      const float ax = lo ? g.x : recv, ay = lo ? recv : g.y;
      const uint32_t ga = lo ? gid : gp, gb = lo ? gp : gid;
      if (k < kAccRow) {
        if (ga != 0xffffffffu && ax != 0.0f) atomicAdd(a.acc + (size_t)ga * kAccFloats + k, ax);
        if (gb != 0xffffffffu && ay != 0.0f) atomicAdd(a.acc + (size_t)gb * kAccFloats + k, ay);
      }
    }
  };

  // rel = position inside the tile's list; every pixel only uses rel < its n_contrib <= tile_last
  // staging lanes: sj = the batch slot this thread stages (HALF: both halves of the workgroup
  // take the batch's records, the lower half staging them and the quadrant-0/1 mask bits, the
  // upper half the quadrant-2/3 bits); its list entry is loaded one batch ahead
  static_assert(!HALF || kThreads == 2 * kBatch, "HALF staging: two threads per record");
  const uint32_t sj = HALF ? (threadIdx.x & (uint32_t)(kBatch - 1)) : threadIdx.x;
  const bool upper = HALF && threadIdx.x >= (uint32_t)kBatch;  // wave-uniform
  uint32_t pid_next = sj < min((uint32_t)kBatch, tile_last) ? a.point_list[range.x + tile_last - 1 - sj] : 0u;
  for (uint32_t done_cnt = 0; done_cnt < tile_last; done_cnt += kBatch) {
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kBatch, tile_last - done_cnt);
    // stage the batch starting at list position done_cnt (back to front)
    if (sj < cnt) {
      const uint32_t gid = min(pid_next, a.P - 1u);
      const float4* rec = a.rec + 4 * (size_t)gid;
      if (!upper) {
        s_gid[sj] = gid;
        const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2], q3 = rec[3];
        s_r0[sj] = make_float4(q0.x, q0.y, q0.z, q1.x);
        s_r1[sj] = make_float2(q0.w, q1.y);
        s_mask[sj] = (uint8_t)(HALF ? half_mask_bands(q0, q1, q3.z, tx, ty, 0)
                                    : wave_mask(q0, q1, q3.z, tx, ty));
        s_c0[sj] = make_float4(q1.w, q2.x, q2.y, q1.z);
        if (FEAT) s_c1[sj] = make_float4(q2.z, q2.w, q3.x, 1.0f);
      } else {
        const float4 q0 = rec[0], q1 = rec[1], q3 = rec[3];
        s_mask23[sj] = (uint8_t)half_mask_bands(q0, q1, q3.z, tx, ty, 2);
      }
    }
    {  // the next batch's list entries, in flight while this batch is replayed
      const uint32_t nd = done_cnt + kBatch;
      if (sj < min((uint32_t)kBatch, tile_last - min(nd, tile_last)))
        pid_next = a.point_list[range.x + tile_last - 1 - nd - sj];
    }
    __syncthreads();
    // nlist: the wave's step count; nmine: the length of the lane's own list (HALF: its half's)
    // (entries behind the list's pixels' last contributor are left out)
    uint32_t nlist, nmine;
    const uint32_t base = tile_last - 1 - done_cnt;
    if (HALF) {
      const uint8_t* msk = wid < 2 ? s_mask : s_mask23;
      const uint32_t n0 = build_wave_list<kBatch>(msk, s_list[wid][0], cnt, 2 * wid, lane, base,
                                                  (uint32_t)__builtin_amdgcn_readlane((int)wave_last, 0));
      const uint32_t n1 = build_wave_list<kBatch>(msk, s_list[wid][HALF ? 1 : 0], cnt,
                                                  2 * wid + 1, lane, base,
                                                  (uint32_t)__builtin_amdgcn_readlane((int)wave_last, 32));
      nmine = half ? n1 : n0;
      nlist = max(n0, n1);
    } else {
      nlist = build_wave_list<kBatch>(s_mask, s_list[wid][0], cnt, wid, lane, base,
                                      (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_last));
      nmine = nlist;
    }
    uint32_t ns = 0;     // phase-2 slots in use (wave-uniform)
    // lane l: batch index of phase-2 slot l & 7 (HALF: of the lane's half; >= kBatch when that
    // half had no contributing pixel at that step)
    uint32_t slotv = 0;
    // Four list entries per group: the per-pair test (power, G, alpha) of all four is evaluated
    // first (independent work), then the entries are replayed in list order.
    for (uint32_t k0 = 0; k0 < nlist; k0 += kGrp) {
      const uint32_t packed = kGrp == 4 ? *reinterpret_cast<const uint32_t*>(&s_list[wid][half][k0])
                                        : (uint32_t)*reinterpret_cast<const uint16_t*>(&s_list[wid][half][k0]);
      // Every LDS read of the group's entries is issued here, before any arithmetic; the colours
      // are consumed at once by the colour dot product, so the replay below reads no records.
      float Gv[kGrp], av[kGrp], cdv[kGrp];
      bool cv[kGrp];
      {
        float4 r0v[kGrp], c0v[kGrp], c1v[kGrp];
        float2 r1v[kGrp];
#pragma unroll
        for (int u = 0; u < kGrp; u++) {
          // (entries past the list's end hold stale bytes: kept inside the batch)
          const uint32_t j = (packed >> (8 * u)) & (uint32_t)(kBatch - 1);
          r0v[u] = s_r0[j];
          r1v[u] = s_r1[j];
          c0v[u] = s_c0[j];
          if (FEAT) c1v[u] = s_c1[j];
        }
        float pw[kGrp];
        float tdist = 1.0f;  // min over the group of |op * G - 1/255| (the exact-path test)
#pragma unroll
        for (int u = 0; u < kGrp; u++) {
          // the reference's -0.5 (ca dx dx + cc dy dy) - cb dx dy, the pairs as packed products
          // (same operations, same order)
          const float4 r0 = r0v[u];
          const float dx = r0.x - pfx, dy = r0.y - pfy;
          pw[u] = -0.5f * (r0.z * dx * dx + r0.w * dy * dy) - r1v[u].x * dx * dy;
          // The backward needs the forward's alpha >= 1/255 DECISION exactly, its G only to
          // gradient precision: G by the hardware exp2 (v_exp_f32, ~1 ulp; 3 instructions
          // instead of the 17 of splat_exp), and splat_exp -- the forward's and the oracle's
          // sequence -- wherever op * G lies within 2e-6 (relative) of 1/255, so the decision is
          // the forward's at every pixel.  The exact path is one wave-uniform branch per group.
          Gv[u] = __builtin_amdgcn_exp2f(pw[u] * 1.44269504088896341f);
          {
            const float d = fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f));
            tdist = d < tdist ? d : tdist;
          }
          // cdot = sum_c col_c * dpix_c as packed FMAs over the colour pairs (gradient-only
          // arithmetic: the forward-consistent quantities G, alpha, T are computed unfused)
          const float4 c0 = c0v[u];
          f2 c2 = mk2(c0.x, c0.y) * dpA;
          c2 = fma2(mk2(c0.z, NC > 3 ? c0.w : 0.f), dpB, c2);
          if (FEAT) c2 = fma2(mk2(c1v[u].x, c1v[u].y), dpC, c2);
          // (FEAT: c1.w holds the alpha channel's 1, read so that the record is one ds_read_b128
          // rather than a ds_read_b96 at twice the LDS cycles)
          if (NC > 3) c2 = fma2(FEAT ? mk2(c1v[u].z, c1v[u].w) : mk2(0.f, 1.0f), dpD, c2);
          cdv[u] = c2.x + c2.y;
          // keep the dot product here (the compiler would sink it into the contributing branch
          // and hold the colours live across the test phase)
          asm volatile("" ::"v"(cdv[u]));
        }
        if (__ballot(tdist <= 2e-6f * (1.0f / 255.0f))) {
#pragma unroll
          for (int u = 0; u < kGrp; u++) {
            if (fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f))
              Gv[u] = splat_exp(pw[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < kGrp; u++) {
          const uint32_t j = (packed >> (8 * u)) & (uint32_t)(kBatch - 1);
          const uint32_t rel = tile_last - 1 - done_cnt - j;
          av[u] = fminf(0.99f, r1v[u].y * Gv[u]);
          cv[u] = (k0 + u < nmine) && rel < last_contributor && !(pw[u] > 0.0f) &&
                  !(av[u] < 1.0f / 255.0f);
        }
      }
#pragma unroll
      for (int u = 0; u < kGrp; u++) {
        const bool contrib = cv[u];
        // wave-uniform skip of entries without a contributing lane
        const uint64_t bal = __ballot(contrib);
        if (bal == 0ull) continue;
        const uint32_t j = (packed >> (8 * u)) & (uint32_t)(kBatch - 1);
        // Branch-free: a lane whose pixel does not take this splat runs the same arithmetic with
        // G = alpha = 0, which makes u and w exactly zero and T / (1 - 0) == T; its recurrence
        // state is kept by selects.  Contributing lanes compute exactly the operations of the
        // reference (backward.cu:486-534).
        const float G = contrib ? Gv[u] : 0.0f;
        const float alpha = contrib ? av[u] : 0.0f;
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
        const float wgt = alpha * T;  // dchannel_dcolor (backward.cu:500)
        const float cdot = cdv[u];
        const float acc_new = last_alpha * last_cdot + (1.f - last_alpha) * acc_dot;
        float dL_dalpha = cdot - acc_new;
        acc_dot = contrib ? acc_new : acc_dot;
        last_cdot = contrib ? cdot : last_cdot;
        last_alpha = contrib ? alpha : last_alpha;
        dL_dalpha *= T;
        if (has_bg) dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
        const float uu = G * dL_dalpha;
        // park (u, w) in the next phase-2 slot
        *reinterpret_cast<f2*>(&s_uw[wid][ns * kUwStride + 2 * lane]) = mk2(uu, wgt);
        if (HALF) {
          // the lanes of a half with a contributing pixel, as a scalar lane mask, selects the
          // entry or "no slot" in one v_cndmask (the per-lane form costs ~5 VALU per step)
          constexpr uint64_t kLo = 0x00000000ffffffffull;
          const uint64_t hm = (((uint32_t)bal != 0u) ? kLo : 0ull) |
                              (((uint32_t)(bal >> 32) != 0u) ? ~kLo : 0ull);
          uint32_t jv;
          asm("v_cndmask_b32_e64 %0, -1, %1, %2" : "=v"(jv) : "v"(j), "s"(hm));
          slotv = ((uint32_t)(lane & 7) == ns) ? jv : slotv;
        } else {
          slotv = ((uint32_t)(lane & 7) == ns) ? j : slotv;
        }
        ns = (uint32_t)__builtin_amdgcn_readfirstlane((int)(ns + 1));
        if (ns == (uint32_t)kSlots) {
          phase2(ns, slotv);
          ns = 0;
        }
      }
    }
    if (ns) phase2(ns, slotv);
    if (!DET) continue;  // flushed from phase 2; the next batch's first barrier protects the records
    __syncthreads();
    // moments -> the reference's dL/dmean2D (NDC-scaled) and dL/dconic, once per (splat, tile)
    if (threadIdx.x < cnt) {
      const float4 r0 = s_r0[threadIdx.x];
      const float2 r1 = s_r1[threadIdx.x];
      float* row = s_acc + threadIdx.x * kAccRow;
      // the four waves' rows, added in wave order, into wave 0's row
#pragma unroll
      for (int k = 0; k < kAccRow; k++)
        row[k] = ((row[k] + row[kBatch * kAccRow + k]) + row[2 * kBatch * kAccRow + k]) +
                 row[3 * kBatch * kAccRow + k];
      const float sx = row[kAccMx], sy = row[kAccMy];
      const float o = r1.y;
      row[kAccMx] = -(o * (r0.z * sx + r1.x * sy)) * ddelx_dx;
      row[kAccMy] = -(o * (r0.w * sy + r1.x * sx)) * ddely_dy;
      row[kAccCa] = (-0.5f * o) * row[kAccCa];
      row[kAccCb] = (-0.5f * o) * row[kAccCb];
      row[kAccCc] = (-0.5f * o) * row[kAccCc];
    }
    __syncthreads();
    // flush: lane l of wave-instruction `it` handles splat (it*16 + tid/16), slot tid%16
#pragma unroll 1
    for (int it = 0; it < kBatch * kAccFloats / kThreads; it++) {
      const uint32_t jj = (uint32_t)it * (kThreads / kAccFloats) + (threadIdx.x >> 4);
      const int k = (int)(threadIdx.x & 15);
      if (jj < cnt) {
        const bool held = k < kAccRow;
        if (ROWS) {  // every slot stored (16 lanes = one 64-B row), then re-zeroed
          const uint32_t q = range.x + tile_last - 1 - done_cnt - jj;
          const float v = held ? s_acc[jj * kAccRow + k] : 0.0f;
          a.partial[(size_t)min(a.einst[q], a.nrows - 1u) * kAccFloats + k] = v;
          if (held)
#pragma unroll
            for (int w = 0; w < 4; w++) s_acc[(w * kBatch + jj) * kAccRow + k] = 0.0f;
        } else {
          const float v = held ? s_acc[jj * kAccRow + k] : 0.0f;
          if (v != 0.0f) atomicAdd(&a.acc[(size_t)s_gid[jj] * kAccFloats + k], v);
          if (held)
#pragma unroll
            for (int w = 0; w < 4; w++) s_acc[(w * kBatch + jj) * kAccRow + k] = 0.0f;
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

// waves per SIMD the backward is compiled for (its LDS holds 4 workgroups per CU)
#ifndef GSR_BWD_MIN_WAVES
#define GSR_BWD_MIN_WAVES 4
#endif
#define GSR_BWD_WAVES(DET) __attribute__((amdgpu_waves_per_eu((DET) ? 1 : GSR_BWD_MIN_WAVES)))

template <bool EXTRA, bool FEAT, bool DET>
__global__ __launch_bounds__(kThreads) GSR_BWD_WAVES(DET) void render_bwd_kernel(RenderBwdArgs a) {
  render_bwd_tile<EXTRA, FEAT, DET>(a, blockIdx.x);
}

// The backward blends of several views of a step in ONE launch: workgroup b belongs to the view k
// with first[k] <= b < first[k + 1] (view-major; inside a view the forward's heaviest-first tile
// order), so the views' launches do not each end in a tail of idle CUs, and one launch's duration
// is the time of all its views' blends.
template <bool EXTRA, bool FEAT, bool DET>
__global__ __launch_bounds__(kThreads) GSR_BWD_WAVES(DET) void render_bwd_views_kernel(RenderBwdViews m) {
  const uint32_t b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.V && b >= m.first[k + 1]) k++;  // workgroup-uniform
  render_bwd_tile<EXTRA, FEAT, DET>(m.v[k], b - m.first[k]);
}

#endif  // GSR_RENDER_PART != 2
#if GSR_RENDER_PART != 1
// ================================================================================================
// Forward with block lists: each wave's 64 lanes are four 16-lane groups, group g = lanes
// 16 g .. 16 g + 15 owning a 4x4 pixel block of the wave's 8x8 quadrant (x = lane & 3,
// y = (lane >> 2) & 3), i.e. exactly one of ds_read_b128's 16-lane groups, so a group's record
// reads are one broadcast address.  Every group walks its OWN compacted list of the batch, so a
// wave step evaluates four (block, splat) entries at once.  Per pixel the blend's operations and
// their order are the reference's (forward.cu:325-362).
// ================================================================================================
__device__ __forceinline__ void pixel_of_blk(uint32_t tx, uint32_t ty, uint32_t t, uint32_t& px,
                                             uint32_t& py) {
  const uint32_t w = t >> 6, l = t & 63u, g = l >> 4;
  px = tx * kTile + (w & 1u) * 8u + (g & 1u) * 4u + (l & 3u);
  py = ty * kTile + (w >> 1) * 8u + (g >> 1) * 4u + ((l >> 2) & 3u);
}

// Which of the 16 4x4 blocks a splat can reach: bit 4w + g for block g of quadrant w (tile column
// 2 (w & 1) + (g & 1), row 2 (w >> 1) + (g >> 1)).  Band form of the cut (gsr_device.h BandCut):
// the x-extent of the margin-widened ellipse in each of the tile's four 4-row bands, each block an
// interval overlap -- exact per block, where the quadrant test AND the ellipse's bounding box kept
// every block of a quadrant that the box met (and cost four rectangle tests).
__device__ __forceinline__ uint32_t block_mask(float4 r0, float4 r1, float qc, uint32_t tx,
                                               uint32_t ty) {
  const BandCut s = make_band_cut_fast(r0.x, r0.y, r0.z, r0.w, r1.x, qc);
  if (s.mode == 0) return 0u;
  if (s.mode == 1) return 0xffffu;
  const float xa = (float)(tx * kTile) - s.mx;  // the tile's first pixel column, relative
  uint32_t bb = 0;
#pragma unroll
  for (int cy = 0; cy < 4; cy++) {
    const float y0 = (float)(ty * kTile + 4u * (uint32_t)cy);
    float xl, xr;
    if (!band_extent(s, y0, y0 + 3.0f, xl, xr)) continue;
#pragma unroll
    for (int cx = 0; cx < 4; cx++) {
      const float x0 = xa + 4.0f * (float)cx;
      const int w = 2 * (cy >> 1) + (cx >> 1), g = 2 * (cy & 1) + (cx & 1);
      bb |= (xl <= x0 + 3.0f && xr >= x0) ? (1u << (4 * w + g)) : 0u;
    }
  }
  return bb;
}

// Per-group compaction: group g's list holds, in batch order, the entries whose mask has bit
// 4 wid + g.  Returns this lane's group's length; `nmax` gets the longest of the wave's four.
// The four lists of a wave sit kListRow bytes apart: a 4-byte pad puts the four groups' list
// reads (one ds_read_b32 per step, four addresses per wave) on four different banks.
constexpr int kListRow = kThreads + 4;
__device__ __forceinline__ uint32_t build_group_lists(const uint16_t* s_mask, uint8_t (*list)[kListRow],
                                                      uint32_t cnt, int wid, int lane, uint32_t grp,
                                                      uint32_t& nmax) {
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
  return grp == 0 ? n[0] : grp == 1 ? n[1] : grp == 2 ? n[2] : n[3];
}

// waves per SIMD the block-list forward is compiled for (VGPR budget 512 / n): 7 (72 VGPRs, no
// scratch) with its 2-entry steps; with 4-entry steps 5 waves (95 VGPRs) was the best (round 4:
// 5 against 4, profiles/r04_fwd_occ_ab.txt).  Round 6: 2-entry steps at 7 waves 0.218 -> 0.204 ms
// per 3-view launch; 1-entry steps at 7 or 8 waves 0.22 (profiles/r06_fwd_group_ab.txt).
#ifndef GSR_FWD_BLK_WAVES
#define GSR_FWD_BLK_WAVES 7
#endif
// list entries per step of a 16-lane group: their power -> G -> alpha tests first, then the
// compositing in list order (2: the registers of a step fit 7 waves per SIMD)
constexpr int kFG = 2;
// G by the hardware exp2 (v_exp_f32, 3 instructions instead of the 17 of splat_exp) with
// splat_exp wherever op * G lies within 2e-6 (relative) of 1/255 -- the alpha >= 1/255 decision
// stays the oracle's exactly, G differs from splat_exp's by < 1e-6 relative (so the T < 1e-4 stop
// can flip only at pixels within ~1e-6 of it, inside the parity tests' threshold margin); the
// backward evaluates the same instruction sequence, so its alpha is the forward's bit for bit.
template <bool FEAT>
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
  const uint32_t grp = (uint32_t)lane >> 4;

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

  // this lane's list entry of the next batch, loaded one batch ahead
  uint32_t pid_next = range.x + threadIdx.x < range.y ? a.point_list[range.x + threadIdx.x] : 0u;
  for (uint32_t base = range.x; base < range.y; base += kThreads) {
    // forward.cu:309-311: stop when every pixel of the tile is saturated
    if (__syncthreads_count(done) == kThreads) break;
    const uint32_t i = base + threadIdx.x;
    if (i < range.y) {
      const uint32_t pid = pid_next;
      if (i + kThreads < range.y) pid_next = a.point_list[i + kThreads];
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
      s_mask[threadIdx.x] = (uint16_t)block_mask(q0, q1, q3.z, tx, ty);
    }
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, range.y - base);
    uint32_t nmax;
    const uint32_t nl = build_group_lists(s_mask, s_list[wid], cnt, wid, lane, grp, nmax);
    const uint32_t rel0 = base - range.x;
    // kFG entries of the group's list per iteration: their (independent) Gaussian weights are
    // evaluated together, then composited in list order exactly as the reference's per-splat
    // loop -- same operations, same order, per pixel
    for (uint32_t k = 0; k < nmax; k += kFG) {
      if (__ballot(!done) == 0ull) break;  // wave-uniform
      static_assert(kFG == 2, "one 16-bit list read per step");
      const uint32_t packed = *reinterpret_cast<const uint16_t*>(&s_list[wid][grp][k]);
      uint32_t jj[kFG];
      float pw[kFG], al[kFG];
      float4 r1v[kFG], r2v[kFG];
      float f2v[kFG];
      float Gv[kFG];
      float tdist = 1.0f;  // min over the step's entries of |op * G - 1/255| (exact-path test)
#pragma unroll
      for (int u = 0; u < kFG; u++) {
        jj[u] = (packed >> (8 * u)) & 0xffu;
        const float4 r0 = s_r0[jj[u]];
        r1v[u] = s_r1[jj[u]];
        r2v[u] = s_r2[jj[u]];
        f2v[u] = FEAT ? s_f2[jj[u]] : 0.0f;
        const float dx = r0.x - pfx, dy = r0.y - pfy;
        const float power = -0.5f * (r0.z * dx * dx + r1v[u].x * dy * dy) - r0.w * dx * dy;
        // entries past the group's list end get power = +1 and are skipped
        pw[u] = (k + u < nl) ? power : 1.0f;
        Gv[u] = __builtin_amdgcn_exp2f(pw[u] * 1.44269504088896341f);
        const float d = fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f));
        tdist = d < tdist ? d : tdist;
      }
      // the exact path as one wave-uniform branch per step (as the backward's test
      // phase) instead of a divergent branch per entry; the per-entry condition is unchanged
      if (__ballot(tdist <= 2e-6f * (1.0f / 255.0f)) != 0ull) {
#pragma unroll
        for (int u = 0; u < kFG; u++)
          if (fabsf(r1v[u].y * Gv[u] - (1.0f / 255.0f)) <= 2e-6f * (1.0f / 255.0f))
            Gv[u] = splat_exp(pw[u]);
      }
#pragma unroll
      for (int u = 0; u < kFG; u++) al[u] = fminf(0.99f, r1v[u].y * Gv[u]);
#pragma unroll
      for (int u = 0; u < kFG; u++) {
        // one predicate per entry (the reference's skip / stop / blend decisions, NaN behaviour
        // included) instead of three nested skips: one exec-mask region per entry
        const float alpha = al[u];
        const float test_T = T * (1 - alpha);
        const bool take = !done && !(pw[u] > 0.0f) && !(alpha < 1.0f / 255.0f);
        const bool stop = take && test_T < 0.0001f;
        done = done || stop;
        if (take && !stop) {
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
          T = test_T;
          // the reference counts every list position (forward.cu:328); skipped entries cannot
          // blend
          last_contributor = rel0 + jj[u] + 1;
        }
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

template <bool FEAT>
__global__ __launch_bounds__(kThreads, GSR_FWD_BLK_WAVES) void render_fwd_blk_kernel(RenderArgs a) {
  render_fwd_blk_tile<FEAT>(a, blockIdx.x);
}

// The forward blends of several views in ONE launch (view-major workgroups, as
// render_bwd_views_kernel): no per-view tail of idle CUs.
template <bool FEAT>
__global__ __launch_bounds__(kThreads, GSR_FWD_BLK_WAVES) void render_fwd_blk_views_kernel(
    RenderFwdViews m) {
  const uint32_t b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.V && b >= m.first[k + 1]) k++;  // workgroup-uniform
  render_fwd_blk_tile<FEAT>(m.v[k], b - m.first[k]);
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

#endif  // GSR_RENDER_PART != 1
}  // namespace

#if GSR_RENDER_PART != 1
hipError_t launch_activations(const float* op_raw, const float* sc_raw, const float* rot_raw,
                              size_t P, float* op, float* sc, float* rot, hipStream_t s) {
  if (P == 0) return hipSuccess;
  hipLaunchKernelGGL(activations_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s,
                     op_raw, sc_raw, reinterpret_cast<const float4*>(rot_raw), P, op, sc,
                     reinterpret_cast<float4*>(rot));
  return hipGetLastError();
}

hipError_t launch_expf_pair(const float* x, float* ref, float* fast, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(expf_pair_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ref,
                     fast, n);
  return hipGetLastError();
}

hipError_t launch_render_schedule(const RenderArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0 || a.sched != 2) return hipSuccess;
  hipLaunchKernelGGL(tile_schedule_kernel, dim3(1), dim3(kSchedThreads), 0, s, a.ranges, ntiles,
                     a.order);
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
  if (feat)
    hipLaunchKernelGGL(render_fwd_blk_views_kernel<true>, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  else
    hipLaunchKernelGGL(render_fwd_blk_views_kernel<false>, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t launch_render_forward(const RenderArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0) return hipSuccess;
  if (hipError_t e = launch_render_schedule(a, s)) return e;
  if (a.include_feature)
    hipLaunchKernelGGL(render_fwd_blk_kernel<true>, dim3(ntiles), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(render_fwd_blk_kernel<false>, dim3(ntiles), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

#endif  // GSR_RENDER_PART != 1
#if GSR_RENDER_PART != 2
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
        (a.partial != nullptr) != (a.det != 0))
      return hipErrorInvalidValue;
    m.v[k] = w;
    m.first[k + 1] = m.first[k] + w.gx * w.gy;
  }
  const uint32_t nblk = m.first[V];
  if (nblk == 0) return hipSuccess;
#define GSR_BWDV(E, F)                                                                            \
  do {                                                                                           \
    if (a.det)                                                                                   \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, true>), dim3(nblk), dim3(kThreads), 0, s, m); \
    else                                                                                         \
      hipLaunchKernelGGL((render_bwd_views_kernel<E, F, false>), dim3(nblk), dim3(kThreads), 0, s, m); \
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
  if ((a.partial != nullptr) != (a.det != 0)) return hipErrorInvalidValue;
  const bool extra = a.dL_ddepth != nullptr || a.dL_dalpha != nullptr;
  const bool feat = a.include_feature && a.dL_dfeature != nullptr;
#define GSR_BWD(E, F)                                                                             \
  do {                                                                                           \
    if (a.det)                                                                                   \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, true>), dim3(ntiles), dim3(kThreads), 0, s, a); \
    else                                                                                         \
      hipLaunchKernelGGL((render_bwd_kernel<E, F, false>), dim3(ntiles), dim3(kThreads), 0, s, a); \
  } while (0)
  if (feat) GSR_BWD(true, true);
  else if (extra) GSR_BWD(true, false);
  else GSR_BWD(false, false);
#undef GSR_BWD
  return hipGetLastError();
}

#endif  // GSR_RENDER_PART != 2
}  // namespace gsr

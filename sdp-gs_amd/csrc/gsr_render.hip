// gsr_render.hip -- per-tile alpha blending, forward and backward, for gfx950.
//
// Reference behaviour: renderCUDA forward (cuda_rasterizer/forward.cu:261-374) and backward
// (cuda_rasterizer/backward.cu:399-557), extended with depth / alpha / 3-channel feature outputs
// (SURVEY.md row A12).
//
// gfx950 design:
//  * one 256-lane workgroup (4 waves of 64) per 16x16 tile; wave w owns pixel rows 4w..4w+3;
//  * XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so block b is remapped
//    to a contiguous band of tiles per XCD and neighbouring tiles (which share most of their
//    splats) hit the same 4 MiB L2;
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

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles) {
  const uint32_t q = ntiles >> 3, r = ntiles & 7u;
  const uint32_t xcd = b & 7u, local = b >> 3;
  const uint32_t start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + local;
}

// Which of the 4 waves (pixel rows 4w..4w+3 of the tile) a splat can reach: bit w set unless the
// conservative test of gsr_device.h proves alpha < 1/255 on all 64 pixels of wave w.
__device__ __forceinline__ uint32_t wave_mask(float4 r0, float4 r1, uint32_t tx, uint32_t ty) {
  const float qc = splat_q_cut(r0.z, r0.w, r1.x, r1.y);
  if (qc == -1.0f) return 0xfu;
  if (qc == -2.0f) return 0u;
  const float x0 = (float)(tx * kTile), x1 = (float)(tx * kTile + kTile - 1);
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const float y0 = (float)(ty * kTile + 4 * w);
    m |= splat_touches_rect(r0.x, r0.y, r0.z, r0.w, r1.x, qc, x0, x1, y0, y0 + 3.0f) ? (1u << w) : 0u;
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
  __shared__ float4 s_r3[FEAT ? kThreads : 1];
  __shared__ uint8_t s_mask[kThreads];
  __shared__ uint8_t s_list[kThreads / 64][kThreads];
  __shared__ uint32_t s_max;
  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);

  const uint32_t ntiles = a.gx * a.gy;
  const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  const uint32_t px = tx * kTile + (threadIdx.x & (kTile - 1));
  const uint32_t py = ty * kTile + (threadIdx.x >> 4);
  const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
  const float pfx = (float)px, pfy = (float)py;
  bool done = !inside;
  if (threadIdx.x == 0) s_max = 0;

  const uint2 range = a.ranges[tile];
  float T = 1.0f;
  uint32_t contributor = 0, last_contributor = 0;
  constexpr int NC = FEAT ? 8 : 5;
  float C[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) C[c] = 0.0f;

  for (uint32_t base = range.x; base < range.y; base += kThreads) {
    // forward.cu:309-311: stop when every pixel of the tile is saturated
    if (__syncthreads_count(done) == kThreads) break;
    const uint32_t i = base + threadIdx.x;
    if (i < range.y) {
      const uint32_t gid = a.point_list[i];
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = q1;
      s_r2[threadIdx.x] = rec[2];
      if (FEAT) s_r3[threadIdx.x] = rec[3];
      s_mask[threadIdx.x] = (uint8_t)wave_mask(q0, q1, tx, ty);
    }
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, range.y - base);
    const uint32_t nlist = build_wave_list(s_mask, s_list[wid], cnt, wid, lane);
    for (uint32_t k = 0; !done && k < nlist; k++) {
      const uint32_t j = s_list[wid][k];
      // the reference counts every list position (forward.cu:328); skipped entries cannot blend
      contributor = base - range.x + j + 1;
      const float4 r0 = s_r0[j];
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      const float4 r1 = s_r1[j];
      const float power = -0.5f * (r0.z * dx * dx + r1.x * dy * dy) - r0.w * dx * dy;
      if (power > 0.0f) continue;
      const float alpha = fminf(0.99f, r1.y * expf(power));
      if (alpha < 1.0f / 255.0f) continue;
      const float test_T = T * (1 - alpha);
      if (test_T < 0.0001f) {
        done = true;
        continue;
      }
      const float4 r2 = s_r2[j];
      C[0] += r1.w * alpha * T;
      C[1] += r2.x * alpha * T;
      C[2] += r2.y * alpha * T;
      C[3] += r1.z * alpha * T;
      C[4] += alpha * T;
      if (FEAT) {
        const float4 r3 = s_r3[j];
        C[5] += r2.z * alpha * T;
        C[6] += r2.w * alpha * T;
        C[7] += r3.x * alpha * T;
      }
      T = test_T;
      last_contributor = contributor;
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

// Halving butterfly: on entry every lane holds 16 partial values; on exit lane l holds the wave
// sum of value index ((l>>5)&1)*8 + ((l>>4)&1)*4 + ((l>>3)&1)*2 + ((l>>2)&1) (4 lanes each).
__device__ __forceinline__ float wave_reduce16(float (&v)[16], int lane) {
  {
    const bool hi = lane & 32;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const float send = hi ? v[i] : v[i + 8];
      const float keep = hi ? v[i + 8] : v[i];
      v[i] = keep + __shfl_xor(send, 32, 64);
    }
  }
  {
    const bool hi = lane & 16;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float send = hi ? v[i] : v[i + 4];
      const float keep = hi ? v[i + 4] : v[i];
      v[i] = keep + __shfl_xor(send, 16, 64);
    }
  }
  {
    const bool hi = lane & 8;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const float send = hi ? v[i] : v[i + 2];
      const float keep = hi ? v[i + 2] : v[i];
      v[i] = keep + __shfl_xor(send, 8, 64);
    }
  }
  float x;
  {
    const bool hi = lane & 4;
    const float send = hi ? v[0] : v[1];
    const float keep = hi ? v[1] : v[0];
    x = keep + __shfl_xor(send, 4, 64);
  }
  x += __shfl_xor(x, 2, 64);
  x += __shfl_xor(x, 1, 64);
  return x;
}

template <bool EXTRA, bool FEAT>
__global__ __launch_bounds__(kThreads) void render_bwd_kernel(RenderBwdArgs a) {
  __shared__ float4 s_r0[kThreads];
  __shared__ float4 s_r1[kThreads];
  __shared__ float4 s_r2[kThreads];
  __shared__ float4 s_r3[FEAT ? kThreads : 1];
  __shared__ uint32_t s_gid[kThreads];
  __shared__ float s_acc[kThreads][kAccFloats];
  __shared__ uint8_t s_mask[kThreads];
  __shared__ uint8_t s_list[kThreads / 64][kThreads];

  const int lane = (int)(threadIdx.x & 63);
  const int wid = (int)(threadIdx.x >> 6);
  const uint32_t ntiles = a.gx * a.gy;
  const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
  const uint32_t tx = tile % a.gx, ty = tile / a.gx;
  const uint32_t px = tx * kTile + (threadIdx.x & (kTile - 1));
  const uint32_t py = ty * kTile + (threadIdx.x >> 4);
  const bool inside = px < (uint32_t)a.W && py < (uint32_t)a.H;
  const float pfx = (float)px, pfy = (float)py;
  const size_t pix = (size_t)py * a.W + px;
  const size_t HW = (size_t)a.W * a.H;

  const uint2 range = a.ranges[tile];
  const uint32_t tile_last = a.tile_last[tile];
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
  float accum_rec[NC], last_color[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) { accum_rec[c] = 0.0f; last_color[c] = 0.0f; }
  float last_alpha = 0.0f;
  const float ddelx_dx = (float)(0.5 * a.W);
  const float ddely_dy = (float)(0.5 * a.H);

#pragma unroll
  for (int k = 0; k < kAccFloats; k++) s_acc[threadIdx.x][k] = 0.0f;

  // rel = position inside the tile's list; every pixel only uses rel < its n_contrib <= tile_last
  for (uint32_t done_cnt = 0; done_cnt < tile_last; done_cnt += kThreads) {
    __syncthreads();
    const uint32_t cnt = min((uint32_t)kThreads, tile_last - done_cnt);
    if (threadIdx.x < cnt) {
      const uint32_t rel = tile_last - 1 - done_cnt - threadIdx.x;
      const uint32_t gid = a.point_list[range.x + rel];
      s_gid[threadIdx.x] = gid;
      const float4* rec = a.rec + 4 * (size_t)gid;
      const float4 q0 = rec[0], q1 = rec[1];
      s_r0[threadIdx.x] = q0;
      s_r1[threadIdx.x] = q1;
      s_mask[threadIdx.x] = (uint8_t)wave_mask(q0, q1, tx, ty);
      s_r2[threadIdx.x] = rec[2];
      if (FEAT) s_r3[threadIdx.x] = rec[3];
    }
    __syncthreads();
    const uint32_t nlist = build_wave_list(s_mask, s_list[wid], cnt, wid, lane);
    for (uint32_t k = 0; k < nlist; k++) {
      const uint32_t j = s_list[wid][k];
      const uint32_t rel = tile_last - 1 - done_cnt - j;
      if (rel >= wave_last) continue;  // wave-uniform: behind every pixel of this wave
      const float4 r0 = s_r0[j];
      const float4 r1 = s_r1[j];
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      bool contrib = rel < last_contributor;
      const float power = -0.5f * (r0.z * dx * dx + r1.x * dy * dy) - r0.w * dx * dy;
      contrib = contrib && !(power > 0.0f);
      const float G = expf(power);
      const float alpha = fminf(0.99f, r1.y * G);
      contrib = contrib && !(alpha < 1.0f / 255.0f);
      if (__ballot(contrib) == 0ull) continue;  // wave-uniform skip

      float g[kAccFloats];
#pragma unroll
      for (int k = 0; k < kAccFloats; k++) g[k] = 0.0f;
      if (contrib) {
        const float4 r2 = s_r2[j];
        T = T / (1.f - alpha);
        const float dchannel_dcolor = alpha * T;
        float col[NC];
        col[0] = r1.w; col[1] = r2.x; col[2] = r2.y;
        if (NC > 3) { col[3 % NC] = r1.z; col[4 % NC] = 1.0f; }
        if (FEAT) {
          const float4 r3 = s_r3[j];
          col[5 % NC] = r2.z; col[6 % NC] = r2.w; col[7 % NC] = r3.x;
        }
        float dL_dalpha = 0.0f;
#pragma unroll
        for (int c = 0; c < NC; c++) {
          accum_rec[c] = last_alpha * last_color[c] + (1.f - last_alpha) * accum_rec[c];
          last_color[c] = col[c];
          dL_dalpha += (col[c] - accum_rec[c]) * dpix[c];
        }
        g[kAccR] = dchannel_dcolor * dpix[0];
        g[kAccG] = dchannel_dcolor * dpix[1];
        g[kAccB] = dchannel_dcolor * dpix[2];
        if (NC > 3) g[kAccDepth] = dchannel_dcolor * dpix[3 % NC];
        if (FEAT) {
          g[kAccF0] = dchannel_dcolor * dpix[5 % NC];
          g[kAccF1] = dchannel_dcolor * dpix[6 % NC];
          g[kAccF2] = dchannel_dcolor * dpix[7 % NC];
        }
        dL_dalpha *= T;
        last_alpha = alpha;
        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
        const float dL_dG = r1.y * dL_dalpha;
        const float gdx = G * dx;
        const float gdy = G * dy;
        const float dG_ddelx = -gdx * r0.z - gdy * r0.w;
        const float dG_ddely = -gdy * r1.x - gdx * r0.w;
        g[kAccMx] = dL_dG * dG_ddelx * ddelx_dx;
        g[kAccMy] = dL_dG * dG_ddely * ddely_dy;
        g[kAccCa] = -0.5f * gdx * dx * dL_dG;
        g[kAccCb] = -0.5f * gdx * dy * dL_dG;
        g[kAccCc] = -0.5f * gdy * dy * dL_dG;
        g[kAccOp] = G * dL_dalpha;
        g[kAccUsed] = 1.0f;
      }
      const float sum = wave_reduce16(g, lane);
      if ((lane & 3) == 0) {
        const int k = ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 +
                      ((lane >> 2) & 1);
        if (sum != 0.0f) atomicAdd(&s_acc[j][k], sum);
      }
    }
    __syncthreads();
    // flush: lane l of wave-instruction `it` handles splat (it*16 + tid/16), slot tid%16
#pragma unroll 4
    for (int it = 0; it < kThreads * kAccFloats / kThreads; it++) {
      const uint32_t jj = (uint32_t)it * (kThreads / kAccFloats) + (threadIdx.x >> 4);
      const int k = (int)(threadIdx.x & 15);
      if (jj < cnt) {
        const float v = s_acc[jj][k];
        if (v != 0.0f) {
          atomicAdd(&a.acc[(size_t)s_gid[jj] * kAccFloats + k], v);
          s_acc[jj][k] = 0.0f;
        }
      }
    }
  }
}

}  // namespace

hipError_t launch_render_forward(const RenderArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0) return hipSuccess;
  if (a.include_feature)
    hipLaunchKernelGGL(render_fwd_kernel<true>, dim3(ntiles), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(render_fwd_kernel<false>, dim3(ntiles), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t s) {
  const uint32_t ntiles = a.gx * a.gy;
  if (ntiles == 0) return hipSuccess;
  const bool extra = a.dL_ddepth != nullptr || a.dL_dalpha != nullptr;
  const bool feat = a.include_feature && a.dL_dfeature != nullptr;
  if (feat)
    hipLaunchKernelGGL((render_bwd_kernel<true, true>), dim3(ntiles), dim3(kThreads), 0, s, a);
  else if (extra)
    hipLaunchKernelGGL((render_bwd_kernel<true, false>), dim3(ntiles), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((render_bwd_kernel<false, false>), dim3(ntiles), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace gsr

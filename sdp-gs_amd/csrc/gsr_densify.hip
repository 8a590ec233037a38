// gsr_densify.hip -- adaptive density control over the SoA Gaussian arrays.
//
// Reference (scene/gaussian_model.py:400-612, train.py:218-224): every training step updates the
// densification statistics through boolean-mask indexing (max_radii2D, xyz_gradient_accum, denom:
// each `t[mask]` is a nonzero() with a device->host sync), and every densification_interval steps
// densify_and_prune clones, splits and prunes by torch.cat / boolean indexing of each parameter
// and of both Adam moments, one full-array pass per tensor per stage (clone cat, split cat, split
// prune, final prune).
//
// Here:
//   stats_kernel     the per-step update of train.py:219-220 in one elementwise pass, no sync;
//   classify_kernel  densify_and_prune's per-Gaussian decisions (clone / split / prune tests) as
//                    one flag byte per Gaussian plus counts;
//   select_*         stable compaction of a flag-byte predicate into an ascending index list
//                    (reduce -> scan -> write, 16 flags per lane);
//   compact_kernel   ONE launch that writes every output array (parameters, moments, confidence,
//                    statistics) of the post-densification set: output row j of array a is row
//                    index[j] of [old rows | appended rows] (or a fill word where that part has no
//                    source), so each surviving byte is read once and written once.
#include "gsr_internal.h"
#include "../../include/gsr_densify.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// ---- per-step statistics -------------------------------------------------------------------------
// train.py:219: max_radii2D[f] = torch.max(max_radii2D[f], radii[f])  (int radii promoted to float)
// gaussian_model.py:607-609: xyz_gradient_accum[f] += norm(grad[f, :2]); denom[f] += 1
__global__ __launch_bounds__(kThreads) void stats_kernel(int64_t P, const float* __restrict__ g,
                                                         int64_t ld, const int32_t* __restrict__ radii,
                                                         const uint8_t* __restrict__ filt,
                                                         float* __restrict__ maxr,
                                                         float* __restrict__ accum,
                                                         float* __restrict__ denom) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= P) return;
  const bool on = filt ? filt[i] != 0 : radii[i] > 0;
  if (!on) return;
  if (maxr) {
    const float m = maxr[i], r = (float)radii[i];
    maxr[i] = (m > r || m != m) ? m : r;  // torch.maximum: NaN propagates
  }
  if (accum) {
    const float gx = g[i * ld], gy = g[i * ld + 1];
    accum[i] = accum[i] + sqrtf(gx * gx + gy * gy);
    denom[i] = denom[i] + 1.0f;
  }
}

// The same update for the V views of a multi-view step in one launch: per Gaussian the views in
// order (the per-view launches' additions and maxima, in the same order), filter radii > 0.
__global__ __launch_bounds__(kThreads) void stats_views_kernel(int V, int64_t P,
                                                               const float* __restrict__ g,
                                                               int64_t ld, int64_t gview,
                                                               const int32_t* __restrict__ radii,
                                                               float* __restrict__ maxr,
                                                               float* __restrict__ accum,
                                                               float* __restrict__ denom) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= P) return;
  float m = maxr ? maxr[i] : 0.f, acc = accum ? accum[i] : 0.f, den = accum ? denom[i] : 0.f;
  bool any = false;
  for (int v = 0; v < V; v++) {
    const int32_t rv = radii[(size_t)v * P + i];
    if (!(rv > 0)) continue;
    any = true;
    const float r = (float)rv;
    m = (m > r || m != m) ? m : r;  // torch.maximum: NaN propagates
    const float* gv = g + (size_t)v * gview + i * ld;
    if (accum) {
      const float gx = gv[0], gy = gv[1];
      acc = acc + sqrtf(gx * gx + gy * gy);
      den = den + 1.0f;
    }
  }
  if (!any) return;
  if (maxr) maxr[i] = m;
  if (accum) {
    accum[i] = acc;
    denom[i] = den;
  }
}

// ---- densify_and_prune decisions -------------------------------------------------------------------
struct ClassifyArgs {
  int64_t P;
  const float *accum, *denom, *scaling, *opacity;
  float grad_threshold, scale_limit, min_opacity, big_limit;
  int big_enable;
  uint8_t* flags;
  uint32_t* counts;
};

__device__ __forceinline__ float max_nan(float a, float b) { return (b > a || b != b) ? b : a; }

// Grid-stride over a bounded grid; the optional counts take ONE atomic per workgroup (same-address
// device-scope atomics from every wave serialise across the XCDs: 180 us at 1M rows).
constexpr int kClassifyMaxGroups = 512;

__global__ __launch_bounds__(kThreads) void classify_kernel(ClassifyArgs a) {
  __shared__ uint32_t s_cnt[2][kThreads / 64];
  uint32_t nc = 0, ns = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.P;
       i += (int64_t)gridDim.x * kThreads) {
    uint32_t f = 0;
    // grads = accum / denom; grads[grads.isnan()] = 0 (:585-586); no denom: the caller's grads
    float g = a.accum[i];
    if (a.denom) {
      g = g / a.denom[i];
      if (g != g) g = 0.0f;
    }
    // torch.max(get_scaling, dim=1).values, get_scaling = exp(_scaling)
    const float s = max_nan(max_nan(expf(a.scaling[3 * i]), expf(a.scaling[3 * i + 1])),
                            expf(a.scaling[3 * i + 2]));
    // densify_and_clone (:566-570): torch.norm(grads, dim=-1) of the [P,1] grads
    if (sqrtf(g * g) >= a.grad_threshold && s <= a.scale_limit) f |= GSR_DENSIFY_CLONE;
    // densify_and_split (:537-542): padded_grad >= threshold
    if (g >= a.grad_threshold && s > a.scale_limit) f |= GSR_DENSIFY_SPLIT;
    // densify_and_prune's prune mask (:593-597): get_opacity < min_opacity; max scale > 0.1 extent
    const float op = 1.0f / (1.0f + expf(-a.opacity[i]));
    if (op < a.min_opacity) f |= GSR_DENSIFY_LOW_OPACITY;
    if (a.big_enable && s > a.big_limit) f |= GSR_DENSIFY_BIG_WS;
    a.flags[i] = (uint8_t)f;
    nc += (f & GSR_DENSIFY_CLONE) ? 1u : 0u;
    ns += (f & GSR_DENSIFY_SPLIT) ? 1u : 0u;
  }
  if (!a.counts) return;  // workgroup-uniform
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    nc += __shfl_xor(nc, d, 64);
    ns += __shfl_xor(ns, d, 64);
  }
  if (lane_id() == 0) {
    s_cnt[0][threadIdx.x >> 6] = nc;
    s_cnt[1][threadIdx.x >> 6] = ns;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t c = s_cnt[0][0] + s_cnt[0][1] + s_cnt[0][2] + s_cnt[0][3];
    const uint32_t t = s_cnt[1][0] + s_cnt[1][1] + s_cnt[1][2] + s_cnt[1][3];
    if (c) atomicAdd(&a.counts[0], c);
    if (t) atomicAdd(&a.counts[1], t);
  }
}

// ---- stable selection ---------------------------------------------------------------------------
constexpr int kSelPerLane = 16;
constexpr int kSelTile = kThreads * kSelPerLane;  // 4096 flags per workgroup

// the 16 flags of this lane as a bitmask of predicate hits
__device__ __forceinline__ uint32_t select_hits(const uint8_t* __restrict__ flags, int64_t n,
                                                uint32_t mask, uint32_t want, int64_t i0) {
  uint32_t hits = 0;
  if (i0 + kSelPerLane <= n && (((uintptr_t)(flags + i0)) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(flags + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < kSelPerLane; k++)
      hits |= (((w[k >> 2] >> (8 * (k & 3))) & mask) == want ? 1u : 0u) << k;
  } else {
    for (int k = 0; k < kSelPerLane; k++)
      if (i0 + k < n && (flags[i0 + k] & mask) == want) hits |= 1u << k;
  }
  return hits;
}

__global__ __launch_bounds__(kThreads) void select_count_kernel(const uint8_t* __restrict__ flags,
                                                                int64_t n, uint32_t mask,
                                                                uint32_t want,
                                                                uint32_t* __restrict__ parts) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i0 = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelPerLane;
  uint32_t c = __popc(select_hits(flags, n, mask, want, i0));
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if (lane_id() == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) parts[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// incl: inclusive scan of the per-workgroup counts
__global__ __launch_bounds__(kThreads) void select_write_kernel(const uint8_t* __restrict__ flags,
                                                                int64_t n, uint32_t mask,
                                                                uint32_t want,
                                                                const uint32_t* __restrict__ incl,
                                                                uint32_t nblocks,
                                                                uint32_t* __restrict__ index,
                                                                uint32_t* __restrict__ count) {
  __shared__ uint32_t s_w[kThreads / 64];
  const int64_t i0 = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelPerLane;
  uint32_t hits = select_hits(flags, n, mask, want, i0);
  const uint32_t c = __popc(hits);
  // exclusive prefix of c over the workgroup
  uint32_t x = c;
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  const int wid = (int)(threadIdx.x >> 6);
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  uint32_t pre = x - c;
  for (int w = 0; w < wid; w++) pre += s_w[w];
  uint32_t o = (blockIdx.x ? incl[blockIdx.x - 1] : 0u) + pre;
  while (hits) {
    const int k = __ffs(hits) - 1;
    hits &= hits - 1;
    index[o++] = (uint32_t)(i0 + k);
  }
  if (blockIdx.x == nblocks - 1 && threadIdx.x == 0 && count) *count = incl[nblocks - 1];
}

// ---- multi-array row compaction -----------------------------------------------------------------
constexpr int kRowsPerGroup = 256;
constexpr int kUnroll = 4;

struct CompactArgs {
  int n;
  const uint32_t* src[GSR_COMPACT_MAX_ARRAYS];
  const uint32_t* extra[GSR_COMPACT_MAX_ARRAYS];
  uint32_t* dst[GSR_COMPACT_MAX_ARRAYS];
  uint32_t w[GSR_COMPACT_MAX_ARRAYS];      // 32-bit words per row
  uint32_t magic[GSR_COMPACT_MAX_ARRAYS];  // ceil(2^32 / w)
  uint32_t fill[GSR_COMPACT_MAX_ARRAYS];
  int64_t n_old, n_out;
  const uint32_t* index;  // [n_out] rows of [old | extra]; NULL = identity
};

__global__ __launch_bounds__(kThreads) void compact_kernel(CompactArgs a) {
  __shared__ uint32_t s_idx[kRowsPerGroup];
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerGroup;
  const int nr = (int)((a.n_out - r0) < kRowsPerGroup ? (a.n_out - r0) : kRowsPerGroup);
  if ((int)threadIdx.x < nr)
    s_idx[threadIdx.x] = a.index ? a.index[r0 + threadIdx.x] : (uint32_t)(r0 + threadIdx.x);
  __syncthreads();
  const uint32_t n_old = (uint32_t)a.n_old;
  for (int t = 0; t < a.n; t++) {  // workgroup-uniform
    const uint32_t w = a.w[t], magic = a.magic[t], fill = a.fill[t];
    const uint32_t* __restrict__ src = a.src[t];
    const uint32_t* __restrict__ extra = a.extra[t];
    uint32_t* __restrict__ dst = a.dst[t] + (size_t)r0 * w;
    const int total = nr * (int)w;
    for (int e0 = (int)threadIdx.x; e0 < total; e0 += kThreads * kUnroll) {
      uint32_t val[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const int e = e0 + u * kThreads;
        val[u] = fill;
        if (e < total) {
          // e / w, exact while e * w < 2^32 (w == 1: magic would be 2^32)
          const uint32_t j = w == 1 ? (uint32_t)e : __umulhi((uint32_t)e, magic);
          const uint32_t k = (uint32_t)e - j * w;
          const uint32_t v = s_idx[j];
          if (v < n_old) {
            if (src) val[u] = src[(size_t)v * w + k];
          } else if (extra) {
            val[u] = extra[(size_t)(v - n_old) * w + k];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const int e = e0 + u * kThreads;
        if (e < total) dst[e] = val[u];
      }
    }
  }
}

size_t select_blocks(int64_t n) { return (size_t)((n + kSelTile - 1) / kSelTile); }

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" int gsr_densify_stats(int64_t P, const float* viewspace_grad, int64_t grad_stride,
                                 const int32_t* radii, const uint8_t* update_filter,
                                 float* max_radii2D, float* grad_accum, float* denom,
                                 void* stream) {
  if (P < 0 || (!update_filter && !radii) || (max_radii2D && !radii) ||
      ((grad_accum != nullptr) != (denom != nullptr)) ||
      (grad_accum && (!viewspace_grad || grad_stride < 2)))
    return 1;
  if (P == 0) return 0;
  hipLaunchKernelGGL(stats_kernel, dim3((unsigned)((P + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, (hipStream_t)stream, P, viewspace_grad, grad_stride, radii, update_filter,
                     max_radii2D, grad_accum, denom);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_densify_stats_views(int V, int64_t P, const float* viewspace_grad,
                                       int64_t grad_stride, int64_t grad_view_stride,
                                       const int32_t* radii, float* max_radii2D,
                                       float* grad_accum, float* denom, void* stream) {
  if (V < 0 || P < 0 || !radii || ((grad_accum != nullptr) != (denom != nullptr)) ||
      (grad_accum && (!viewspace_grad || grad_stride < 2)))
    return 1;
  if (P == 0 || V == 0) return 0;
  hipLaunchKernelGGL(stats_views_kernel, dim3((unsigned)((P + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, (hipStream_t)stream, V, P, viewspace_grad, grad_stride,
                     grad_view_stride, radii, max_radii2D, grad_accum, denom);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_densify_classify(int64_t P, const float* grad_accum, const float* denom,
                                    const float* scaling, const float* opacity,
                                    float grad_threshold, float scale_limit, float min_opacity,
                                    int big_enable, float big_limit, uint8_t* flags,
                                    uint32_t* counts, void* stream) {
  if (P < 0 || P > 0xffffffffLL) return 1;
  if (P > 0 && (!grad_accum || !scaling || !opacity || !flags)) return 1;
  hipStream_t s = (hipStream_t)stream;
  if (counts && hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), s) != hipSuccess) return 2;
  if (P == 0) return 0;
  ClassifyArgs a{P, grad_accum, denom, scaling, opacity, grad_threshold, scale_limit,
                 min_opacity, big_limit, big_enable, flags, counts};
  const int64_t groups = (P + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(classify_kernel,
                     dim3((unsigned)(groups < kClassifyMaxGroups ? groups : kClassifyMaxGroups)),
                     dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" size_t gsr_select_scratch_bytes(int64_t n) {
  if (n <= 0) return 0;
  const size_t nb = select_blocks(n);
  return (2 * nb + scan_parts(nb)) * sizeof(uint32_t);
}

extern "C" int gsr_select_rows(int64_t n, const uint8_t* flags, uint32_t mask, uint32_t want,
                               uint32_t* index, uint32_t* count, void* scratch, void* stream) {
  if (n < 0 || n > 0xffffffffLL || mask > 0xff || (want & ~mask)) return 1;
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    if (count && hipMemsetAsync(count, 0, sizeof(uint32_t), s) != hipSuccess) return 2;
    return 0;
  }
  if (!flags || !index || !scratch) return 1;
  const size_t nb = select_blocks(n);
  uint32_t* parts = (uint32_t*)scratch;
  uint32_t* incl = parts + nb;
  uint32_t* scan_scratch = incl + nb;
  hipLaunchKernelGGL(select_count_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, flags, n, mask,
                     want, parts);
  if (scan_u32(parts, nullptr, incl, nb, true, scan_scratch, s) != hipSuccess) return 2;
  hipLaunchKernelGGL(select_write_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, flags, n, mask,
                     want, incl, (uint32_t)nb, index, count);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_compact_rows(int n_arrays, const void* const* src, const void* const* extra,
                                void* const* dst, const int64_t* row_bytes, const uint32_t* fill,
                                int64_t n_old, const uint32_t* index, int64_t n_out,
                                void* stream) {
  if (n_arrays < 0 || n_arrays > GSR_COMPACT_MAX_ARRAYS || n_old < 0 || n_out < 0 ||
      n_old > 0xffffffffLL || n_out > 0xffffffffLL)
    return 1;
  if (n_arrays == 0 || n_out == 0) return 0;
  CompactArgs a{};
  a.n = n_arrays;
  for (int t = 0; t < n_arrays; t++) {
    const int64_t rb = row_bytes[t];
    // whole 32-bit words per row; e / w by multiply-high needs e * w < 2^32, e < 256 w
    if (rb <= 0 || (rb & 3) || rb / 4 > 1024 || !dst[t] || ((uintptr_t)dst[t] & 3) ||
        ((uintptr_t)(src ? src[t] : nullptr) & 3) || ((uintptr_t)(extra ? extra[t] : nullptr) & 3))
      return 1;
    a.src[t] = src ? (const uint32_t*)src[t] : nullptr;
    a.extra[t] = extra ? (const uint32_t*)extra[t] : nullptr;
    a.dst[t] = (uint32_t*)dst[t];
    a.w[t] = (uint32_t)(rb / 4);
    a.magic[t] = a.w[t] == 1 ? 0u : (uint32_t)((0x100000000ull + a.w[t] - 1) / a.w[t]);
    a.fill[t] = fill ? fill[t] : 0u;
  }
  a.n_old = n_old;
  a.n_out = n_out;
  a.index = index;
  const unsigned blocks = (unsigned)((n_out + kRowsPerGroup - 1) / kRowsPerGroup);
  hipLaunchKernelGGL(compact_kernel, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

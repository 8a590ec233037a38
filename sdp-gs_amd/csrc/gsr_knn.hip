// gsr_knn.hip -- exact 3-nearest-neighbour search over a point set.
//
// Replaces simple_knn._C.distCUDA2, an un-vendored native dependency of the reference
// (scene/gaussian_model.py:20), called by create_from_pcd for the initial scales (:198) and by
// proximity densification (:514) as `dist, nearest_indices = distCUDA2(xyz)`: per point the mean
// squared distance to its 3 nearest other points, and their indices.  The published simple_knn
// algorithm (Morton-order sort, boxes of consecutive sorted points, an initial bound from the
// sorted neighbours, boxes skipped when their distance exceeds the current third-best) is exact;
// so is this search, with a layout for wave64:
//
//   bbox       two-level min/max reduction of the coordinates
//   morton     30-bit Morton code of each point in the bounding box; stable radix sort
//              (gsr_sort.hip) of (code, index)
//   layout     sorted points as float4 (x, y, z, index bits); a BOX is 64 consecutive sorted points
//              = one wave, a SUPERBOX is 64 boxes; AABBs of both
//   query      one wave per box, one lane per point: the own box first (points broadcast by
//              v_readlane), then superboxes / boxes outward from the own one, each skipped unless
//              some lane's distance to its AABB is <= that lane's current third-best; visited boxes
//              are scanned point by point with the same broadcast.
//
// Neighbour order is (squared distance, index) ascending -- a total order, so the result does not
// depend on the traversal order (simple_knn keeps the first-visited of equal distances, i.e.
// Morton order; this differs only for exactly equal distances).  Squared distance is
// fma(dz, dz, fma(dy, dy, dx * dx)) with d = candidate - query, the contraction nvcc applies to
// simple_knn's `d.x * d.x + d.y * d.y + d.z * d.z`; the mean is (b0 + b1 + b2) / 3.  Missing
// neighbours (P < 4) count as FLT_MAX with index -1, as simple_knn initialises them.
#include <float.h>

#include "gsr_internal.h"
#include "../../include/gsr_knn.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kBox = 64;           // points per box = lanes per wave
constexpr int kSuper = 64;         // boxes per superbox
constexpr int kBBoxTile = 4096;    // points per bbox-partial workgroup
constexpr int kMortonBits = 30;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

struct KnnState {
  float* bbox_parts;   // [nparts][6]
  float* bbox;         // [6] min xyz, max xyz
  uint32_t *ka, *va, *kb, *vb;
  SortScratch sort;
  float4* pts;         // [P] sorted (x, y, z, index bits)
  float4* boxes;       // [nbox][2] (min, max)
  float4* supers;      // [nsuper][2]
  size_t bytes;
};

KnnState carve_knn(char* base, size_t P) {
  Carver c(base);
  KnnState k{};
  const size_t nparts = (P + kBBoxTile - 1) / kBBoxTile;
  const size_t nbox = (P + kBox - 1) / kBox;
  const size_t nsup = (nbox + kSuper - 1) / kSuper;
  k.bbox_parts = c.take<float>(6 * (nparts ? nparts : 1));
  k.bbox = c.take<float>(8);
  k.ka = c.take<uint32_t>(P);
  k.va = c.take<uint32_t>(P);
  k.kb = c.take<uint32_t>(P);
  k.vb = c.take<uint32_t>(P);
  k.sort = take_sort_scratch(c, P);
  k.pts = c.take<float4>(P);
  k.boxes = c.take<float4>(2 * nbox);
  k.supers = c.take<float4>(2 * nsup);
  k.bytes = c.size();
  return k;
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = fminf(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = fmaxf(v, __shfl_xor(v, d, 64));
  return v;
}

// min / max of x, y, z over [lo, hi) per workgroup -> out[6]
__device__ void block_bbox(const float* __restrict__ pts3, size_t lo, size_t hi, float* out) {
  __shared__ float s[6][kThreads / 64];
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (size_t i = lo + threadIdx.x; i < hi; i += kThreads)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const float v = pts3[3 * i + c];
      mn[c] = fminf(mn[c], v);
      mx[c] = fmaxf(mx[c], v);
    }
  const int w = (int)(threadIdx.x >> 6);
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float a = wave_min(mn[c]), b = wave_max(mx[c]);
    if (lane_id() == 0) {
      s[c][w] = a;
      s[3 + c][w] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float r = s[threadIdx.x][0];
    for (int k = 1; k < kThreads / 64; k++)
      r = threadIdx.x < 3 ? fminf(r, s[threadIdx.x][k]) : fmaxf(r, s[threadIdx.x][k]);
    out[threadIdx.x] = r;
  }
}

__global__ __launch_bounds__(kThreads) void bbox_parts_kernel(const float* __restrict__ xyz,
                                                              size_t P, float* __restrict__ parts) {
  const size_t lo = (size_t)blockIdx.x * kBBoxTile;
  const size_t hi = lo + kBBoxTile < P ? lo + kBBoxTile : P;
  block_bbox(xyz, lo, hi, parts + 6 * blockIdx.x);
}

// parts viewed as [nparts] points of 6 floats: reduce mins of the first three, maxes of the rest
__global__ __launch_bounds__(kThreads) void bbox_final_kernel(const float* __restrict__ parts,
                                                              size_t nparts, float* __restrict__ bbox) {
  __shared__ float s[6][kThreads / 64];
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (size_t i = threadIdx.x; i < nparts; i += kThreads)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      mn[c] = fminf(mn[c], parts[6 * i + c]);
      mx[c] = fmaxf(mx[c], parts[6 * i + 3 + c]);
    }
  const int w = (int)(threadIdx.x >> 6);
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float a = wave_min(mn[c]), b = wave_max(mx[c]);
    if (lane_id() == 0) {
      s[c][w] = a;
      s[3 + c][w] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float r = s[threadIdx.x][0];
    for (int k = 1; k < kThreads / 64; k++)
      r = threadIdx.x < 3 ? fminf(r, s[threadIdx.x][k]) : fmaxf(r, s[threadIdx.x][k]);
    bbox[threadIdx.x] = r;
  }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__global__ __launch_bounds__(kThreads) void morton_kernel(const float* __restrict__ xyz, size_t P,
                                                          const float* __restrict__ bbox,
                                                          uint32_t* __restrict__ key,
                                                          uint32_t* __restrict__ val) {
  const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= P) return;
  uint32_t q[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float lo = bbox[c], ext = bbox[3 + c] - lo;
    float t = ext > 0.f ? (xyz[3 * i + c] - lo) / ext : 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);  // NaN -> 0
    q[c] = (uint32_t)(t * 1023.f);
  }
  key[i] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
  val[i] = (uint32_t)i;
}

// sorted float4 points + box AABBs (one wave per box)
__global__ __launch_bounds__(kThreads) void layout_kernel(const float* __restrict__ xyz, size_t P,
                                                          const uint32_t* __restrict__ order,
                                                          float4* __restrict__ pts,
                                                          float4* __restrict__ boxes, size_t nbox) {
  const size_t box = (size_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (box >= nbox) return;  // wave-uniform
  const size_t i = box * kBox + lane_id();
  const bool valid = i < P;
  float x = 0.f, y = 0.f, z = 0.f;
  if (valid) {
    const uint32_t id = order[i];
    x = xyz[3 * (size_t)id];
    y = xyz[3 * (size_t)id + 1];
    z = xyz[3 * (size_t)id + 2];
    pts[i] = make_float4(x, y, z, __uint_as_float(id));
  }
  const float mnx = wave_min(valid ? x : FLT_MAX), mny = wave_min(valid ? y : FLT_MAX),
              mnz = wave_min(valid ? z : FLT_MAX);
  const float mxx = wave_max(valid ? x : -FLT_MAX), mxy = wave_max(valid ? y : -FLT_MAX),
              mxz = wave_max(valid ? z : -FLT_MAX);
  if (lane_id() == 0) {
    boxes[2 * box] = make_float4(mnx, mny, mnz, 0.f);
    boxes[2 * box + 1] = make_float4(mxx, mxy, mxz, 0.f);
  }
}

__global__ __launch_bounds__(kThreads) void super_kernel(const float4* __restrict__ boxes,
                                                         size_t nbox, float4* __restrict__ supers,
                                                         size_t nsup) {
  const size_t s = (size_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (s >= nsup) return;
  const size_t b = s * kSuper + lane_id();
  const bool valid = b < nbox;
  const float4 lo = valid ? boxes[2 * b] : make_float4(FLT_MAX, FLT_MAX, FLT_MAX, 0.f);
  const float4 hi = valid ? boxes[2 * b + 1] : make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f);
  const float a = wave_min(lo.x), bb = wave_min(lo.y), c = wave_min(lo.z);
  const float d = wave_max(hi.x), e = wave_max(hi.y), f = wave_max(hi.z);
  if (lane_id() == 0) {
    supers[2 * s] = make_float4(a, bb, c, 0.f);
    supers[2 * s + 1] = make_float4(d, e, f, 0.f);
  }
}

__device__ __forceinline__ float sq_dist(float dx, float dy, float dz) {
  return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// squared distance from p to an AABB (0 inside), same rounded formula as the point distance:
// every correctly rounded step is monotone, so it never exceeds the distance of a point in the box
// and skipping boxes with box_dist > third-best is exact
__device__ __forceinline__ float box_dist(float px, float py, float pz, float4 lo, float4 hi) {
  const float dx = fmaxf(fmaxf(lo.x - px, px - hi.x), 0.f);
  const float dy = fmaxf(fmaxf(lo.y - py, py - hi.y), 0.f);
  const float dz = fmaxf(fmaxf(lo.z - pz, pz - hi.z), 0.f);
  return sq_dist(dx, dy, dz);
}

struct Best3 {
  float d0, d1, d2;
  int32_t i0, i1, i2;
};

__device__ __forceinline__ bool before(float d, int32_t i, float bd, int32_t bi) {
  return d < bd || (d == bd && (uint32_t)i < (uint32_t)bi);  // index -1 sorts last
}

__device__ __forceinline__ void consider(Best3& b, float d, int32_t id) {
  if (!before(d, id, b.d2, b.i2)) return;
  if (before(d, id, b.d1, b.i1)) {
    b.d2 = b.d1; b.i2 = b.i1;
    if (before(d, id, b.d0, b.i0)) {
      b.d1 = b.d0; b.i1 = b.i0;
      b.d0 = d; b.i0 = id;
    } else {
      b.d1 = d; b.i1 = id;
    }
  } else {
    b.d2 = d; b.i2 = id;
  }
}

// scan the 64 points held one per lane (c = this lane's copy) against every lane's query point
__device__ __forceinline__ void scan_wave_points(Best3& b, float px, float py, float pz,
                                                 int32_t self, float4 c, int count) {
  for (int j = 0; j < count; j++) {
    const float cx = __shfl(c.x, j, 64), cy = __shfl(c.y, j, 64), cz = __shfl(c.z, j, 64);
    const int32_t cid = (int32_t)__float_as_uint(__shfl(c.w, j, 64));
    const float dx = cx - px, dy = cy - py, dz = cz - pz;
    const float d = sq_dist(dx, dy, dz);
    if (cid != self) consider(b, d, cid);
  }
}

__global__ __launch_bounds__(kThreads) void query_kernel(const float4* __restrict__ pts, size_t P,
                                                         const float4* __restrict__ boxes,
                                                         size_t nbox,
                                                         const float4* __restrict__ supers,
                                                         size_t nsup, float* __restrict__ mean,
                                                         int32_t* __restrict__ nn) {
  const size_t box = (size_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (box >= nbox) return;  // wave-uniform
  const size_t i = box * kBox + lane_id();
  const bool valid = i < P;
  const float4 me = valid ? pts[i] : make_float4(0.f, 0.f, 0.f, __uint_as_float(0xffffffffu));
  const float px = me.x, py = me.y, pz = me.z;
  const int32_t self = (int32_t)__float_as_uint(me.w);
  Best3 b{FLT_MAX, FLT_MAX, FLT_MAX, -1, -1, -1};
  const int own_count = (int)((P - box * kBox) < (size_t)kBox ? (P - box * kBox) : kBox);
  scan_wave_points(b, px, py, pz, self, me, own_count);
  const long own_s = (long)(box / kSuper);
  // superboxes outward from the own one: own, own+1, own-1, own+2, ...
  for (long k = 0; k < 2 * (long)nsup; k++) {
    const long s = own_s + ((k & 1) ? (k + 1) / 2 : -(k / 2));
    if (s < 0 || s >= (long)nsup) continue;
    const float sd = box_dist(px, py, pz, supers[2 * s], supers[2 * s + 1]);
    if (__ballot(valid && sd <= b.d2) == 0ull) continue;
    const size_t b0 = (size_t)s * kSuper;
    const size_t b1 = b0 + kSuper < nbox ? b0 + kSuper : nbox;
    for (size_t bb = b0; bb < b1; bb++) {
      if (bb == box) continue;
      const float bd = box_dist(px, py, pz, boxes[2 * bb], boxes[2 * bb + 1]);
      if (__ballot(valid && bd <= b.d2) == 0ull) continue;
      const size_t j = bb * kBox + lane_id();
      const int cnt = (int)((P - bb * kBox) < (size_t)kBox ? (P - bb * kBox) : kBox);
      const float4 c = j < P ? pts[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      scan_wave_points(b, px, py, pz, self, c, cnt);
    }
  }
  if (!valid) return;
  mean[self] = (b.d0 + b.d1 + b.d2) / 3.0f;
  if (nn) {
    nn[3 * (size_t)self] = b.i0;
    nn[3 * (size_t)self + 1] = b.i1;
    nn[3 * (size_t)self + 2] = b.i2;
  }
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" size_t gsr_knn_scratch_bytes(int64_t P) {
  return carve_knn(nullptr, (size_t)(P > 0 ? P : 0)).bytes;
}

extern "C" int gsr_dist_knn3(int64_t P, const float* points, float* mean_dist, int32_t* indices,
                             void* scratch, void* stream) {
  if (P < 0 || P > 0x7fffffffLL) return 1;
  if (P == 0) return 0;
  if (!points || !mean_dist || !scratch) return 1;
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)P;
  KnnState k = carve_knn((char*)scratch, n);
  const size_t nparts = (n + kBBoxTile - 1) / kBBoxTile;
  const size_t nbox = (n + kBox - 1) / kBox;
  const size_t nsup = (nbox + kSuper - 1) / kSuper;
  const size_t waves_per_group = kThreads / 64;
  hipLaunchKernelGGL(bbox_parts_kernel, dim3((unsigned)nparts), dim3(kThreads), 0, s, points, n,
                     k.bbox_parts);
  hipLaunchKernelGGL(bbox_final_kernel, dim3(1), dim3(kThreads), 0, s, k.bbox_parts, nparts,
                     k.bbox);
  hipLaunchKernelGGL(morton_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, points, n, k.bbox, k.ka, k.va);
  bool in_b = false;
  if (radix_sort_pairs(k.ka, k.va, k.kb, k.vb, n, kMortonBits, k.sort, &in_b, s) != hipSuccess)
    return 2;
  const uint32_t* order = in_b ? k.vb : k.va;
  hipLaunchKernelGGL(layout_kernel, dim3((unsigned)((nbox + waves_per_group - 1) / waves_per_group)),
                     dim3(kThreads), 0, s, points, n, order, k.pts, k.boxes, nbox);
  hipLaunchKernelGGL(super_kernel, dim3((unsigned)((nsup + waves_per_group - 1) / waves_per_group)),
                     dim3(kThreads), 0, s, k.boxes, nbox, k.supers, nsup);
  hipLaunchKernelGGL(query_kernel, dim3((unsigned)((nbox + waves_per_group - 1) / waves_per_group)),
                     dim3(kThreads), 0, s, k.pts, n, k.boxes, nbox, k.supers, nsup, mean_dist,
                     indices);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

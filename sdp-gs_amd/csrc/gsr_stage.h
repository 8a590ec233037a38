// gsr_stage.h -- cooperative global <-> LDS staging of per-Gaussian SH planes (device code).
//
// Shared by the forward preprocess (gsr_preprocess.hip, loads only) and the backward preprocess
// (gsr_backward.hip, loads + gradient stores / accumulation).
#pragma once
#include "gsr_internal.h"

namespace gsr {

// ---- SH staging ----------------------------------------------------------------------------------
// A workgroup's SH data is one contiguous segment per plane in global memory (fused: features_dc
// w = 3 floats per Gaussian and features_rest w = 3(M-1); reference layout: sh w = 3M).  Each plane
// is copied into LDS with the SAME layout, as 16-byte vectors (ds_write_b128 / ds_read_b128 at
// consecutive addresses: no bank conflicts, no index arithmetic), kStageBatch vectors in flight per
// lane.  The per-Gaussian compute then reads its row at stride w (odd for the fused planes, so
// lane-strided access is conflict-free), works in place, and the gradient plane goes back the
// same way (ACC: read-add-write).  A vector spans at most two rows (w >= 3); vectors whose rows
// are all culled are skipped in ACC mode.
constexpr int kShMaxFloats = 48;  // 16 coefficients x 3 per Gaussian (M <= 16, checked by the API)
#ifndef GSR_STAGE_BATCH
#define GSR_STAGE_BATCH 4
#endif
constexpr int kStageBatch = GSR_STAGE_BATCH;

// 1: the staged global rows are loaded and stored nontemporally (read / written once per step,
// larger than the caches) -- and so are sh_precolor's per-view outputs
#ifndef GSR_STAGE_NT
#define GSR_STAGE_NT 1
#endif
__device__ __forceinline__ float4 stream_ld4(const float4* p) {
  if (GSR_STAGE_NT) {
    const float* f = reinterpret_cast<const float*>(p);
    return make_float4(__builtin_nontemporal_load(f), __builtin_nontemporal_load(f + 1),
                       __builtin_nontemporal_load(f + 2), __builtin_nontemporal_load(f + 3));
  }
  return *p;
}
__device__ __forceinline__ void stream_st4(float4* p, float4 v) {
  if (GSR_STAGE_NT) {
    float* f = reinterpret_cast<float*>(p);
    __builtin_nontemporal_store(v.x, f);
    __builtin_nontemporal_store(v.y, f + 1);
    __builtin_nontemporal_store(v.z, f + 2);
    __builtin_nontemporal_store(v.w, f + 3);
    return;
  }
  *p = v;
}
template <typename T>
__device__ __forceinline__ void stream_st(T* p, T v) {
  if (GSR_STAGE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

struct ShPlane {
  const float* src;  // global input plane (row-major [P, w])
  float* dst;        // global gradient plane
  int w;             // floats per Gaussian
  int lds;           // float offset of the plane in the LDS buffer
};

__device__ __forceinline__ uint32_t div_small(uint32_t e, uint32_t magic) {
  return __umulhi(e, magic);  // e / w for e < 2^32 / w^2 with magic = ceil(2^32 / w)
}

// global <-> LDS copy of one plane segment; IN: global -> LDS, else LDS -> global (ACC: add)
template <int NT, bool IN, bool ACC>
__device__ __forceinline__ void stage(const ShPlane& p, int base, int n, const uint8_t* live,
                                      float* lds) {
  if (p.w == 0) return;
  const uint32_t w = (uint32_t)p.w;
  // e / w by multiply-high (w = 1: the identity; its magic 2^32 does not fit 32 bits)
  const uint32_t magic = w == 1 ? 0u : (uint32_t)((0x100000000ull + w - 1) / w);
  auto row = [&](uint32_t e) { return w == 1 ? e : div_small(e, magic); };
  const size_t gofs = (size_t)base * w;
  const float* src = p.src + gofs;
  float* dst = p.dst + gofs;
  float* l = lds + p.lds;
  const int total = n * p.w;
  const bool vec_ok = ((((uintptr_t)(IN ? (const void*)src : (const void*)dst)) & 15) == 0);
  const int nvec = vec_ok ? (total >> 2) : 0;
  // in ACC mode (or when loading) vectors covering only culled rows are skipped
  auto needed = [&](int q) {
    return live[row(4u * q)] || live[row(4u * q + 3u)];
  };
  for (int q0 = (int)threadIdx.x; q0 < nvec; q0 += kStageBatch * NT) {
    float4 v[kStageBatch], o[kStageBatch];
    bool on[kStageBatch];
#pragma unroll
    for (int j = 0; j < kStageBatch; j++) {
      const int q = q0 + j * NT;
      on[j] = q < nvec && (!(IN || ACC) || needed(q));
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      o[j] = v[j];
      if (on[j]) {
        if (IN) {
          v[j] = stream_ld4(reinterpret_cast<const float4*>(src) + q);
        } else {
          v[j] = reinterpret_cast<const float4*>(l)[q];
          if (ACC) o[j] = stream_ld4(reinterpret_cast<const float4*>(dst) + q);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kStageBatch; j++) {
      const int q = q0 + j * NT;
      if (on[j]) {
        if (IN) {
          reinterpret_cast<float4*>(l)[q] = v[j];
        } else {
          float4 r = v[j];
          if (ACC) r = make_float4(o[j].x + r.x, o[j].y + r.y, o[j].z + r.z, o[j].w + r.w);
          stream_st4(reinterpret_cast<float4*>(dst) + q, r);
        }
      }
    }
  }
  // scalar tail (everything when the global pointer is not 16-byte aligned)
  for (int e = 4 * nvec + (int)threadIdx.x; e < total; e += NT) {
    if (IN) l[e] = src[e];
    else if (ACC) { if (live[row((uint32_t)e)]) dst[e] += l[e]; }
    else dst[e] = l[e];
  }
}


}  // namespace gsr

// gsr_sh.h -- spherical-harmonics colour, its basis and its direction Jacobian (device code),
// shared by the forward preprocess, the backward preprocess, the multi-view colour pre-pass and
// the deferred SH-gradient flush, so that every path evaluates the same float expressions in the
// same order (the reference's forward.cu:20-71 and backward.cu:20-139).
#pragma once
#include "gsr_device.h"

namespace gsr {

// forward.cu:20-71 (float32, same evaluation order as the CPU restatement)
// s0: coefficient 0 of this Gaussian, s1: its coefficients 1.. (contiguous); for the reference's
// [P,M,3] layout s1 = s0 + 3, for the fused split layout s0 = features_dc, s1 = features_rest.
// (coefficient k of the row from SH(k): LDS rows or registers, the same operations either way)
template <class ShAt>
__device__ __forceinline__ V3 sh_to_rgb_at(ShAt SH, int deg, V3 dir, uint8_t& clamped) {
  V3 result = SH_C0 * SH(0);
  if (deg > 0) {
    const float x = dir.x, y = dir.y, z = dir.z;
    result = ((result - (SH_C1 * y) * SH(1)) + (SH_C1 * z) * SH(2)) - (SH_C1 * x) * SH(3);
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z;
      const float xy = x * y, yz = y * z, xz = x * z;
      result = result + (SH_C2_0 * xy) * SH(4);
      result = result + (SH_C2_1 * yz) * SH(5);
      result = result + (SH_C2_2 * (2.0f * zz - xx - yy)) * SH(6);
      result = result + (SH_C2_3 * xz) * SH(7);
      result = result + (SH_C2_4 * (xx - yy)) * SH(8);
      if (deg > 2) {
        result = result + (SH_C3_0 * y * (3.0f * xx - yy)) * SH(9);
        result = result + (SH_C3_1 * xy * z) * SH(10);
        result = result + (SH_C3_2 * y * (4.0f * zz - xx - yy)) * SH(11);
        result = result + (SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * SH(12);
        result = result + (SH_C3_4 * x * (4.0f * zz - xx - yy)) * SH(13);
        result = result + (SH_C3_5 * z * (xx - yy)) * SH(14);
        result = result + (SH_C3_6 * x * (xx - 3.0f * yy)) * SH(15);
      }
    }
  }
  result = v3(result.x + 0.5f, result.y + 0.5f, result.z + 0.5f);
  clamped = (uint8_t)((result.x < 0) | ((result.y < 0) << 1) | ((result.z < 0) << 2));
  return v3(fmaxf(result.x, 0.0f), fmaxf(result.y, 0.0f), fmaxf(result.z, 0.0f));
}
__device__ __forceinline__ V3 sh_to_rgb(const float* __restrict__ s0, const float* __restrict__ s1,
                                        int deg, V3 dir, uint8_t& clamped) {
  return sh_to_rgb_at(
      [&](int k) {
        return k == 0 ? v3(s0[0], s0[1], s0[2])
                      : v3(s1[3 * (k - 1)], s1[3 * (k - 1) + 1], s1[3 * (k - 1) + 2]);
      },
      deg, dir, clamped);
}

// dRGB/dsh_k for a normalised direction (backward.cu:36-76): the SH gradient of a view is
// basis_k(dir) x dL/dRGB.
__device__ __forceinline__ void sh_basis_dir(V3 dir, int deg, float (&b)[16]) {
  const float x = dir.x, y = dir.y, z = dir.z;
#pragma unroll
  for (int k = 0; k < 16; k++) b[k] = 0.0f;
  b[0] = SH_C0;
  if (deg > 0) {
    b[1] = -SH_C1 * y;
    b[2] = SH_C1 * z;
    b[3] = -SH_C1 * x;
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z;
      const float xy = x * y, yz = y * z, xz = x * z;
      b[4] = SH_C2_0 * xy;
      b[5] = SH_C2_1 * yz;
      b[6] = SH_C2_2 * (2.f * zz - xx - yy);
      b[7] = SH_C2_3 * xz;
      b[8] = SH_C2_4 * (xx - yy);
      if (deg > 2) {
        b[9] = SH_C3_0 * y * (3.f * xx - yy);
        b[10] = SH_C3_1 * xy * z;
        b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
        b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
        b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
        b[14] = SH_C3_5 * z * (xx - yy);
        b[15] = SH_C3_6 * x * (xx - 3.f * yy);
      }
    }
  }
}

// the same for an unnormalised direction (mean - campos), normalised as backward.cu:26-27
__device__ __forceinline__ void sh_basis(V3 dir_orig, int deg, float (&b)[16]) {
  const float len = sqrtf(dot3(dir_orig, dir_orig));
  sh_basis_dir(v3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len), deg, b);
}

// dRGB/ddir (three vec3 over the colour channels) of the SH colour at a normalised direction,
// backward.cu:56-131 (the products and sums in the reference's order).
__device__ __forceinline__ void sh_dir_jacobian(const V3 (&c)[16], int deg, V3 dir, V3& dRGBdx,
                                                V3& dRGBdy, V3& dRGBdz) {
#define SH(k) c[k]
  dRGBdx = v3(0, 0, 0); dRGBdy = v3(0, 0, 0); dRGBdz = v3(0, 0, 0);
  const float x = dir.x, y = dir.y, z = dir.z;
  if (deg > 0) {
    dRGBdx = -SH_C1 * SH(3);
    dRGBdy = -SH_C1 * SH(1);
    dRGBdz = SH_C1 * SH(2);
    if (deg > 1) {
      const float xx = x * x, yy = y * y, zz = z * z;
      const float xy = x * y, yz = y * z, xz = x * z;
      const V3 tx = (((SH_C2_0 * y) * SH(4) + (SH_C2_2 * 2.f * -x) * SH(6)) + (SH_C2_3 * z) * SH(7)) +
                    (SH_C2_4 * 2.f * x) * SH(8);
      const V3 ty = (((SH_C2_0 * x) * SH(4) + (SH_C2_1 * z) * SH(5)) + (SH_C2_2 * 2.f * -y) * SH(6)) +
                    (SH_C2_4 * 2.f * -y) * SH(8);
      const V3 tz = ((SH_C2_1 * y) * SH(5) + (SH_C2_2 * 2.f * 2.f * z) * SH(6)) + (SH_C2_3 * x) * SH(7);
      dRGBdx = dRGBdx + tx;
      dRGBdy = dRGBdy + ty;
      dRGBdz = dRGBdz + tz;
      if (deg > 2) {
        // backward.cu:99-122: (scalar * vec3) followed by vec3 * scalar products, summed left to right
        V3 ax = (((SH_C3_0 * SH(9)) * 3.f) * 2.f) * xy;
        ax = ax + (SH_C3_1 * SH(10)) * yz;
        ax = ax + ((SH_C3_2 * SH(11)) * -2.f) * xy;
        ax = ax + (((SH_C3_3 * SH(12)) * -3.f) * 2.f) * xz;
        ax = ax + (SH_C3_4 * SH(13)) * (-3.f * xx + 4.f * zz - yy);
        ax = ax + ((SH_C3_5 * SH(14)) * 2.f) * xz;
        ax = ax + ((SH_C3_6 * SH(15)) * 3.f) * (xx - yy);
        V3 ay = ((SH_C3_0 * SH(9)) * 3.f) * (xx - yy);
        ay = ay + (SH_C3_1 * SH(10)) * xz;
        ay = ay + (SH_C3_2 * SH(11)) * (-3.f * yy + 4.f * zz - xx);
        ay = ay + (((SH_C3_3 * SH(12)) * -3.f) * 2.f) * yz;
        ay = ay + ((SH_C3_4 * SH(13)) * -2.f) * xy;
        ay = ay + ((SH_C3_5 * SH(14)) * -2.f) * yz;
        ay = ay + (((SH_C3_6 * SH(15)) * -3.f) * 2.f) * xy;
        V3 az = (SH_C3_1 * SH(10)) * xy;
        az = az + (((SH_C3_2 * SH(11)) * 4.f) * 2.f) * yz;
        az = az + ((SH_C3_3 * SH(12)) * 3.f) * (2.f * zz - xx - yy);
        az = az + (((SH_C3_4 * SH(13)) * 4.f) * 2.f) * xz;
        az = az + (SH_C3_5 * SH(14)) * (xx - yy);
        dRGBdx = dRGBdx + ax;
        dRGBdy = dRGBdy + ay;
        dRGBdz = dRGBdz + az;
      }
    }
  }
#undef SH
}

// auxiliary.h:107-117 dnormvdv: gradient through dir = v / |v|
__device__ __forceinline__ V3 dnormvdv(V3 v, V3 dv) {
  const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  return v3(((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
            (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
            (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

}  // namespace gsr

// gsr_device.h -- per-Gaussian device maths for the gfx950 rasterizer.
//
// Semantics follow the reference CUDA rasterizer (paths relative to
// /root/reference/submodules/diff-gaussian-rasterization/): auxiliary.h:21-164 (helpers, SH
// constants), forward.cu:20-152 (SH colour, 2D/3D covariance) and backward.cu:20-341 (their
// gradients).  The reference evaluates its 3x3 maths with glm (column-major, left-to-right sums);
// the helpers below keep that evaluation order so float32 results match the CPU restatement in
// oracle/ bit for bit (the library is compiled with -ffp-contract=off; expf is the only libm call
// whose last bit may differ).  This is fresh code for wave64 CDNA4, not a translation of the
// reference's glm-based device functions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsr_internal.h"

namespace gsr {

__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

// Grid-stride share of a SideClear (gsr_internal.h) for thread `tid` of `nthreads`.
// GSR_CLEAR_NT: the zeroes are stored nontemporally (the accumulator rows are next touched by the
// backward blend's atomics, long after)
#ifndef GSR_CLEAR_NT
#define GSR_CLEAR_NT 0
#endif
__device__ __forceinline__ void side_clear(void* p, size_t bytes, size_t tid, size_t nthreads) {
  if (!p) return;
  uint4* q = reinterpret_cast<uint4*>(p);
  const size_t n16 = bytes >> 4;
  for (size_t i = tid; i < n16; i += nthreads) {
#if GSR_CLEAR_NT
    uint32_t* f = reinterpret_cast<uint32_t*>(q + i);
    __builtin_nontemporal_store(0u, f);
    __builtin_nontemporal_store(0u, f + 1);
    __builtin_nontemporal_store(0u, f + 2);
    __builtin_nontemporal_store(0u, f + 3);
#else
    q[i] = make_uint4(0u, 0u, 0u, 0u);
#endif
  }
  uint32_t* w = reinterpret_cast<uint32_t*>(p);
  const size_t tail = (bytes & 15u) >> 2;
  if (tid < tail) w[4 * n16 + tid] = 0u;
}

struct V3 { float x, y, z; };
struct M3 { float m[3][3]; };  // m[col][row], glm::mat3 convention

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot3(V3 a, V3 b) {
  float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return tx + ty + tz;
}

__device__ __forceinline__ M3 m3_cols(float a0, float a1, float a2, float b0, float b1, float b2,
                                      float c0, float c1, float c2) {
  M3 r;
  r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
  r.m[1][0] = b0; r.m[1][1] = b1; r.m[1][2] = b2;
  r.m[2][0] = c0; r.m[2][1] = c1; r.m[2][2] = c2;
  return r;
}
// glm mat3*mat3: R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2]
__device__ __forceinline__ M3 m3_mul(const M3& a, const M3& b) {
  M3 r;
#pragma unroll
  for (int c = 0; c < 3; c++)
#pragma unroll
    for (int w = 0; w < 3; w++) {
      float t0 = a.m[0][w] * b.m[c][0];
      float t1 = a.m[1][w] * b.m[c][1];
      float t2 = a.m[2][w] * b.m[c][2];
      r.m[c][w] = t0 + t1 + t2;
    }
  return r;
}
__device__ __forceinline__ M3 m3_T(const M3& a) {
  M3 r;
#pragma unroll
  for (int c = 0; c < 3; c++)
#pragma unroll
    for (int w = 0; w < 3; w++) r.m[c][w] = a.m[w][c];
  return r;
}

// HIP float->int conversion (v_cvt_i32_f32) truncates and saturates, NaN -> 0: the same as the
// reference's CUDA cvt.rzi; written explicitly so the compiler cannot assume an in-range value.
__device__ __forceinline__ int f2i_sat(float f) {
  if (f != f) return 0;
  if (f >= 2147483648.0f) return 2147483647;
  if (f <= -2147483648.0f) return -2147483647 - 1;
  return (int)f;
}

// auxiliary.h:41-44 (double promotion is part of the reference's numerics)
__device__ __forceinline__ float ndc2pix(float v, int S) {
  return (float)((((double)v + 1.0) * S - 1.0) * 0.5);
}

// auxiliary.h:46-56: tile rectangle [min, max) of a splat, clamped to the tile grid.
__device__ __forceinline__ void tile_rect(float px, float py, int r, uint32_t gx, uint32_t gy,
                                          uint32_t& x0, uint32_t& y0, uint32_t& x1, uint32_t& y1) {
  int a = f2i_sat((px - (float)r) / (float)kTile);
  int b = f2i_sat((py - (float)r) / (float)kTile);
  int c = f2i_sat((((px + (float)r) + (float)kTile) - 1.0f) / (float)kTile);
  int d = f2i_sat((((py + (float)r) + (float)kTile) - 1.0f) / (float)kTile);
  a = a > 0 ? a : 0; b = b > 0 ? b : 0; c = c > 0 ? c : 0; d = d > 0 ? d : 0;
  x0 = min((uint32_t)a, gx); y0 = min((uint32_t)b, gy);
  x1 = min((uint32_t)c, gx); y1 = min((uint32_t)d, gy);
}

// ---- GaussianModel activations (scene/gaussian_model.py:33-41), for the fused-activation path ----
// torch.nn.functional.normalize(r, dim=1): r / max(||r||_2, 1e-12).  torch's row norm of 4 floats
// sums the squares pairwise, (x^2 + y^2) + (z^2 + w^2) (its vectorised reduction's two
// accumulators); this order reproduces F.normalize bit for bit (scripts/probe_activations.py on
// MI355X: 0 of 4M rows differ; the sequential sum differed in 12 %)
__device__ __forceinline__ float quat_norm(float4 r) {
  const float a = r.x * r.x + r.y * r.y;
  const float b = r.z * r.z + r.w * r.w;
  return sqrtf(a + b);
}
__device__ __forceinline__ float4 normalize_quat(float4 r) {
  const float d = fmaxf(quat_norm(r), 1e-12f);
  return make_float4(r.x / d, r.y / d, r.z / d, r.w / d);
}
// backward of normalize: dL/dr = go/d - (sum(go * r) / d^2) * r / n   (n = ||r||, d = max(n, eps))
__device__ __forceinline__ float4 normalize_quat_backward(float4 r, float4 go) {
  const float n = quat_norm(r);
  const float d = fmaxf(n, 1e-12f);
  const float s = (go.x * r.x + go.y * r.y + go.z * r.z + go.w * r.w) / (d * d);
  const float k = (n > 1e-12f && n > 0.0f) ? s / n : 0.0f;
  return make_float4(go.x / d - k * r.x, go.y / d - k * r.y, go.z / d - k * r.z,
                     go.w / d - k * r.w);
}
// torch.sigmoid on float: 1 / (1 + exp(-x)); backward: go * (1 - y) * y
// exp for the blends' Gaussian weight G = exp(power) (forward.cu:343, backward.cu:498 call expf).
// A deterministic single-precision exp: Cody-Waite reduction by ln 2 and a degree-5 polynomial
// (Cephes expf coefficients), every step a correctly rounded IEEE operation (explicit fma, no
// hardware exp approximation).  Its error is <= 1.01 ulp of exp over [-87, 0] (~90 % correctly
// rounded; the reference's CUDA expf is specified to 2 ulp), and the oracle evaluates the SAME
// sequence (the CPU restatement's splat_exp), so GPU and oracle take identical alpha >= 1/255 and
// T < 1e-4 decisions on every pixel -- with a libm / OCML expf pair a 1-ulp disagreement at a
// threshold flips a pixel at 5M Gaussians x 1080p.  Below -104 it returns 0 (alpha < 1/255 there
// for any opacity); the blends never use power > 0.
__device__ __forceinline__ float splat_exp(float x) {
  const float k = __builtin_rintf(x * 1.44269504088896341f);
  float r = __builtin_fmaf(-k, 0.693359375f, x);
  r = __builtin_fmaf(-k, -2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = __builtin_fmaf(p, r, 1.3981999507e-3f);
  p = __builtin_fmaf(p, r, 8.3334519073e-3f);
  p = __builtin_fmaf(p, r, 4.1665795894e-2f);
  p = __builtin_fmaf(p, r, 1.6666665459e-1f);
  p = __builtin_fmaf(p, r, 5.0000001201e-1f);
  const float r2 = r * r;
  const float y = __builtin_fmaf(p, r2, r) + 1.0f;
  const float res = __builtin_amdgcn_ldexpf(y, (int)k);
  return x < -104.0f ? 0.0f : res;
}
// splat_exp of N independent arguments, its steps interleaved across the N chains (the same
// operations per element, so bit-identical to N splat_exp calls): one wave then has N independent
// instructions in flight per step instead of one 15-deep dependent chain per argument
template <int N>
__device__ __forceinline__ void splat_exp_n(const float (&x)[N], float (&out)[N]) {
  float k[N], r[N], p[N];
#pragma unroll
  for (int i = 0; i < N; i++) k[i] = __builtin_rintf(x[i] * 1.44269504088896341f);
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = __builtin_fmaf(-k[i], 0.693359375f, x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = __builtin_fmaf(-k[i], -2.12194440e-4f, r[i]);
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = __builtin_fmaf(1.9875691500e-4f, r[i], 1.3981999507e-3f);
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = __builtin_fmaf(p[i], r[i], 8.3334519073e-3f);
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = __builtin_fmaf(p[i], r[i], 4.1665795894e-2f);
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = __builtin_fmaf(p[i], r[i], 1.6666665459e-1f);
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = __builtin_fmaf(p[i], r[i], 5.0000001201e-1f);
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float y = __builtin_fmaf(p[i], r[i] * r[i], r[i]) + 1.0f;
    const float res = __builtin_amdgcn_ldexpf(y, (int)k[i]);
    out[i] = x[i] < -104.0f ? 0.0f : res;
  }
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// Natural log for the culling threshold q_cut (positive normal x only): Cephes logf -- frexp to
// m in [sqrt(1/2), sqrt(2)), a degree-8 polynomial in m - 1 and the split ln 2 -- every step an
// explicit IEEE operation, as splat_exp.  The CPU restatement evaluates the same sequence, so
// the tests can pin the kept tile instances bit for bit;
// its error (~1 ulp) is irrelevant next to the 2e-2 margin of the band cut below.
__device__ __forceinline__ float splat_log(float x) {
  int e;
  float m = __builtin_frexpf(x, &e);  // x = m 2^e, m in [0.5, 1)
  if (m < 0.707106781186547524f) {
    e -= 1;
    m = (m + m) - 1.0f;
  } else {
    m = m - 1.0f;
  }
  const float z = m * m;
  float y = 7.0376836292e-2f;
  y = __builtin_fmaf(y, m, -1.1514610310e-1f);
  y = __builtin_fmaf(y, m, 1.1676998740e-1f);
  y = __builtin_fmaf(y, m, -1.2420140846e-1f);
  y = __builtin_fmaf(y, m, 1.4249322787e-1f);
  y = __builtin_fmaf(y, m, -1.6668057665e-1f);
  y = __builtin_fmaf(y, m, 2.0000714765e-1f);
  y = __builtin_fmaf(y, m, -2.4999993993e-1f);
  y = __builtin_fmaf(y, m, 3.3333331174e-1f);
  y = (y * m) * z;
  const float fe = (float)e;
  y = __builtin_fmaf(fe, -2.12194440e-4f, y);
  y = __builtin_fmaf(-0.5f, z, y);
  const float r = m + y;
  return __builtin_fmaf(fe, 0.693359375f, r);
}

// ---- conservative splat / pixel-rectangle culling ----------------------------------------------
// The blend skips a (splat, pixel) pair when alpha = min(0.99, op * exp(power)) < 1/255 with
// power = -q/2, q = ca dx^2 + 2 cb dx dy + cc dy^2 (forward.cu:335-345).  A splat that fails that
// test at EVERY pixel centre of a rectangle changes no output bit there, so it may be dropped from
// the rectangle's list.  `q_cut` is the squared Mahalanobis radius beyond which alpha < 1/255,
// or a negative value when nothing can be culled (conic not positive definite) and -2 when the
// splat can never reach 1/255 (op < 1/255: max alpha is op at power = 0).
__device__ __forceinline__ float splat_q_cut(float ca, float cb, float cc, float op) {
  if (!(op >= 1.0f / 255.0f)) return -2.0f;
  if (!(ca > 0.0f && cc > 0.0f && ca * cc - cb * cb > 0.0f)) return -1.0f;
  // 255 op >= 1: a positive normal float
  return 2.0f * splat_log(255.0f * op);
}

// ---- band form of the cut: the binning's tile ranges and the blends' per-wave list masks --------
// Every consumer asks the same question of a splat: which cells of a grid of pixel rectangles can
// it reach with alpha >= 1/255 -- the binning per tile (16 x 16), the forward per 4x4 block, the
// backward per 8x4 wave half.  The cells come in bands of pixel rows, so the x-extent of the
// ellipse q <= Q inside each band is found once (two square roots) and every cell of the band is
// an interval overlap.  Q widens q_cut by the margin 2e-2 + 1e-4 |terms| (|terms| <= Q ta on the
// ellipse), far above the float error of the blend's own evaluation (dx = mx - px carries up to
// ulp(2048) = 2.4e-4 px, i.e. |dq| <= 2 sqrt(ca q) 2.4e-4 < 3e-3 for q <= 11, ca <= 1/0.3), and
// the extents get a pixel slack for their own float evaluation: a superset of the cells where any
// pixel centre can reach alpha >= 1/255.  The blends' lists only decide which work is done, never
// an output bit; the binning's ranges are restated by the oracle operation for operation and every
// dropped instance is checked against the reference's own test (tests/test_index_parity.py).
struct BandCut {
  float mx, my, ica, cb, det, caQ, hx, hy, dyl, slack;
  int mode;  // 0: none reachable (q_cut -2), 1: every group (not positive definite / degenerate), 2: test
};
__device__ __forceinline__ BandCut make_band_cut(float mx, float my, float ca, float cb, float cc,
                                                 float qc) {
  BandCut s{};
  s.mx = mx; s.my = my;
  if (qc == -2.0f) { s.mode = 0; return s; }
  s.mode = 1;
  if (qc < 0.0f) return s;
  const float det = ca * cc - cb * cb;
  if (!(det > 0.0f)) return s;
  const float h2x = cc / det, h2y = ca / det;  // (half-extent)^2 per unit Q
  const float ta = ca * h2x + cc * h2y + 2.0f * fabsf(cb) * sqrtf(h2x * h2y);
  if (!(1e-4f * ta < 0.5f)) return s;
  const float Q = (qc + 2e-2f) / (1.0f - 1e-4f * ta) * 1.001f;
  s.mode = 2;
  s.ica = 1.0f / ca;
  s.cb = cb;
  s.det = det;
  s.caQ = ca * Q;
  s.hx = sqrtf(Q * h2x) * 1.001f + 1e-3f;
  s.hy = sqrtf(Q * h2y) * 1.001f + 1e-3f;
  s.dyl = cb * (s.hx / cc);  // dy of the leftmost point (the rightmost one is at -dyl)
  s.slack = 2e-3f + 4e-6f * fabsf(mx) + 1e-4f * s.hx;
  return s;
}
// The blends' form of the same cut: hardware reciprocals (v_rcp_f32, ~1 ulp) in place of the five
// IEEE divisions (~10 instructions each), on every list entry of every tile of both blends.  Its
// Q, hx, hy, 1/ca and dyl differ from make_band_cut's by a few ulp, against margins of 2e-2 on Q,
// 1e-3 px on the half-extents and 2e-3 px of slack (above), so the cells it keeps are still a
// superset of those any pixel centre can reach with alpha >= 1/255; a non-finite reciprocal (a
// denormal conic term) falls back to "every cell".  The binning keeps make_band_cut, which the
// oracle restates operation for operation.
__device__ __forceinline__ BandCut make_band_cut_fast(float mx, float my, float ca, float cb,
                                                      float cc, float qc) {
  BandCut s{};
  s.mx = mx; s.my = my;
  if (qc == -2.0f) { s.mode = 0; return s; }
  s.mode = 1;
  if (qc < 0.0f) return s;
  const float det = ca * cc - cb * cb;
  if (!(det > 0.0f)) return s;
  const float idet = __builtin_amdgcn_rcpf(det), ica = __builtin_amdgcn_rcpf(ca),
              icc = __builtin_amdgcn_rcpf(cc);
  if (!(idet < 3.0e38f && ica < 3.0e38f && icc < 3.0e38f)) return s;
  const float h2x = cc * idet, h2y = ca * idet;
  const float ta = ca * h2x + cc * h2y + 2.0f * fabsf(cb) * sqrtf(h2x * h2y);
  if (!(1e-4f * ta < 0.5f)) return s;
  const float Q = (qc + 2e-2f) * __builtin_amdgcn_rcpf(1.0f - 1e-4f * ta) * 1.001f;
  s.mode = 2;
  s.ica = ica;
  s.cb = cb;
  s.det = det;
  s.caQ = ca * Q;
  s.hx = sqrtf(Q * h2x) * 1.001f + 1e-3f;
  s.hy = sqrtf(Q * h2y) * 1.001f + 1e-3f;
  s.dyl = cb * (s.hx * icc);
  s.slack = 2e-3f + 4e-6f * fabsf(mx) + 1e-4f * s.hx;
  return s;
}
// The ellipse's x-extent [xl, xr] (relative to mx, slack included) over the pixel-centre rows
// [y0, y1]; false when it misses the band.
__device__ __forceinline__ bool band_extent(const BandCut& s, float y0, float y1, float& xl,
                                            float& xr) {
  const float lo = fmaxf(y0 - s.my, -s.hy), hi = fminf(y1 - s.my, s.hy);
  if (lo > hi) return false;
  // x-roots of the line dy: (-cb dy -+ sqrt(ca Q - det dy^2)) / ca
  const float rl = sqrtf(fmaxf(s.caQ - s.det * lo * lo, 0.0f));
  const float rh = sqrtf(fmaxf(s.caQ - s.det * hi * hi, 0.0f));
  const float cl = -s.cb * lo, ch = -s.cb * hi;
  xl = fminf(cl - rl, ch - rh) * s.ica;
  xr = fmaxf(cl + rl, ch + rh) * s.ica;
  if (s.dyl >= lo && s.dyl <= hi) xl = -s.hx;   // the leftmost point lies in the band
  if (-s.dyl >= lo && -s.dyl <= hi) xr = s.hx;  // the rightmost point lies in the band
  xl -= s.slack;
  xr += s.slack;
  return true;
}

// The binning's cut (the preprocess counts, the duplication emits): per tile row of the splat's
// rectangle [x0, x1), the tiles [a, b) the ellipse's x-extent in the row's 16-pixel band meets --
// one contiguous range by construction, O(1) per row.  Empty rows give a = b = x1.
__device__ __forceinline__ void band_row_range(const BandCut& s, uint32_t ty, uint32_t x0,
                                               uint32_t x1, uint32_t& a, uint32_t& b) {
  if (s.mode != 2) {
    a = x0;
    b = s.mode == 0 ? x0 : x1;
    return;
  }
  const float y0 = (float)(ty * kTile);
  float xl, xr;
  if (!band_extent(s, y0, y0 + (float)(kTile - 1), xl, xr)) {
    a = b = x1;
    return;
  }
  // tile t (pixel columns 16 t .. 16 t + 15) is met iff 16 t <= mx + xr and 16 t + 15 >= mx + xl
  const float fa = fminf(fmaxf(ceilf((s.mx + xl - (float)(kTile - 1)) * (1.0f / kTile)), (float)x0), (float)x1);
  const float fb = fminf(fmaxf(floorf((s.mx + xr) * (1.0f / kTile)) + 1.0f, (float)x0), (float)x1);
  a = (uint32_t)fa;
  b = (uint32_t)fb;
  if (a >= b) a = b = x1;
}

// auxiliary.h:58-77 (the 4x4 matrices are row-major tensors read as column-major)
__device__ __forceinline__ V3 xform_point43(V3 p, const float* m) {
  return v3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
            m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float xform_w(V3 p, const float* m) {
  return m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}
// auxiliary.h:89-97
__device__ __forceinline__ V3 xform_vec43_T(V3 p, const float* m) {
  return v3(m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z);
}

// forward.cu:118-152: Sigma = (S R)^T (S R), quaternion (w,x,y,z) NOT normalised in-kernel.
__device__ __forceinline__ void cov3d_from_scale_rot(float sx, float sy, float sz, float mod,
                                                     float r, float x, float y, float z,
                                                     float out[6]) {
  M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
  S.m[0][0] = mod * sx;
  S.m[1][1] = mod * sy;
  S.m[2][2] = mod * sz;
  M3 R = m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
  M3 M = m3_mul(S, R);
  M3 Sig = m3_mul(m3_T(M), M);
  out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
  out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

// EWA projection of a world covariance (forward.cu:74-113 and the recomputation at
// backward.cu:166-199).  Returns T = W*J (for the backward) and the un-filtered 2D covariance.
struct Ewa {
  M3 T, W, Vrk;
  V3 t;             // clamped view-space mean
  float txtz, tytz, limx, limy;
  float a, b, c;    // 2D covariance with the +0.3 low-pass on the diagonal
};
__device__ __forceinline__ Ewa ewa_project(V3 mean, float fx, float fy, float tanx, float tany,
                                           const float* c3, const float* view) {
  Ewa e;
  V3 t = xform_point43(mean, view);
  e.limx = 1.3f * tanx;
  e.limy = 1.3f * tany;
  e.txtz = t.x / t.z;
  e.tytz = t.y / t.z;
  t.x = fminf(e.limx, fmaxf(-e.limx, e.txtz)) * t.z;
  t.y = fminf(e.limy, fmaxf(-e.limy, e.tytz)) * t.z;
  e.t = t;
  M3 J = m3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z,
                 -(fy * t.y) / (t.z * t.z), 0, 0, 0);
  e.W = m3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
  e.T = m3_mul(e.W, J);
  e.Vrk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
  M3 cov = m3_mul(m3_mul(m3_T(e.T), m3_T(e.Vrk)), e.T);
  e.a = cov.m[0][0] + 0.3f;
  e.b = cov.m[0][1];
  e.c = cov.m[1][1] + 0.3f;
  return e;
}

}  // namespace gsr

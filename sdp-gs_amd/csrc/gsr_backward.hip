// gsr_backward.hip -- fused per-Gaussian backward preprocess for gfx950.
//
// One launch replaces the reference's two per-Gaussian backward kernels, computeCov2DCUDA
// (cuda_rasterizer/backward.cu:144-274) and preprocessCUDA (:346-396, with
// computeColorFromSH-bwd :20-139 and computeCov3D-bwd :278-341), plus the grad zero-fill of
// RasterizeGaussiansBackwardCUDA (rasterize_points.cu:151-159): every output element is written
// exactly once (zeros for culled Gaussians), so the caller may hand in uninitialised buffers.
// Inputs come from the 64-byte accumulator row the backward blend filled (gsr_internal.h AccSlot).
#include "gsr_device.h"
#include "gsr_internal.h"
#include "gsr_sh.h"
#include "gsr_stage.h"

namespace gsr {
namespace {

#ifndef GSR_BWD_THREADS
#define GSR_BWD_THREADS 256
#endif
constexpr int kThreads = GSR_BWD_THREADS;  // Gaussians per workgroup (LDS staging: 192 B each)

__device__ __forceinline__ void put3(float* p, size_t i, V3 v) {
  p[3 * i] = v.x; p[3 * i + 1] = v.y; p[3 * i + 2] = v.z;
}
// planar [3][P] store (the deferred dL/dRGB: every store instruction of a wave is one contiguous
// 256-byte run, and so is every load of the step's SH flush)
__device__ __forceinline__ void put3p(float* p, size_t P, size_t i, V3 v) {
  p[i] = v.x; p[P + i] = v.y; p[2 * P + i] = v.z;
}
// store or accumulate (fused path with accumulate = 1 adds into existing .grad buffers)
template <bool ACC>
__device__ __forceinline__ void st(float* p, float v) {
  if (ACC) *p += v; else *p = v;
}
template <bool ACC>
__device__ __forceinline__ void st3(float* p, size_t i, V3 v) {
  st<ACC>(p + 3 * i, v.x); st<ACC>(p + 3 * i + 1, v.y); st<ACC>(p + 3 * i + 2, v.z);
}

// backward.cu:20-139: writes dL/dsh for coefficient k < (deg+1)^2 and returns dL/dmean.
// s0: coefficient 0 of this Gaussian, s1: its coefficients 1.. (rows of the LDS staging planes);
// the gradients go to the same places.  The used coefficients are read into registers first, so
// the computation is in place.
template <bool WRITE = true>
__device__ __forceinline__ V3 sh_backward(float* s0, float* s1, int deg, V3 dir_orig,
                                          V3 dL_dRGB) {
  V3 c[16];
  const int ncoef_used = (deg + 1) * (deg + 1);
  c[0] = v3(s0[0], s0[1], s0[2]);
#pragma unroll
  for (int k = 1; k < 16; k++)
    c[k] = k < ncoef_used ? v3(s1[3 * k - 3], s1[3 * k - 2], s1[3 * k - 1]) : v3(0, 0, 0);
  const float len = sqrtf(dot3(dir_orig, dir_orig));
  const V3 dir = v3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
  if (WRITE) {
    float b[16];
    sh_basis_dir(dir, deg, b);
    float* d = s0;
    d[0] = b[0] * dL_dRGB.x; d[1] = b[0] * dL_dRGB.y; d[2] = b[0] * dL_dRGB.z;
#pragma unroll
    for (int k = 1; k < 16; k++) {
      if (k < ncoef_used) {
        d = s1 + 3 * k - 3;
        const V3 t = b[k] * dL_dRGB;
        d[0] = t.x; d[1] = t.y; d[2] = t.z;
      }
    }
  }
  V3 dRGBdx, dRGBdy, dRGBdz;
  sh_dir_jacobian(c, deg, dir, dRGBdx, dRGBdy, dRGBdz);
  const V3 dL_ddir = v3(dot3(dRGBdx, dL_dRGB), dot3(dRGBdy, dL_dRGB), dot3(dRGBdz, dL_dRGB));
  return dnormvdv(dir_orig, dL_ddir);
}

// Culled Gaussian, store mode: zero every per-Gaussian output except the SH grads (those are
// written by the cooperative store of the kernel).
__device__ __forceinline__ void zero_outputs(const BwdPreArgs& a, size_t i) {
  put3(a.dL_dmeans2D, i, v3(0, 0, 0));
  if (a.dL_dcolors) put3(a.dL_dcolors, i, v3(0, 0, 0));
  a.dL_dopacity[i] = 0.0f;
  put3(a.dL_dmeans3D, i, v3(0, 0, 0));
  if (a.dL_dcov3D) for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * i + k] = 0.0f;
  if (a.dL_dscales) put3(a.dL_dscales, i, v3(0, 0, 0));
  if (a.dL_drotations) reinterpret_cast<float4*>(a.dL_drotations)[i] = make_float4(0, 0, 0, 0);
  if (a.dL_dsh_language) put3(a.dL_dsh_language, i, v3(0, 0, 0));
  if (a.dL_dlanguage_feature) put3(a.dL_dlanguage_feature, i, v3(0, 0, 0));
}

// Failed forward (its status word is set): every gradient element the normal path would write
// for Gaussian i becomes NaN -- stored, or added (NaN + x = NaN) in accumulate mode -- so the
// call's gradients are NaN-poisoned whatever the buffers held before (gsr.h GSR_ERR_SORT).
template <bool ACC>
__device__ __forceinline__ void poison_outputs(const BwdPreArgs& a, size_t i) {
  const float nan = __builtin_nanf("");
  const V3 n3 = v3(nan, nan, nan);
  put3(a.dL_dmeans2D, i, n3);
  st3<ACC>(a.dL_dmeans3D, i, n3);
  if (a.dL_dcolors) st3<ACC>(a.dL_dcolors, i, n3);
  st<ACC>(a.dL_dopacity + i, nan);
  if (a.dL_dcov3D)
    for (int k = 0; k < 6; k++) st<ACC>(a.dL_dcov3D + 6 * i + k, nan);
  if (a.dL_dscales) st3<ACC>(a.dL_dscales, i, n3);
  if (a.dL_drotations)
    for (int k = 0; k < 4; k++) st<ACC>(a.dL_drotations + 4 * i + k, nan);
  if (a.dL_dsh_language) st3<ACC>(a.dL_dsh_language, i, n3);
  if (a.dL_dlanguage_feature) st3<ACC>(a.dL_dlanguage_feature, i, n3);
  if (a.dRGB_out) {
    put3p(a.dRGB_out, (size_t)a.P, i, n3);  // deferred: the step's flush spreads the NaN
  } else if (a.fused) {
    if (a.dL_dsh) st3<ACC>(a.dL_dsh, i, n3);  // features_dc [P,1,3]
    if (a.dL_dsh_rest)
      for (int k = 0; k < 3 * (a.M - 1); k++) st<ACC>(a.dL_dsh_rest + (size_t)3 * (a.M - 1) * i + k, nan);
  } else if (a.dL_dsh) {
    for (int k = 0; k < 3 * a.M; k++) st<ACC>(a.dL_dsh + (size_t)3 * a.M * i + k, nan);
  }
}

__device__ __forceinline__ void add4(float4& t, float4 x) {
  t.x += x.x; t.y += x.y; t.z += x.z; t.w += x.w;
}
// 1: the once-read per-view streams of the backward preprocess (accumulator rows, the pre-pass
// Jacobian planes) are loaded nontemporally
#ifndef GSR_BWD_NT
#define GSR_BWD_NT 0
#endif
// The Gaussian's 16-float gradient row (gsr_internal.h AccSlot): its accumulator row (atomic
// mode), or the sum of its instances' rows in emission order (rows layout; zero without any).
__device__ __forceinline__ void grad_row(const BwdPreArgs& a, size_t i, float4& q0, float4& q1,
                                         float4& q2, float4& q3) {
  if (!a.use_rows) {
    const float4* accp = reinterpret_cast<const float4*>(a.acc + i * kAccFloats);
    if (GSR_BWD_NT) {  // read once per step (the next forward re-zeroes the rows)
      q0 = stream_ld4(accp); q1 = stream_ld4(accp + 1); q2 = stream_ld4(accp + 2); q3 = stream_ld4(accp + 3);
    } else {
      q0 = accp[0]; q1 = accp[1]; q2 = accp[2]; q3 = accp[3];
    }
    return;
  }
  const uint32_t n = a.count[i];
  if (n == 0) {
    q0 = q1 = q2 = q3 = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float4* r = a.rows + (size_t)a.ebeg[i] * (kAccFloats / 4);
  q0 = r[0]; q1 = r[1]; q2 = r[2]; q3 = r[3];
  for (uint32_t e = 1; e < n; e++) {
    r += kAccFloats / 4;
    add4(q0, r[0]); add4(q1, r[1]); add4(q2, r[2]); add4(q3, r[3]);
  }
}

// Where gaussian_bwd's per-Gaussian gradients go.  MemSink: stored (ACC = 0) or added (ACC = 1)
// straight into the gradient buffers, one view per launch.  RegSink (preprocess_bwd_views_kernel):
// summed over the views of a step in registers, in view order, and written once -- the same
// operations in the same order as one launch per view (the first view stores unless ACC).
template <bool ACC>
struct MemSink {
  const BwdPreArgs& a;
  size_t i;
  __device__ void colors(V3 v) { if (a.dL_dcolors) st3<ACC>(a.dL_dcolors, i, v); }
  __device__ void rgb(V3) {}
  __device__ void opacity(float v) { st<ACC>(a.dL_dopacity + i, v); }
  __device__ void cov3D(const float* d) {
    if (a.dL_dcov3D)
#pragma unroll
      for (int k = 0; k < 6; k++) st<ACC>(a.dL_dcov3D + 6 * i + k, d[k]);
  }
  __device__ void scales(V3 v) { st3<ACC>(a.dL_dscales, i, v); }
  __device__ void rotation(float4 dq) {
    float4* dr = reinterpret_cast<float4*>(a.dL_drotations) + i;
    if (ACC) {
      const float4 o = *dr;
      *dr = make_float4(o.x + dq.x, o.y + dq.y, o.z + dq.z, o.w + dq.w);
    } else {
      *dr = dq;
    }
  }
  __device__ void means3D(V3 v) { st3<ACC>(a.dL_dmeans3D, i, v); }
  __device__ void lang_feature(V3 v) { if (a.dL_dlanguage_feature) st3<ACC>(a.dL_dlanguage_feature, i, v); }
  __device__ void sh_language(V3 v) { if (a.dL_dsh_language) st3<ACC>(a.dL_dsh_language, i, v); }
};
struct RegSink {
  bool assign;  // the next contribution is the first one of store mode (assigned, not added)
  float op;
  V3 m3, sc, lf, shl;
  float4 rot;
  // the view's clamp-masked dL/dRGB, when the launch forms the SH gradients itself: this
  // Gaussian's slot of the view's LDS plane (stride kThreads per channel), else null
  float* rgb_lds;
  __device__ static V3 add3(bool as, V3 acc, V3 v) {
    return as ? v : v3(acc.x + v.x, acc.y + v.y, acc.z + v.z);
  }
  __device__ void colors(V3) {}
  __device__ void rgb(V3 v) {
    if (rgb_lds) {
      rgb_lds[0] = v.x;
      rgb_lds[kThreads] = v.y;
      rgb_lds[2 * kThreads] = v.z;
    }
  }
  __device__ void opacity(float v) { op = assign ? v : op + v; }
  __device__ void cov3D(const float*) {}
  __device__ void scales(V3 v) { sc = add3(assign, sc, v); }
  __device__ void rotation(float4 dq) {
    rot = assign ? dq : make_float4(rot.x + dq.x, rot.y + dq.y, rot.z + dq.z, rot.w + dq.w);
  }
  __device__ void means3D(V3 v) { m3 = add3(assign, m3, v); }
  __device__ void lang_feature(V3 v) { lf = add3(assign, lf, v); }
  __device__ void sh_language(V3 v) { shl = add3(assign, shl, v); }
};

// The view-independent inputs of one Gaussian's backward in the fused scale / rotation
// configuration: its mean, raw and normalised rotation, activated scale, 3D covariance and
// activated opacity.  The multi-view kernel evaluates them once for all views; gaussian_bwd
// evaluates the same functions on the same inputs itself when handed none (bit-identical).
struct BwdModel {
  V3 mean;
  float4 qraw, q;
  V3 sc;
  float c3[6];
  float y;
};
// An opaque copy (no instruction emitted): what is derived from it inside the multi-view loop
// cannot be hoisted out of the loop by the compiler, which otherwise keeps ~80 more registers
// live across the views (207 vs 129 VGPRs measured)
__device__ __forceinline__ BwdModel opaque(const BwdModel& m) {
  BwdModel o = m;
  float* f = reinterpret_cast<float*>(&o);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(BwdModel) / sizeof(float)); k++) asm volatile("" : "+v"(f[k]));
  return o;
}
__device__ __forceinline__ void bwd_model(const BwdPreArgs& a, size_t i, BwdModel& md) {
  md.mean = v3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
  md.qraw = reinterpret_cast<const float4*>(a.rotations)[i];
  md.sc = v3(expf(a.scales[3 * i]), expf(a.scales[3 * i + 1]), expf(a.scales[3 * i + 2]));
  md.q = normalize_quat(md.qraw);
  cov3d_from_scale_rot(md.sc.x, md.sc.y, md.sc.z, a.scale_modifier, md.q.x, md.q.y, md.q.z,
                       md.q.w, md.c3);
  md.y = sigmoid_f(a.opacities_raw[i]);
}

// One view's pre-pass colour Jacobian (planar [9][P]) and clamp bits of one Gaussian, loaded one
// view ahead by the multi-view kernel with its gradient row
struct ViewJac {
  float j[9];
  uint32_t cl;
};
__device__ __forceinline__ void view_jac(const BwdPreArgs& a, size_t i, ViewJac& o) {
  const float* j = a.pre_jac + i;
  const size_t P = (size_t)a.P;
#pragma unroll
  for (int k = 0; k < 9; k++) o.j[k] = GSR_BWD_NT ? __builtin_nontemporal_load(j + k * P) : j[k * P];
  o.cl = a.clamped[i];
}

// Backward of one visible Gaussian.  sh0 / sh1: its rows (coefficient 0 / coefficients 1..) of
// the LDS staging planes: SH coefficients in, SH gradients out; unused without SH.  The
// per-view outputs (screen-space gradient, deferred dL/dRGB, SH rows) are written here; the
// per-Gaussian gradients go to `sk`.  md: the view-independent inputs if already evaluated
// (fused scale / rotation only), row: the gradient row if already loaded.
template <bool ACC, class Sink>
__device__ __forceinline__ void gaussian_bwd(const BwdPreArgs& a, size_t i, float* sh0,
                                             float* sh1, Sink& sk, const BwdModel* md = nullptr,
                                             const float4* row = nullptr,
                                             const ViewJac* vj = nullptr) {
  float4 q0, q1, q2, q3;
  if (row) {
    q0 = row[0]; q1 = row[1]; q2 = row[2]; q3 = row[3];
  } else {
    grad_row(a, i, q0, q1, q2, q3);
  }
  // slots: q0 = {mx, my, ca, cb}, q1 = {cc, op, r, g}, q2 = {b, depth, f0, f1}, q3 = {f2, used, -, -}
  const float gmx = q0.x, gmy = q0.y;
  const float dcx = q0.z, dcy = q0.w, dcz = q1.x;
  put3(a.dL_dmeans2D, i, v3(gmx, gmy, 0.0f));  // per-call output, stored in both modes
  const V3 dL_dcolor = v3(q1.z, q1.w, q2.x);
  sk.colors(dL_dcolor);
  {
    float dop = a.confidence ? q1.y * a.confidence[i] : q1.y;
    if (a.fused) {  // through get_opacity = sigmoid(_opacity): go * (1 - y) * y
      const float y = md ? md->y : sigmoid_f(a.opacities_raw[i]);
      dop = dop * (1.0f - y) * y;
    }
    sk.opacity(dop);
  }

  const V3 mean = md ? md->mean : v3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
  // 3D covariance: precomputed, or recomputed from scale / rotation with the forward's own
  // function and inputs (bit-identical to what the forward projected; not stored in between)
  float c3buf[6];  // always a register array (a pointer select would force it into scratch)
  const float* c3 = c3buf;
  if (md) {
#pragma unroll
    for (int k = 0; k < 6; k++) c3buf[k] = md->c3[k];
  } else if (a.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; k++) c3buf[k] = a.cov3D[6 * i + k];
  } else {
    float4 q = reinterpret_cast<const float4*>(a.rotations)[i];
    float sx = a.scales[3 * i], sy = a.scales[3 * i + 1], sz = a.scales[3 * i + 2];
    if (a.fused) {
      sx = expf(sx); sy = expf(sy); sz = expf(sz);
      q = normalize_quat(q);
    }
    cov3d_from_scale_rot(sx, sy, sz, a.scale_modifier, q.x, q.y, q.z, q.w, c3buf);
  }

  // ---- computeCov2DCUDA, backward.cu:164-273 ----
  const Ewa e = ewa_project(mean, a.fx, a.fy, a.tanx, a.tany, c3, a.view);
  const float x_grad_mul = e.txtz < -e.limx || e.txtz > e.limx ? 0 : 1;
  const float y_grad_mul = e.tytz < -e.limy || e.tytz > e.limy ? 0 : 1;
  const float ca = e.a, cb = e.b, cc = e.c;
  const float denom = ca * cc - cb * cb;
  float dL_da = 0, dL_db = 0, dL_dc = 0;
  const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
  float dcov[6];
#define Tm(c_, r_) e.T.m[c_][r_]
#define Vk(c_, r_) e.Vrk.m[c_][r_]
  if (denom2inv != 0) {
    dL_da = denom2inv * (-cc * cc * dcx + 2 * cb * cc * dcy + (denom - ca * cc) * dcz);
    dL_dc = denom2inv * (-ca * ca * dcz + 2 * ca * cb * dcy + (denom - ca * cc) * dcx);
    dL_db = denom2inv * 2 * (cb * cc * dcx - (denom + 2 * cb * cb) * dcy + ca * cb * dcz);
    dcov[0] = (Tm(0, 0) * Tm(0, 0) * dL_da + Tm(0, 0) * Tm(1, 0) * dL_db + Tm(1, 0) * Tm(1, 0) * dL_dc);
    dcov[3] = (Tm(0, 1) * Tm(0, 1) * dL_da + Tm(0, 1) * Tm(1, 1) * dL_db + Tm(1, 1) * Tm(1, 1) * dL_dc);
    dcov[5] = (Tm(0, 2) * Tm(0, 2) * dL_da + Tm(0, 2) * Tm(1, 2) * dL_db + Tm(1, 2) * Tm(1, 2) * dL_dc);
    dcov[1] = 2 * Tm(0, 0) * Tm(0, 1) * dL_da + (Tm(0, 0) * Tm(1, 1) + Tm(0, 1) * Tm(1, 0)) * dL_db +
              2 * Tm(1, 0) * Tm(1, 1) * dL_dc;
    dcov[2] = 2 * Tm(0, 0) * Tm(0, 2) * dL_da + (Tm(0, 0) * Tm(1, 2) + Tm(0, 2) * Tm(1, 0)) * dL_db +
              2 * Tm(1, 0) * Tm(1, 2) * dL_dc;
    dcov[4] = 2 * Tm(0, 2) * Tm(0, 1) * dL_da + (Tm(0, 1) * Tm(1, 2) + Tm(0, 2) * Tm(1, 1)) * dL_db +
              2 * Tm(1, 1) * Tm(1, 2) * dL_dc;
  } else {
#pragma unroll
    for (int k = 0; k < 6; k++) dcov[k] = 0.0f;
  }
  sk.cov3D(dcov);
  const float dL_dT00 = 2 * (Tm(0, 0) * Vk(0, 0) + Tm(0, 1) * Vk(0, 1) + Tm(0, 2) * Vk(0, 2)) * dL_da +
                        (Tm(1, 0) * Vk(0, 0) + Tm(1, 1) * Vk(0, 1) + Tm(1, 2) * Vk(0, 2)) * dL_db;
  const float dL_dT01 = 2 * (Tm(0, 0) * Vk(1, 0) + Tm(0, 1) * Vk(1, 1) + Tm(0, 2) * Vk(1, 2)) * dL_da +
                        (Tm(1, 0) * Vk(1, 0) + Tm(1, 1) * Vk(1, 1) + Tm(1, 2) * Vk(1, 2)) * dL_db;
  const float dL_dT02 = 2 * (Tm(0, 0) * Vk(2, 0) + Tm(0, 1) * Vk(2, 1) + Tm(0, 2) * Vk(2, 2)) * dL_da +
                        (Tm(1, 0) * Vk(2, 0) + Tm(1, 1) * Vk(2, 1) + Tm(1, 2) * Vk(2, 2)) * dL_db;
  const float dL_dT10 = 2 * (Tm(1, 0) * Vk(0, 0) + Tm(1, 1) * Vk(0, 1) + Tm(1, 2) * Vk(0, 2)) * dL_dc +
                        (Tm(0, 0) * Vk(0, 0) + Tm(0, 1) * Vk(0, 1) + Tm(0, 2) * Vk(0, 2)) * dL_db;
  const float dL_dT11 = 2 * (Tm(1, 0) * Vk(1, 0) + Tm(1, 1) * Vk(1, 1) + Tm(1, 2) * Vk(1, 2)) * dL_dc +
                        (Tm(0, 0) * Vk(1, 0) + Tm(0, 1) * Vk(1, 1) + Tm(0, 2) * Vk(1, 2)) * dL_db;
  const float dL_dT12 = 2 * (Tm(1, 0) * Vk(2, 0) + Tm(1, 1) * Vk(2, 1) + Tm(1, 2) * Vk(2, 2)) * dL_dc +
                        (Tm(0, 0) * Vk(2, 0) + Tm(0, 1) * Vk(2, 1) + Tm(0, 2) * Vk(2, 2)) * dL_db;
#undef Tm
#undef Vk
  const M3& Wm = e.W;
  const float dL_dJ00 = Wm.m[0][0] * dL_dT00 + Wm.m[0][1] * dL_dT01 + Wm.m[0][2] * dL_dT02;
  const float dL_dJ02 = Wm.m[2][0] * dL_dT00 + Wm.m[2][1] * dL_dT01 + Wm.m[2][2] * dL_dT02;
  const float dL_dJ11 = Wm.m[1][0] * dL_dT10 + Wm.m[1][1] * dL_dT11 + Wm.m[1][2] * dL_dT12;
  const float dL_dJ12 = Wm.m[2][0] * dL_dT10 + Wm.m[2][1] * dL_dT11 + Wm.m[2][2] * dL_dT12;
  const float h_x = a.fx, h_y = a.fy;
  const float tz = 1.f / e.t.z;
  const float tz2 = tz * tz;
  const float tz3 = tz2 * tz;
  const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
  const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
  const float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * e.t.x) * tz3 * dL_dJ02 +
                       (2 * h_y * e.t.y) * tz3 * dL_dJ12;
  V3 dmean = xform_vec43_T(v3(dL_dtx, dL_dty, dL_dtz), a.view);

  // ---- preprocessCUDA (bwd), backward.cu:370-387: screen-space mean gradient ----
  const float* proj = a.proj;
  const float m_w = 1.0f / (xform_w(mean, proj) + 0.0000001f);
  const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
  const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
  V3 dm2;
  dm2.x = (proj[0] * m_w - proj[3] * mul1) * gmx + (proj[1] * m_w - proj[3] * mul2) * gmy;
  dm2.y = (proj[4] * m_w - proj[7] * mul1) * gmx + (proj[5] * m_w - proj[7] * mul2) * gmy;
  dm2.z = (proj[8] * m_w - proj[11] * mul1) * gmx + (proj[9] * m_w - proj[11] * mul2) * gmy;
  dmean = dmean + dm2;

  // ---- SH colour backward (backward.cu:390-391) ----
  if (a.shs || a.fused) {
    const uint32_t cl = vj ? vj->cl : (uint32_t)a.clamped[i];
    V3 dRGB = dL_dcolor;
    dRGB.x *= (cl & 1) ? 0 : 1;
    dRGB.y *= (cl & 2) ? 0 : 1;
    dRGB.z *= (cl & 4) ? 0 : 1;
    const V3 dir_orig = mean - v3(a.campos[0], a.campos[1], a.campos[2]);
    if (a.pre_jac) {  // Jacobian from the multi-view pre-pass; dL/dRGB deferred or to the sink
      if (a.dRGB_out) put3p(a.dRGB_out, (size_t)a.P, i, dRGB);
      sk.rgb(dRGB);
      ViewJac own;
      if (!vj) {
        view_jac(a, i, own);
        vj = &own;
      }
      const V3 jx = v3(vj->j[0], vj->j[1], vj->j[2]), jy = v3(vj->j[3], vj->j[4], vj->j[5]),
               jz = v3(vj->j[6], vj->j[7], vj->j[8]);
      const V3 dL_ddir = v3(dot3(jx, dRGB), dot3(jy, dRGB), dot3(jz, dRGB));
      dmean = dmean + dnormvdv(dir_orig, dL_ddir);
    } else if (a.dRGB_out) {  // deferred: dL/dsh = basis(dir) x dRGB is formed by the step's flush
      put3p(a.dRGB_out, (size_t)a.P, i, dRGB);
      dmean = dmean + sh_backward<false>(sh0, sh1, a.D, dir_orig, dRGB);
    } else {
      dmean = dmean + sh_backward<true>(sh0, sh1, a.D, dir_orig, dRGB);
    }
  }

  // ---- cov3D -> scale / rotation (backward.cu:278-341, 393-395) ----
  if (a.scales) {
    const float4 qraw = md ? md->qraw : reinterpret_cast<const float4*>(a.rotations)[i];
    // fused: the kernel saw normalize(_rotation) and exp(_scaling) (gsr_preprocess.hip)
    const float4 q = md ? md->q : (a.fused ? normalize_quat(qraw) : qraw);
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    M3 R = m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    V3 sc;
    if (md) {
      sc = md->sc;
    } else {
      sc = v3(a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]);
      if (a.fused) sc = v3(expf(sc.x), expf(sc.y), expf(sc.z));
    }
    const V3 s = a.scale_modifier * sc;
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    const M3 Mm = m3_mul(S, R);
    const float* g6 = dcov;
    const M3 dL_dSigma = m3_cols(g6[0], 0.5f * g6[1], 0.5f * g6[2], 0.5f * g6[1], g6[3], 0.5f * g6[4],
                                 0.5f * g6[2], 0.5f * g6[4], g6[5]);
    M3 M2;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
      for (int w = 0; w < 3; w++) M2.m[c][w] = 2.0f * Mm.m[c][w];
    const M3 dL_dM = m3_mul(M2, dL_dSigma);
    const M3 Rt = m3_T(R);
    M3 Dt = m3_T(dL_dM);
    V3 ds;
    ds.x = dot3(v3(Rt.m[0][0], Rt.m[0][1], Rt.m[0][2]), v3(Dt.m[0][0], Dt.m[0][1], Dt.m[0][2]));
    ds.y = dot3(v3(Rt.m[1][0], Rt.m[1][1], Rt.m[1][2]), v3(Dt.m[1][0], Dt.m[1][1], Dt.m[1][2]));
    ds.z = dot3(v3(Rt.m[2][0], Rt.m[2][1], Rt.m[2][2]), v3(Dt.m[2][0], Dt.m[2][1], Dt.m[2][2]));
    // fused: through exp (torch exp backward: grad * result)
    sk.scales(a.fused ? v3(ds.x * sc.x, ds.y * sc.y, ds.z * sc.z) : ds);
#pragma unroll
    for (int w = 0; w < 3; w++) {
      Dt.m[0][w] *= s.x;
      Dt.m[1][w] *= s.y;
      Dt.m[2][w] *= s.z;
    }
#define D(c_, r_) Dt.m[c_][r_]
    float4 dq;
    dq.x = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    dq.y = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) -
           4 * x * (D(2, 2) + D(1, 1));
    dq.z = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) -
           4 * y * (D(2, 2) + D(0, 0));
    dq.w = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) -
           4 * z * (D(1, 1) + D(0, 0));
#undef D
    if (a.fused) dq = normalize_quat_backward(qraw, dq);  // through F.normalize
    sk.rotation(dq);
  }

  // ---- depth channel: z_view = view[2] x + view[6] y + view[10] z + view[14] ----
  const float dz = q2.y;
  dmean.x += dz * a.view[2];
  dmean.y += dz * a.view[6];
  dmean.z += dz * a.view[10];
  sk.means3D(dmean);

  // ---- language feature channels ----
  sk.lang_feature((a.include_feature && a.lang_precomp) ? v3(q2.z, q2.w, q3.x) : v3(0, 0, 0));
  if (a.dL_dsh_language) {
    V3 out = v3(0, 0, 0);
    if (a.include_feature && a.lang_precomp == nullptr) {
      const float* l = a.sh_language + 3 * i;
      const float u0 = SH_C0 * l[0], u1 = SH_C0 * l[1], u2 = SH_C0 * l[2];
      const float n = sqrtf(u0 * u0 + u1 * u1 + u2 * u2);
      const float den = n + 1e-9f;
      const float g0 = q2.z, g1 = q2.w, g2 = q3.x;
      const float ug = u0 * g0 + u1 * g1 + u2 * g2;
      const float k2 = n > 0.0f ? ug / (den * den * n) : 0.0f;
      out = v3(SH_C0 * (g0 / den - u0 * k2), SH_C0 * (g1 / den - u1 * k2), SH_C0 * (g2 / den - u2 * k2));
    }
    sk.sh_language(out);
  }
}

// One workgroup = kThreads consecutive Gaussians.  The SH coefficients (48 of the ~60 floats a
// Gaussian reads, and 48 of the grads it writes) go through LDS so that global traffic is
// coalesced 16-byte vectors instead of lane-strided by 180-192 bytes.
template <bool ACC, bool STAGE>
__global__ __launch_bounds__(kThreads) void preprocess_bwd_kernel(BwdPreArgs a) {
  // STAGE = false (colour Jacobian from the multi-view pre-pass): no SH rows, no 48 KB of LDS
  __shared__ float4 s_sh4[STAGE ? kThreads * kShMaxFloats / 4 : 4];
  __shared__ uint8_t s_live[kThreads];
  float* s_sh = reinterpret_cast<float*>(s_sh4);
  const int base = (int)(blockIdx.x * kThreads);
  const int n = min(kThreads, a.P - base);
  const int t = (int)threadIdx.x;
  const size_t i = (size_t)base + t;
  if (a.status && *a.status) {  // the forward failed (grid-uniform): NaN gradients
    if (t < n) poison_outputs<ACC>(a, i);
    return;
  }
  const bool live = t < n && a.radii[i] > 0;
  s_live[t] = live;
  // the SH rows are staged unless the colour Jacobian comes from the multi-view pre-pass
  const bool has_sh = STAGE && (a.shs || a.fused) && !a.pre_jac;
  ShPlane p0{}, p1{};
  if (has_sh) {
    const int ncoef = a.M * 3;
    if (a.fused) {
      p0 = ShPlane{a.sh_dc, a.dL_dsh, 3, 0};
      p1 = ShPlane{a.sh_rest, a.dL_dsh_rest, ncoef - 3, kThreads * 3};
    } else {
      p0 = ShPlane{a.shs, a.dL_dsh, ncoef, 0};
    }
    __syncthreads();
    stage<kThreads, true, ACC>(p0, base, n, s_live, s_sh);
    stage<kThreads, true, ACC>(p1, base, n, s_live, s_sh);
    __syncthreads();
  }
  // this Gaussian's rows: coefficient 0 and coefficients 1..
  float* r0 = s_sh + p0.lds + t * p0.w;
  float* r1 = a.fused ? s_sh + p1.lds + t * p1.w : r0 + 3;
  const bool defer = a.dRGB_out != nullptr;
  if (live) {
    MemSink<ACC> sk{a, i};
    gaussian_bwd<ACC>(a, i, r0, r1, sk);
    if (has_sh && !defer) {  // coefficients above the active degree: zero gradient
      const int used = (a.D + 1) * (a.D + 1) * 3;
      for (int k = used; k < a.M * 3; k++) r1[k - 3] = 0.0f;
    }
  } else {
    if (!ACC && t < n) zero_outputs(a, i);
    if (ACC && t < n) put3(a.dL_dmeans2D, i, v3(0, 0, 0));  // stored output: zeros when culled
    if (defer && t < n) put3p(a.dRGB_out, (size_t)a.P, i, v3(0, 0, 0));
    if (has_sh && !defer && t < n) {  // culled: zero rows (written in store mode, skipped or +0 in ACC)
      for (int k = 0; k < 3; k++) r0[k] = 0.0f;
      for (int k = 3; k < a.M * 3; k++) r1[k - 3] = 0.0f;
    }
  }
  if (has_sh && !defer) {
    __syncthreads();
    stage<kThreads, false, ACC>(p0, base, n, s_live, s_sh);
    stage<kThreads, false, ACC>(p1, base, n, s_live, s_sh);
  }
}

// The per-Gaussian backwards of several views in ONE launch (multi-view calls, deferred SH
// gradients with the pre-pass Jacobian): per Gaussian the views are processed in order with
// gaussian_bwd, their gradients summed in registers (RegSink: the same additions, in the same
// order, as one launch per view) and written once -- the parameters and the leaves' gradients
// cross HBM once per step instead of once per view.  View 0's `accumulate` decides store / add.
// waves per SIMD the views kernel is compiled for: 1 = the compiler's choice (143 VGPRs, 3 waves).
// Forcing 4 (128 VGPRs) spills 10 registers and measured 8 % slower, 4 without the per-view row
// prefetch 17 % slower (profiles/r05_pbwd_occupancy_ab.txt)
#ifndef GSR_BWDV_MINBLK
#define GSR_BWDV_MINBLK 1
#endif
// One Gaussian's views (the body of preprocess_bwd_views_kernel).  rgb: its slot of view 0's
// LDS dL/dRGB plane when the launch forms the SH gradients itself (planes kThreads * 3 apart).
template <bool ACC>
__device__ __forceinline__ void views_body(const BwdPreViews& m, size_t i, float* rgb) {
  const BwdPreArgs& a0 = m.v[0];
  RegSink sk;
  sk.assign = !ACC;
  if (ACC) {
    sk.op = a0.dL_dopacity[i];
    sk.m3 = v3(a0.dL_dmeans3D[3 * i], a0.dL_dmeans3D[3 * i + 1], a0.dL_dmeans3D[3 * i + 2]);
    sk.sc = a0.dL_dscales ? v3(a0.dL_dscales[3 * i], a0.dL_dscales[3 * i + 1], a0.dL_dscales[3 * i + 2])
                          : v3(0, 0, 0);
    sk.rot = a0.dL_drotations ? reinterpret_cast<const float4*>(a0.dL_drotations)[i]
                              : make_float4(0, 0, 0, 0);
    sk.shl = a0.dL_dsh_language ? v3(a0.dL_dsh_language[3 * i], a0.dL_dsh_language[3 * i + 1],
                                     a0.dL_dsh_language[3 * i + 2]) : v3(0, 0, 0);
    sk.lf = a0.dL_dlanguage_feature ? v3(a0.dL_dlanguage_feature[3 * i], a0.dL_dlanguage_feature[3 * i + 1],
                                         a0.dL_dlanguage_feature[3 * i + 2]) : v3(0, 0, 0);
  } else {  // a view-0-culled Gaussian is zero in store mode (zero_outputs)
    sk.op = 0.0f;
    sk.m3 = sk.sc = sk.shl = sk.lf = v3(0, 0, 0);
    sk.rot = make_float4(0, 0, 0, 0);
  }
  bool touched = !ACC;
  // the model side once; each view's gradient row and radius loaded one view ahead, so their
  // latency hides behind the previous view's arithmetic
  BwdModel md;
  bwd_model(a0, i, md);
  float4 cur[4], nxt[4];
  ViewJac jcur, jnxt;
  int rcur = a0.radii[i], rnxt = 0;
  grad_row(a0, i, cur[0], cur[1], cur[2], cur[3]);
  view_jac(a0, i, jcur);
#pragma unroll 1
  for (int v = 0; v < m.V; v++) {
    const BwdPreArgs& a = m.v[v];
    if (v + 1 < m.V) {
      const BwdPreArgs& an = m.v[v + 1];
      rnxt = an.radii[i];
      grad_row(an, i, nxt[0], nxt[1], nxt[2], nxt[3]);
      view_jac(an, i, jnxt);
    }
    sk.rgb_lds = rgb ? rgb + v * 3 * kThreads : nullptr;
    if (a.status && *a.status) {  // this view's forward failed (view-uniform): NaN gradients
      const float nan = __builtin_nanf("");
      const V3 n3 = v3(nan, nan, nan);
      put3(a.dL_dmeans2D, i, n3);
      if (a.dRGB_out) put3p(a.dRGB_out, (size_t)a.P, i, n3);
      sk.rgb(n3);
      sk.opacity(nan); sk.means3D(n3); sk.scales(n3); sk.rotation(make_float4(nan, nan, nan, nan));
      sk.lang_feature(n3); sk.sh_language(n3);
      sk.assign = false;
      touched = true;
    } else if (rcur > 0) {
      const BwdModel mv = opaque(md);
      gaussian_bwd<true>(a, i, nullptr, nullptr, sk, &mv, cur, &jcur);
      sk.assign = false;
      touched = true;
    } else {
      put3(a.dL_dmeans2D, i, v3(0, 0, 0));
      if (a.dRGB_out) put3p(a.dRGB_out, (size_t)a.P, i, v3(0, 0, 0));
      sk.rgb(v3(0, 0, 0));
      if (v == 0) sk.assign = false;  // store mode: the zeros of the culled first view
    }
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    jcur = jnxt;
    rcur = rnxt;
  }
  if (!touched) return;  // accumulate mode, culled in every view: nothing to add
  a0.dL_dopacity[i] = sk.op;
  put3(a0.dL_dmeans3D, i, sk.m3);
  if (a0.dL_dscales) put3(a0.dL_dscales, i, sk.sc);
  if (a0.dL_drotations) reinterpret_cast<float4*>(a0.dL_drotations)[i] = sk.rot;
  if (a0.dL_dsh_language) put3(a0.dL_dsh_language, i, sk.shl);
  if (a0.dL_dlanguage_feature) put3(a0.dL_dlanguage_feature, i, sk.lf);
}

// SH = true: the launch holds every view of the step and forms the SH gradients itself --
//   dL/dsh_k = sum over the views v, in order, of basis_k(normalize(mean - campos_v)) * dL/dRGB_v
// (backward.cu:20-139, the same operations as sh_flush_kernel), each view's dL/dRGB kept in LDS
// instead of a [3][P] plane stored here and read back by a flush launch; the rows go out
// through the LDS staging planes (stored, or added under ACC).
template <bool ACC, bool SH>
__global__ __launch_bounds__(kThreads, GSR_BWDV_MINBLK) void preprocess_bwd_views_kernel(BwdPreViews m) {
  const uint32_t base = m.row0 + blockIdx.x * (uint32_t)kThreads;
  const int t = (int)threadIdx.x;
  const size_t i = (size_t)base + t;
  const bool valid = i < (size_t)m.row1;
  if (!SH) {
    if (valid) views_body<ACC>(m, i, nullptr);
    return;
  }
  // the views' dL/dRGB planes ([V][3][kThreads] floats, V <= kMaxBwdViews), then the same LDS as
  // the staging planes of half the workgroup's rows at a time (24 KB instead of 48: the LDS no
  // longer caps the launch at 3 workgroups per CU)
  constexpr int kHalf = kThreads / 2;
  static_assert(kMaxBwdViews * 3 * kThreads == kHalf * kShMaxFloats, "LDS: planes = half staging");
  __shared__ float4 s_sh4[SH ? kHalf * kShMaxFloats / 4 : 1];
  __shared__ uint8_t s_live[kThreads];
  float* s_sh = reinterpret_cast<float*>(s_sh4);
  const BwdPreArgs& a0 = m.v[0];
  const int n = (int)min((uint32_t)kThreads, m.row1 - base);
  s_live[t] = t < n;
  if (valid) views_body<ACC>(m, i, s_sh + t);
  V3 g[16];
  const int used = (a0.D + 1) * (a0.D + 1);
  if (valid) {
    const V3 mean = v3(a0.means3D[3 * i], a0.means3D[3 * i + 1], a0.means3D[3 * i + 2]);
    for (int v = 0; v < m.V; v++) {
      const float* cp = m.v[v].campos;
      float b[16];
      sh_basis(mean - v3(cp[0], cp[1], cp[2]), a0.D, b);  // gsr_sh.h
      const float* d = s_sh + v * 3 * kThreads + t;
      const V3 dRGB = v3(d[0], d[kThreads], d[2 * kThreads]);
#pragma unroll
      for (int k = 0; k < 16; k++) g[k] = v == 0 ? b[k] * dRGB : g[k] + b[k] * dRGB;
    }
  }
  const ShPlane p0{nullptr, a0.dL_dsh, 3, 0};
  const ShPlane p1{nullptr, a0.dL_dsh_rest, (a0.M - 1) * 3, kHalf * 3};
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    // h = 0: every dL/dRGB plane read, the LDS becomes the staging planes; h = 1: the first
    // half's rows are out
    __syncthreads();
    const int r = t - h * kHalf;
    if (valid && r >= 0 && r < kHalf) {
      float* r0 = s_sh + p0.lds + r * p0.w;
      float* r1 = s_sh + p1.lds + r * p1.w;
      r0[0] = g[0].x; r0[1] = g[0].y; r0[2] = g[0].z;
#pragma unroll
      for (int k = 1; k < 16; k++) {  // static indices: g stays in registers
        if (k < a0.M) {
          const V3 v = k < used ? g[k] : v3(0, 0, 0);
          r1[3 * k - 3] = v.x; r1[3 * k - 2] = v.y; r1[3 * k - 1] = v.z;
        }
      }
    }
    __syncthreads();
    const int hn = min(kHalf, n - h * kHalf);  // workgroup-uniform
    if (hn > 0) {
      stage<kThreads, false, ACC>(p0, (int)base + h * kHalf, hn, s_live + h * kHalf, s_sh);
      stage<kThreads, false, ACC>(p1, (int)base + h * kHalf, hn, s_live + h * kHalf, s_sh);
    }
  }
}

// Deferred SH gradients of a multi-view step: per Gaussian, for each view v in order,
//   dL/dsh_k += basis_k(normalize(mean - campos_v)) * dL/dRGB_v      (backward.cu:20-139 PUTs)
// with the same basis arithmetic as sh_backward, summed in registers, written once (store) or
// added once (ACC) through the LDS staging planes -- instead of one 192-byte read-modify-write of
// the SH gradient rows per view.
#ifndef GSR_SH_THREADS
#define GSR_SH_THREADS 256
#endif
constexpr int kShThreads = GSR_SH_THREADS;  // see gsr_preprocess.hip kPcThreads
template <bool ACC>
__global__ __launch_bounds__(kShThreads) void sh_flush_kernel(ShFlushArgs a) {
  __shared__ float4 s_sh4[kShThreads * kShMaxFloats / 4];
  __shared__ uint8_t s_live[kShThreads];
  float* s_sh = reinterpret_cast<float*>(s_sh4);
  const int base = (int)(blockIdx.x * kShThreads);
  const int n = min(kShThreads, a.P - base);
  const int t = (int)threadIdx.x;
  const size_t i = (size_t)base + t;
  s_live[t] = t < n;
  const ShPlane p0{nullptr, a.dL_dsh_dc, 3, 0};
  const ShPlane p1{nullptr, a.dL_dsh_rest, (a.M - 1) * 3, kShThreads * 3};
  if (t < n) {
    const V3 mean = v3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
    V3 g[16];
    const int used = (a.D + 1) * (a.D + 1);
    for (int v = 0; v < a.nviews; v++) {
      const float* cp = a.campos[v];
      float b[16];
      sh_basis(mean - v3(cp[0], cp[1], cp[2]), a.D, b);  // gsr_sh.h
      const float* d = a.dRGB[v] + i;  // planar [3][rgb_stride]
      const V3 dRGB = v3(d[0], d[a.rgb_stride], d[2 * a.rgb_stride]);
#pragma unroll
      for (int k = 0; k < 16; k++) g[k] = v == 0 ? b[k] * dRGB : g[k] + b[k] * dRGB;
    }
    float* r0 = s_sh + p0.lds + t * p0.w;
    float* r1 = s_sh + p1.lds + t * p1.w;
    r0[0] = g[0].x; r0[1] = g[0].y; r0[2] = g[0].z;
#pragma unroll
    for (int k = 1; k < 16; k++) {  // static indices: g stays in registers
      if (k < a.M) {
        const V3 v = k < used ? g[k] : v3(0, 0, 0);
        r1[3 * k - 3] = v.x; r1[3 * k - 2] = v.y; r1[3 * k - 1] = v.z;
      }
    }
  }
  __syncthreads();
  stage<kShThreads, false, ACC>(p0, base, n, s_live, s_sh);
  stage<kShThreads, false, ACC>(p1, base, n, s_live, s_sh);
}

}  // namespace

hipError_t launch_sh_grad_flush(const ShFlushArgs& a, hipStream_t s) {
  if (a.P == 0 || a.nviews <= 0) return hipSuccess;
  const dim3 grid((a.P + kShThreads - 1) / kShThreads);
  if (a.accumulate)
    hipLaunchKernelGGL(sh_flush_kernel<true>, grid, dim3(kShThreads), 0, s, a);
  else
    hipLaunchKernelGGL(sh_flush_kernel<false>, grid, dim3(kShThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_preprocess_backward_views(const BwdPreArgs* views, int V, hipStream_t s,
                                            uint32_t row0, uint32_t row1) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBwdViews) return hipErrorNotSupported;
  BwdPreViews m{};
  m.V = V;
  // SH gradients formed in the launch (pre-pass Jacobian, no deferred dL/dRGB plane, the SH
  // gradient planes given) or deferred to the step's flush (dL/dRGB planes)
  const bool sh = views[0].dRGB_out == nullptr;
  for (int k = 0; k < V; k++) {
    const BwdPreArgs& a = views[k];
    // the multi-view kernel covers the fused, pre-pass configuration of one model
    if (!a.fused || !a.pre_jac || a.cov3D || a.colors_precomp || a.dL_dcolors ||
        a.dL_dcov3D || a.P != views[0].P || a.means3D != views[0].means3D ||
        a.dL_dmeans3D != views[0].dL_dmeans3D || a.dL_dopacity != views[0].dL_dopacity ||
        a.dL_dscales != views[0].dL_dscales || a.dL_drotations != views[0].dL_drotations ||
        a.dL_dsh_language != views[0].dL_dsh_language ||
        a.dL_dlanguage_feature != views[0].dL_dlanguage_feature || (k > 0 && !a.accumulate) ||
        (a.dRGB_out == nullptr) != sh ||
        (sh && (!a.dL_dsh || a.dL_dsh != views[0].dL_dsh || a.dL_dsh_rest != views[0].dL_dsh_rest ||
                (a.M > 1 && !a.dL_dsh_rest) || a.M != views[0].M || a.D != views[0].D)))
      return hipErrorNotSupported;
    m.v[k] = a;
  }
  m.row0 = row0;
  m.row1 = row1 < (uint32_t)views[0].P ? row1 : (uint32_t)views[0].P;
  if (m.row1 <= m.row0) return hipSuccess;
  const dim3 grid((m.row1 - m.row0 + kThreads - 1) / kThreads);
  if (views[0].accumulate) {
    if (sh) hipLaunchKernelGGL((preprocess_bwd_views_kernel<true, true>), grid, dim3(kThreads), 0, s, m);
    else hipLaunchKernelGGL((preprocess_bwd_views_kernel<true, false>), grid, dim3(kThreads), 0, s, m);
  } else {
    if (sh) hipLaunchKernelGGL((preprocess_bwd_views_kernel<false, true>), grid, dim3(kThreads), 0, s, m);
    else hipLaunchKernelGGL((preprocess_bwd_views_kernel<false, false>), grid, dim3(kThreads), 0, s, m);
  }
  return hipGetLastError();
}

hipError_t launch_preprocess_backward(const BwdPreArgs& a, hipStream_t s) {
  if (a.P == 0) return hipSuccess;
  const dim3 grid((a.P + kThreads - 1) / kThreads);
  const bool stage = (a.shs || a.fused) && !a.pre_jac;
  if (a.accumulate) {
    if (stage) hipLaunchKernelGGL((preprocess_bwd_kernel<true, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((preprocess_bwd_kernel<true, false>), grid, dim3(kThreads), 0, s, a);
  } else {
    if (stage) hipLaunchKernelGGL((preprocess_bwd_kernel<false, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((preprocess_bwd_kernel<false, false>), grid, dim3(kThreads), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace gsr

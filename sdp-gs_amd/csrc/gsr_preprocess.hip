// gsr_preprocess.hip -- per-Gaussian forward preprocess and the near-plane visibility test.
//
// Behaviour follows preprocessCUDA (cuda_rasterizer/forward.cu:155-256), computeColorFromSH
// (:20-71), in_frustum (auxiliary.h:139-164) and checkFrustum (rasterizer_impl.cu:54-66).
// gfx950 design: one lane per Gaussian over the SoA inputs; the kernel writes everything the
// later stages need in one pass -- the depth-sort key (float bits of view z, which sort
// monotonically because z > 0.2), the tile count, and a 64-byte "splat record" packed for the
// blend's tile gather:
//   rec[4g+0] = {x_px, y_px, conic.a, conic.b}
//   rec[4g+1] = {conic.c, opacity*confidence, depth, r}
//   rec[4g+2] = {g, b, f0, f1}
//   rec[4g+3] = {f2, radius, q_cut, rows} (radius as float: exact; q_cut: the culling threshold of
//                                        gsr_device.h, computed once here for the binning and blends;
//                                        rows: the kept tile range of each row, packed (kNoRowPack:
//                                        not packed), so the duplication does not re-run the cut)
// so the blend reads one contiguous record per instance instead of five scattered arrays.  A
// Gaussian with tiles also gets its 8-B binning word (GeomState::bword): the duplication, which
// visits the Gaussians in depth order, gathers that word instead of two 16-B parts of the 64-B
// record (round 6: the record gather fetched ~2x the duplication's algorithmic bytes).
#include "gsr_device.h"
#include "gsr_internal.h"
#include "gsr_sh.h"
#include "gsr_stage.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
#ifndef GSR_PRE_OPAQUE
#define GSR_PRE_OPAQUE 1
#endif
#ifndef GSR_PRE_VIEWS_MINBLK
#define GSR_PRE_VIEWS_MINBLK 5  // 5 waves per SIMD: 96 VGPRs, 28 B spilled (measured 0.142 -> 0.134 ms per 3 views)
#endif

// The view-independent inputs of one Gaussian: its mean, 3D covariance (precomputed, or from
// the activated scale / rotation), effective opacity and language feature.  The single-view kernel
// evaluates them per view; the multi-view kernel once per Gaussian for all its views (the same
// functions on the same inputs: bit-identical).
struct PreModelIn {
  V3 p_orig;
  float c3[6];
  float op, f0, f1, f2;
};
__device__ __forceinline__ void pre_model_in(const PreArgs& a, int idx, const float* pm,
                                             const float* ps, const float* pl, PreModelIn& o) {
  o.p_orig = v3(pm[0], pm[1], pm[2]);
  if (a.cov3D_precomp) {
#pragma unroll
    for (int k = 0; k < 6; k++) o.c3[k] = a.cov3D_precomp[6 * (size_t)idx + k];
  } else {
    float4 q = reinterpret_cast<const float4*>(a.rotations)[idx];
    float sx = ps[0], sy = ps[1], sz = ps[2];
    if (a.fused) {  // GaussianModel activations: exp(_scaling), normalize(_rotation)
      sx = expf(sx); sy = expf(sy); sz = expf(sz);
      q = normalize_quat(q);
    }
    // not stored: the backward recomputes it bit-identically from the same inputs
    cov3d_from_scale_rot(sx, sy, sz, a.scale_modifier, q.x, q.y, q.z, q.w, o.c3);
  }
  float op = a.opacities[idx];
  if (a.fused) op = sigmoid_f(op);  // GaussianModel.get_opacity
  if (a.confidence) op = op * a.confidence[idx];
  o.op = op;
  o.f0 = o.f1 = o.f2 = 0.f;
  if (a.include_feature) {
    if (a.lang_precomp) {
      o.f0 = a.lang_precomp[3 * idx]; o.f1 = a.lang_precomp[3 * idx + 1];
      o.f2 = a.lang_precomp[3 * idx + 2];
    } else if (a.sh_language) {
      const float u0 = SH_C0 * pl[0];
      const float u1 = SH_C0 * pl[1];
      const float u2 = SH_C0 * pl[2];
      const float n = sqrtf(u0 * u0 + u1 * u1 + u2 * u2);
      const float den = n + 1e-9f;
      o.f0 = u0 / den; o.f1 = u1 / den; o.f2 = u2 / den;
    }
  }
}

// One Gaussian in the view of `a`; returns its exact tile count (0 when culled), sets rect_tiles
// to the tile count of its full 3-sigma rectangle (the reference's tiles_touched, forward.cu:255;
// 0 when culled) and writes its splat record to rec[0..3] (the workgroup's LDS staging row; all
// zero when culled: such a record is never read).
// pm / ps / pl: this Gaussian's 3 floats of means3D / scales / sh_language.  in: its
// view-independent inputs if already evaluated (multi-view kernel), else null (evaluated here,
// after the near-plane test).
// rec: the lane's 4 LDS record slots, part k at rec[k ^ sw] (rec_swizzle).
__device__ __forceinline__ uint32_t preprocess_gaussian(const PreArgs& a, int idx, float4* rec,
                                                        uint32_t sw, const float* pm,
                                                        const float* ps, const float* pl,
                                                        uint32_t& rect_tiles,
                                                        const PreModelIn* in) {
  // zeros in the same swizzled slots as the record (k -> k ^ sw): unswizzled, the 8 lanes of a
  // ds_write_b128 group hit 2 slots four ways each (profiles/pmc_r04.json: 4.5 M conflict cycles)
#pragma unroll
  for (int k = 0; k < 4; k++) rec[k ^ sw] = make_float4(0.f, 0.f, 0.f, 0.f);
  rect_tiles = 0;
  const V3 p_orig = in ? in->p_orig : v3(pm[0], pm[1], pm[2]);
  const V3 p_view = xform_point43(p_orig, a.view);
  // in_frustum: near-plane test only (auxiliary.h:154)
  const bool near_ok = !(p_view.z <= 0.2f);
  const GeomState& g = a.g;
  a.radii[idx] = 0;
  g.tiles_touched[idx] = 0;
  g.dkey_a[idx] = kSortSentinel;  // culled: no tiles, any sorted position is fine
  g.dval_a[idx] = (uint32_t)idx;
  if (!near_ok) {
    if (a.prefiltered) atomicOr(&g.flags[0], 1u);  // reference __trap()s (auxiliary.h:156-160)
    return 0;
  }
  const V3 ph = xform_point43(p_orig, a.proj);
  const float pw = 1.0f / (xform_w(p_orig, a.proj) + 0.0000001f);
  const float pproj_x = ph.x * pw, pproj_y = ph.y * pw;

  PreModelIn own;
  if (!in) {
    pre_model_in(a, idx, pm, ps, pl, own);
    in = &own;
  }
  const Ewa e = ewa_project(p_orig, a.fx, a.fy, a.tanx, a.tany, in->c3, a.view);
  const float det = (e.a * e.c - e.b * e.b);
  if (det == 0.0f) return 0;
  const float det_inv = 1.f / det;
  const float con_a = e.c * det_inv, con_b = -e.b * det_inv, con_c = e.a * det_inv;
  const float mid = 0.5f * (e.a + e.c);
  const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
  const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
  const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
  const float px = ndc2pix(pproj_x, a.W), py = ndc2pix(pproj_y, a.H);
  const int r = f2i_sat(my_radius);
  uint32_t x0, y0, x1, y1;
  tile_rect(px, py, r, a.gx, a.gy, x0, y0, x1, y1);
  if ((x1 - x0) * (y1 - y0) == 0) return 0;

  float cr, cg, cb;
  if (a.pre_color) {  // multi-view pre-pass: the same sh_to_rgb, evaluated for all views at once
    cr = a.pre_color[idx]; cg = a.pre_color[(size_t)a.P + idx];  // planar [3][P]
    cb = a.pre_color[2 * (size_t)a.P + idx];
    g.clamped[idx] = a.pre_clamp[idx];
  } else if (a.colors_precomp == nullptr) {
    V3 dir = p_orig - v3(a.campos[0], a.campos[1], a.campos[2]);
    const float len = sqrtf(dot3(dir, dir));
    dir = v3(dir.x / len, dir.y / len, dir.z / len);
    uint8_t cl;
    const float* s0 = a.fused ? a.sh_dc + 3 * (size_t)idx : a.shs + (size_t)idx * a.M * 3;
    const float* s1 = a.fused ? a.sh_rest + (size_t)idx * (a.M - 1) * 3 : s0 + 3;
    const V3 c = sh_to_rgb(s0, s1, a.D, dir, cl);
    g.clamped[idx] = cl;
    cr = c.x; cg = c.y; cb = c.z;
  } else {
    cr = a.colors_precomp[3 * idx];
    cg = a.colors_precomp[3 * idx + 1];
    cb = a.colors_precomp[3 * idx + 2];
  }
  const float op = in->op;
  const float depth = p_view.z;
  a.radii[idx] = r;
  rect_tiles = (y1 - y0) * (x1 - x0);
  // Exact tile list: the reference emits every tile of the 3-sigma square (forward.cu:255); tiles
  // in which no pixel can reach alpha >= 1/255 are dropped here (no output bit changes)
  const float qc = splat_q_cut(con_a, con_b, con_c, op);
  uint32_t count = 0;
  // the kept per-row ranges, packed for the duplication when the rectangle has at most 4 rows
  // of at most 15 tiles (row r: bits 8r..8r+3 = first tile - x0, bits 8r+4..8r+7 = its length)
  const bool pack = (y1 - y0) <= 4u && (x1 - x0) <= 15u;
  uint32_t packed = pack ? 0u : kNoRowPack;
  if (qc == -1.0f) {
    count = (y1 - y0) * (x1 - x0);
    if (pack)
      for (uint32_t r = 0; r < y1 - y0; r++) packed |= ((x1 - x0) << 4) << (8 * r);
  } else if (qc >= 0.0f) {
    // per tile row, the kept tiles form one range (band_row_range)
    const BandCut cut = make_band_cut(px, py, con_a, con_b, con_c, qc);
    for (uint32_t ty = y0; ty < y1; ty++) {
      uint32_t ra, rb;
      band_row_range(cut, ty, x0, x1, ra, rb);
      count += rb - ra;
      if (pack) packed |= ((ra - x0) | ((rb - ra) << 4)) << (8 * (ty - y0));
    }
  }
  g.tiles_touched[idx] = count;
  if (count) {
    const bool word = pack && x0 < (1u << 14) && y0 < (1u << 14);
    g.bword[idx] = make_uint2(x0 | (y0 << 14) | ((y1 - y0) << 28), word ? packed : kNoRowPack);
  }
  g.dkey_a[idx] = __float_as_uint(depth);
  if (a.vpack) g.dval_a[idx] = (uint32_t)idx | (count << a.vpack);
  rec[0 ^ sw] = make_float4(px, py, con_a, con_b);
  rec[1 ^ sw] = make_float4(con_c, op, depth, cr);
  rec[2 ^ sw] = make_float4(cg, cb, in->f0, in->f1);
  rec[3 ^ sw] = make_float4(in->f2, (float)r, qc, __uint_as_float(packed));
  return count;
}

// one lane per Gaussian; SH rows are read directly (an LDS-staged variant, gsr_stage.h, measured
// slower here: its 48 KB of LDS cut occupancy below what this latency-bound kernel needs).  The
// 64-byte records and accumulator rows (128 of the 145 bytes a Gaussian writes) leave as the
// workgroup's contiguous 16-KB segments: lane t stores 16-byte chunk t, t + 256, ... (records
// transposed through LDS at an 80-byte row stride) instead of 16-byte pieces at a 64-byte lane
// stride.  Each workgroup also writes the sum of its tile counts (a.parts), so R = sum of the
// partials needs one more small launch instead of a separate pass over tiles_touched.
// The workgroup's records in LDS, 4 float4 slots per lane, part k of lane l's record in slot
// 4 l + (k ^ rec_swizzle(l)).  Lane stores (ds_write_b128, 8-lane groups over 32 banks): the
// swizzle puts the 8 lanes of a group on 8 different 16-byte bank quads; the epilogue's linear
// reads (ds_read_b128, 16-lane groups over 64 banks) cover 16 consecutive slots: conflict-free
// both ways.  (Round 3's 80-byte padded rows made the reads ~3-way conflicted: 4.03 M conflict
// cycles per 3-view launch against 1.38 M LDS instructions)
constexpr int kRecStride = 4;
__device__ __forceinline__ uint32_t rec_swizzle(uint32_t lane) { return (lane >> 1) & 3u; }
// (__launch_bounds__(256, 6), 80 VGPRs with a 12-byte spill, measured equal to the unbounded 82)
// The workgroup's outputs after its lanes' preprocess_gaussian: the records (from LDS), the
// zeroed accumulator rows and the partial sums of the tile counts.
__device__ __forceinline__ void pre_epilogue_blk(const PreArgs& a, int base, int n, uint32_t count,
                                                 uint32_t rect, const float4* s_rec,
                                                 uint32_t* s_sum, uint32_t* s_rect, uint32_t blk,
                                                 uint32_t nblk) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    count += (uint32_t)__shfl_xor((int)count, d, 64);
    rect += (uint32_t)__shfl_xor((int)rect, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_sum[threadIdx.x >> 6] = count;
    s_rect[threadIdx.x >> 6] = rect;
  }
  __syncthreads();
  {
    float4* out = a.g.rec + 4 * (size_t)base;
    for (int q = (int)threadIdx.x; q < 4 * n; q += kThreads)  // slot q holds part k of record q / 4
      out[(q & ~3) | ((q & 3) ^ (int)rec_swizzle((uint32_t)q >> 2))] = s_rec[q];
  }
  if (a.acc_zero) {  // the workgroup's 64-B gradient accumulator rows (zeroed before the backward)
    float4* z = reinterpret_cast<float4*>(a.g.acc + (size_t)base * kAccFloats);
    for (int q = (int)threadIdx.x; q < n * (kAccFloats / 4); q += kThreads)
      z[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (threadIdx.x == 0) {
    uint32_t t = 0, tr = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) {
      t += s_sum[w];
      tr += s_rect[w];
    }
    a.parts[blk] = t;
    a.parts[nblk + blk] = tr;
  }
}
__device__ __forceinline__ void pre_epilogue(const PreArgs& a, int base, int n, uint32_t count,
                                             uint32_t rect, const float4* s_rec,
                                             uint32_t* s_sum, uint32_t* s_rect) {
  pre_epilogue_blk(a, base, n, count, rect, s_rec, s_sum, s_rect, blockIdx.x, gridDim.x);
}

// (__launch_bounds__(256, 6), 80 VGPRs with a 12-byte spill, measured equal to the unbounded 82)
__global__ __launch_bounds__(kThreads) void preprocess_kernel(PreArgs a) {
  __shared__ float4 s_rec[kThreads * kRecStride];
  __shared__ uint32_t s_sum[kThreads / 64], s_rect[kThreads / 64];
  const int base = (int)(blockIdx.x * kThreads);
  const int idx = base + (int)threadIdx.x;
  const int n = min(kThreads, a.P - base);
  side_clear(a.clear.p, a.clear.bytes, (size_t)idx, (size_t)gridDim.x * kThreads);
  const float* pm = a.means3D + 3 * (size_t)idx;
  const float* ps = a.scales + 3 * (size_t)idx;
  const float* pl = a.sh_language + 3 * (size_t)idx;
  uint32_t rect = 0;
  const uint32_t count = idx < a.P ? preprocess_gaussian(a, idx, s_rec + threadIdx.x * kRecStride,
                                                         rec_swizzle(threadIdx.x), pm, ps, pl,
                                                         rect, nullptr) : 0u;
  pre_epilogue(a, base, n, count, rect, s_rec, s_sum, s_rect);
}

// Several views of the same Gaussians in one launch (the multi-view call, gsr_api.cpp): a lane
// reads its Gaussian's model inputs and evaluates the view-independent part (covariance,
// opacity, feature) once, then runs every view's part with that view's arguments -- per view the
// same outputs as preprocess_kernel, bit for bit, without re-reading 56 B of model rows and
// re-evaluating exp / normalize / the covariance per view.  Views in m.v[0 .. V); the model
// fields of m.v[0] are those of every view.
__global__ __launch_bounds__(kThreads, GSR_PRE_VIEWS_MINBLK) void preprocess_views_kernel(PreViews m) {
  __shared__ float4 s_rec[kThreads * kRecStride];
  __shared__ uint32_t s_sum[kThreads / 64], s_rect[kThreads / 64];
  const PreArgs& a0 = m.v[0];
  const int base = (int)(blockIdx.x * kThreads);
  const int idx = base + (int)threadIdx.x;
  const int n = min(kThreads, a0.P - base);
  for (int k = 0; k < m.V; k++)
    side_clear(m.v[k].clear.p, m.v[k].clear.bytes, (size_t)idx, (size_t)gridDim.x * kThreads);
  const bool live = idx < a0.P;
  const float* pm = a0.means3D + 3 * (size_t)idx;
  const float* ps = a0.scales + 3 * (size_t)idx;
  const float* pl = a0.sh_language + 3 * (size_t)idx;
  PreModelIn in;
  if (live) pre_model_in(a0, idx, pm, ps, pl, in);
  for (int k = 0; k < m.V; k++) {
    const PreArgs& a = m.v[k];
    uint32_t rect = 0;
#if GSR_PRE_OPAQUE
    // an opaque copy per view (no instruction): nothing derived from the model inputs is hoisted
    // out of the view loop into registers
    PreModelIn iv = in;
    {
      float* f = reinterpret_cast<float*>(&iv);
#pragma unroll
      for (int q = 0; q < (int)(sizeof(PreModelIn) / sizeof(float)); q++) asm volatile("" : "+v"(f[q]));
    }
#else
    const PreModelIn& iv = in;
#endif
    const uint32_t count = live ? preprocess_gaussian(a, idx, s_rec + threadIdx.x * kRecStride,
                                                      rec_swizzle(threadIdx.x), pm, ps, pl, rect,
                                                      &iv) : 0u;
    pre_epilogue(a, base, n, count, rect, s_rec, s_sum, s_rect);
    __syncthreads();  // s_rec / s_sum are the next view's
  }
}

// Workgroup size of the SH-row kernels (colour pre-pass here, SH flush in gsr_backward.hip):
// their LDS staging takes 192 B per lane, so the CU holds the same number of lanes at any size;
// smaller workgroups only desynchronise the load / compute / store phases of its residents.
#ifndef GSR_SH_THREADS
#define GSR_SH_THREADS 256
#endif
constexpr int kPcThreads = GSR_SH_THREADS;

// Multi-view colour pre-pass (gsr_amd/pipeline.py): one pass over the SH rows serves the
// forward colour and the backward's colour Jacobian of every view of a step, instead of every
// view's preprocess and backward preprocess reading the 192-byte rows again.  Per Gaussian and
// view: sh_to_rgb (forward.cu:20-71, the forward's own function) -> colour [3][P] + clamp bits,
// and sh_dir_jacobian (backward.cu:56-131) -> dRGB/ddir [9][P].  The rows go through LDS
// (gsr_stage.h) so the global reads are coalesced 16-byte vectors.
// The rows are staged half a workgroup at a time (24 KB of LDS instead of 48, so the LDS no longer
// caps the launch at 3 workgroups per CU) and copied into registers, the colour and the Jacobian
// then read the registers.
template <bool COL, bool JAC>
__global__ __launch_bounds__(kPcThreads) void sh_precolor_kernel(PrecolorArgs a) {
  constexpr int kHalf = kPcThreads / 2;
  __shared__ float4 s_sh4[kHalf * kShMaxFloats / 4];
  __shared__ uint8_t s_live[kPcThreads];
  float* s_sh = reinterpret_cast<float*>(s_sh4);
  const int base = (int)(a.row0 + blockIdx.x * kPcThreads);
  const int n = min(kPcThreads, (int)a.row1 - base);
  const int t = (int)threadIdx.x;
  const size_t i = (size_t)base + t;
  s_live[t] = t < n;
  const ShPlane p0{a.sh_dc, nullptr, 3, 0};
  const ShPlane p1{a.sh_rest, nullptr, (a.M - 1) * 3, kHalf * 3};
  const int used = (a.D + 1) * (a.D + 1);
  V3 c[16];
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    const int hn = min(kHalf, n - h * kHalf);  // workgroup-uniform
    __syncthreads();  // (h = 1: the first half's rows are in registers)
    if (hn > 0) {
      stage<kPcThreads, true, false>(p0, base + h * kHalf, hn, s_live + h * kHalf, s_sh);
      stage<kPcThreads, true, false>(p1, base + h * kHalf, hn, s_live + h * kHalf, s_sh);
    }
    __syncthreads();
    const int r = t - h * kHalf;
    if (r >= 0 && r < hn) {
      const float* r0 = s_sh + p0.lds + r * p0.w;
      const float* r1 = s_sh + p1.lds + r * p1.w;
      c[0] = v3(r0[0], r0[1], r0[2]);
#pragma unroll
      for (int k = 1; k < 16; k++)
        c[k] = (k < used && k < a.M) ? v3(r1[3 * k - 3], r1[3 * k - 2], r1[3 * k - 1]) : v3(0, 0, 0);
    }
  }
  if (t >= n) return;
  const V3 p_orig = v3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
  for (int v = 0; v < a.nviews; v++) {
    const float* cp = a.campos[v];
    const V3 dir_orig = p_orig - v3(cp[0], cp[1], cp[2]);
    // forward: gsr_preprocess_kernel's direction and colour
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const V3 dir = v3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    // planar outputs ([3][P] colour, [9][P] Jacobian): every store instruction of the wave is
    // one contiguous 256-byte run, and so is every load of the consuming preprocesses
    const size_t P = (size_t)a.P;
    if (COL) {
      uint8_t cl;
      const V3 col = sh_to_rgb_at([&](int k) { return c[k]; }, a.D, dir, cl);
      float* co = a.color[v] + i;
      stream_st(co, col.x); stream_st(co + P, col.y); stream_st(co + 2 * P, col.z);
      stream_st(a.clamp[v] + i, cl);
    }
    if (!JAC) continue;
    // backward: sh_backward's Jacobian at the same normalised direction
    V3 jx, jy, jz;
    sh_dir_jacobian(c, a.D, dir, jx, jy, jz);
    float* jo = a.jac[v] + i;
    stream_st(jo, jx.x); stream_st(jo + P, jx.y); stream_st(jo + 2 * P, jx.z);
    stream_st(jo + 3 * P, jy.x); stream_st(jo + 4 * P, jy.y); stream_st(jo + 5 * P, jy.z);
    stream_st(jo + 6 * P, jz.x); stream_st(jo + 7 * P, jz.y); stream_st(jo + 8 * P, jz.z);
  }
}

__global__ __launch_bounds__(kThreads) void mark_visible_kernel(int P, const float* __restrict__ m,
                                                                const float* __restrict__ view,
                                                                uint8_t* __restrict__ present) {
  const int idx = (int)(blockIdx.x * kThreads + threadIdx.x);
  if (idx >= P) return;
  const V3 pv = xform_point43(v3(m[3 * idx], m[3 * idx + 1], m[3 * idx + 2]), view);
  present[idx] = !(pv.z <= 0.2f);
}

}  // namespace

hipError_t launch_preprocess(const PreArgs& a, hipStream_t s) {
  if (a.P == 0) return hipSuccess;
  hipLaunchKernelGGL(preprocess_kernel, dim3((a.P + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     s, a);
  return hipGetLastError();
}

hipError_t launch_preprocess_views(const PreArgs* views, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  const PreArgs& a0 = views[0];
  if (a0.P == 0) return hipSuccess;
  PreViews m{};
  m.V = V;
  for (int k = 0; k < V; k++) {
    const PreArgs& a = views[k];
    // one model: the view-independent fields must agree
    if (a.P != a0.P || a.means3D != a0.means3D || a.scales != a0.scales ||
        a.rotations != a0.rotations || a.opacities != a0.opacities ||
        a.cov3D_precomp != a0.cov3D_precomp || a.confidence != a0.confidence ||
        a.sh_language != a0.sh_language || a.lang_precomp != a0.lang_precomp ||
        a.fused != a0.fused || a.include_feature != a0.include_feature ||
        a.scale_modifier != a0.scale_modifier)
      return hipErrorInvalidValue;
    m.v[k] = a;
  }
  const uint32_t nblk = (uint32_t)((a0.P + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(preprocess_views_kernel, dim3(nblk), dim3(kThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t launch_sh_precolor(const PrecolorArgs& a, hipStream_t s) {
  if (a.P == 0 || a.nviews <= 0 || a.row1 <= a.row0) return hipSuccess;
  if (a.row1 > (uint32_t)a.P) return hipErrorInvalidValue;
  const dim3 grid((a.row1 - a.row0 + kPcThreads - 1) / kPcThreads);
  if (a.color[0] && a.jac[0])
    hipLaunchKernelGGL((sh_precolor_kernel<true, true>), grid, dim3(kPcThreads), 0, s, a);
  else if (a.color[0])
    hipLaunchKernelGGL((sh_precolor_kernel<true, false>), grid, dim3(kPcThreads), 0, s, a);
  else
    hipLaunchKernelGGL((sh_precolor_kernel<false, true>), grid, dim3(kPcThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present,
                               hipStream_t s) {
  if (P == 0) return hipSuccess;
  hipLaunchKernelGGL(mark_visible_kernel, dim3((P + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     s, P, means3D, view, present);
  return hipGetLastError();
}

}  // namespace gsr

/*
 * gsr_oracle.c -- CPU restatement of the reference differentiable Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY (see gsr_oracle.h).  Never linked into the product.
 *
 * Every function cites the reference file:line it restates; paths are relative to
 * /root/reference/submodules/diff-gaussian-rasterization/.  Parity pinning: the reference ships no
 * tests or golden vectors for this path and its CUDA sources cannot be built
 * here (no nvcc, un-vendored glm: SURVEY.md 8(c)), so this restatement is pinned by (a) golden
 * vectors generated from the importable reference Python maths (eval_sh, getProjectionMatrix,
 * getWorld2View2) in tests/golden/, (b) analytic known-answer cases, and (c) a float64 autograd
 * cross-check of the backward (tests/test_oracle.py).  Host threads (oracle_set_threads) only
 * split loops into fixed chunks; see the comment above par_for.
 */
#include "gsr_oracle.h"

#include <pthread.h>
#include <tgmath.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLOCK_X 16 /* config.h:16 */
#define BLOCK_Y 16 /* config.h:17 */
#define NCH 8      /* blend channels: r g b | depth | alpha | f0 f1 f2 */

/* Arithmetic type of the restatement (gsr_oracle.h ORACLE_REAL): float, the reference's own
 * type, for the checker the GPU path is compared with; double for the float64 build
 * (oracle/Makefile: _build/libgsr_oracle_f64.so), which evaluates the same expressions, in the
 * same order, on the same float32 inputs with the same float constants, so that per-entry
 * differences of float32 results against it measure float32 rounding (tests/test_f64_parity.py).
 * The float-defined helpers (splat_exp / splat_log and the exact tile cull) stay float. */
typedef ORACLE_REAL real;

/* SH constants, auxiliary.h:22-39 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ------------------------------------------------------------------------------------------ */
/* glm-like column-major 3x3 maths with glm's evaluation order (the reference uses glm, which  */
/* is un-vendored; column-major constructor semantics matter).                   */
/* ------------------------------------------------------------------------------------------ */
typedef struct { real x, y, z; } v3;
typedef struct { real m[3][3]; } m3; /* m[col][row] like glm::mat3 */

static m3 m3_cols(real a0, real a1, real a2, real b0, real b1, real b2, real c0, real c1,
                  real c2) {
    m3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = b0; r.m[1][1] = b1; r.m[1][2] = b2;
    r.m[2][0] = c0; r.m[2][1] = c1; r.m[2][2] = c2;
    return r;
}
/* glm operator*(mat3, mat3): R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2] */
static m3 m3_mul(m3 a, m3 b) {
    m3 r;
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++) {
            real t0 = a.m[0][w] * b.m[c][0];
            real t1 = a.m[1][w] * b.m[c][1];
            real t2 = a.m[2][w] * b.m[c][2];
            r.m[c][w] = t0 + t1 + t2;
        }
    return r;
}
static m3 m3_T(m3 a) {
    m3 r;
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++) r.m[c][w] = a.m[w][c];
    return r;
}
static m3 m3_scale(real s, m3 a) {
    m3 r;
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++) r.m[c][w] = s * a.m[c][w];
    return r;
}
static real v3_dot(v3 a, v3 b) {
    real tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return tx + ty + tz;
}
static v3 v3_mk(real x, real y, real z) { v3 r = {x, y, z}; return r; }
static v3 v3_add(v3 a, v3 b) { return v3_mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 v3_sub(v3 a, v3 b) { return v3_mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 v3_muls(real s, v3 a) { return v3_mk(s * a.x, s * a.y, s * a.z); }
static v3 v3_mul_s(v3 a, real s) { return v3_mk(a.x * s, a.y * s, a.z * s); }

/* CUDA/HIP float->int conversion semantics: round toward zero, saturate, NaN -> 0. */
static int f2i_sat(real f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}
static real fminf_cuda(real a, real b) { return fmin(a, b); }
static real fmaxf_cuda(real a, real b) { return fmax(a, b); }

/* The blend's Gaussian weight exp(power) (forward.cu:343, backward.cu:498 call expf): the same
 * deterministic single-precision exp the HIP kernels evaluate (sdp-gs_amd/csrc/gsr_device.h
 * splat_exp), every step a correctly rounded IEEE operation (fmaf, rintf, ldexpf).  <= 1.01 ulp of
 * exp over [-87, 0]; the reference's CUDA expf is specified to 2 ulp.  Sharing it makes the
 * alpha >= 1/255 and T < 1e-4 decisions of GPU and oracle identical pixel for pixel. */
static float splat_exp(float x) {
    const float k = rintf(x * 1.44269504088896341f);
    float r = fmaf(-k, 0.693359375f, x);
    r = fmaf(-k, -2.12194440e-4f, r);
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    const float r2 = r * r;
    const float y = fmaf(p, r2, r) + 1.0f;
    const float res = ldexpf(y, (int)k);
    return x < -104.0f ? 0.0f : res;
}
/* The blend's G = exp(power) in the arithmetic type: splat_exp for the float checker (or libm's
 * expf under -DORACLE_LIBM_EXP, the build the threshold census compares with), exp() in the
 * float64 build. */
static real blend_exp(real x) {
#if defined(ORACLE_LIBM_EXP)
    return expf(x);
#else
    if (sizeof(real) == sizeof(float)) return splat_exp((float)x);
    return exp(x);
#endif
}
void oracle_splat_exp(long n, const float* x, float* out) {
    for (long i = 0; i < n; i++) out[i] = splat_exp(x[i]);
}

/* ------------------------------------------------------------------------------------------ */
/* Exact tile culling of the HIP build (sdp-gs_amd/csrc/gsr_device.h).  Not in the  */
/* reference: its duplicateWithKeys emits every tile of the 3-sigma rectangle                    */
/* (rasterizer_impl.cu:94-109).  The build bins only the tiles of that rectangle where a splat   */
/* can reach alpha >= 1/255 at some pixel centre; this restatement (same float operations, same */
/* order, -ffp-contract=off) lets the tests pin the build's instance list to the reference's     */
/* list filtered by that predicate (tests/test_index_parity.py).                                */
/* ------------------------------------------------------------------------------------------ */
static float splat_log(float x) { /* gsr_device.h splat_log: Cephes logf, explicit fmaf steps */
    int e;
    float m = frexpf(x, &e);
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = (m + m) - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = fmaf(y, m, -1.1514610310e-1f);
    y = fmaf(y, m, 1.1676998740e-1f);
    y = fmaf(y, m, -1.2420140846e-1f);
    y = fmaf(y, m, 1.4249322787e-1f);
    y = fmaf(y, m, -1.6668057665e-1f);
    y = fmaf(y, m, 2.0000714765e-1f);
    y = fmaf(y, m, -2.4999993993e-1f);
    y = fmaf(y, m, 3.3333331174e-1f);
    y = (y * m) * z;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    const float r = m + y;
    return fmaf(fe, 0.693359375f, r);
}
void oracle_splat_log(long n, const float* x, float* out) {
    for (long i = 0; i < n; i++) out[i] = splat_log(x[i]);
}
typedef struct { float mx, my, ica, cb, det, caQ, hx, hy, dyl, slack; int mode; } band_cut;
static float cut_q(float ca, float cb, float cc, float op) { /* gsr_device.h splat_q_cut */
    if (!(op >= 1.0f / 255.0f)) return -2.0f;
    if (!(ca > 0.0f && cc > 0.0f && ca * cc - cb * cb > 0.0f)) return -1.0f;
    return 2.0f * splat_log(255.0f * op);
}
/* gsr_device.h make_band_cut / band_extent / band_row_range: the binning's cut, the tiles of each
 * tile row that the x-extent of the margin-widened cut ellipse in that row's 16-pixel band meets
 * (float, the same operations in the same order as the kernels) */
static band_cut make_band_cut(float mx, float my, float ca, float cb, float cc, float qc) {
    band_cut s;
    memset(&s, 0, sizeof s);
    s.mx = mx; s.my = my;
    if (qc == -2.0f) { s.mode = 0; return s; }
    s.mode = 1;
    if (qc < 0.0f) return s;
    const float det = ca * cc - cb * cb;
    if (!(det > 0.0f)) return s;
    const float h2x = cc / det, h2y = ca / det;
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
    s.dyl = cb * (s.hx / cc);
    s.slack = 2e-3f + 4e-6f * fabsf(mx) + 1e-4f * s.hx;
    return s;
}
static int band_extent(const band_cut* s, float y0, float y1, float* pxl, float* pxr) {
    const float lo = fmaxf(y0 - s->my, -s->hy), hi = fminf(y1 - s->my, s->hy);
    if (lo > hi) return 0;
    const float rl = sqrtf(fmaxf(s->caQ - s->det * lo * lo, 0.0f));
    const float rh = sqrtf(fmaxf(s->caQ - s->det * hi * hi, 0.0f));
    const float cl = -s->cb * lo, ch = -s->cb * hi;
    float xl = fminf(cl - rl, ch - rh) * s->ica;
    float xr = fmaxf(cl + rl, ch + rh) * s->ica;
    if (s->dyl >= lo && s->dyl <= hi) xl = -s->hx;
    if (-s->dyl >= lo && -s->dyl <= hi) xr = s->hx;
    *pxl = xl - s->slack;
    *pxr = xr + s->slack;
    return 1;
}
static void band_row_range(const band_cut* s, unsigned ty, unsigned x0, unsigned x1, unsigned* pa,
                           unsigned* pb) {
    if (s->mode != 2) {
        *pa = x0;
        *pb = s->mode == 0 ? x0 : x1;
        return;
    }
    const float y0 = (float)(ty * BLOCK_Y);
    float xl, xr;
    if (!band_extent(s, y0, y0 + (float)(BLOCK_Y - 1), &xl, &xr)) {
        *pa = *pb = x1;
        return;
    }
    const float fa = fminf(fmaxf(ceilf((s->mx + xl - (float)(BLOCK_X - 1)) * (1.0f / BLOCK_X)), (float)x0), (float)x1);
    const float fb = fminf(fmaxf(floorf((s->mx + xr) * (1.0f / BLOCK_X)) + 1.0f, (float)x0), (float)x1);
    unsigned a = (unsigned)fa, b = (unsigned)fb;
    if (a >= b) a = b = x1;
    *pa = a;
    *pb = b;
}

/* auxiliary.h:41-44: promoted to double */
static real ndc2Pix(real v, int S) { return (real)((((double)v + 1.0) * S - 1.0) * 0.5); }

typedef struct { unsigned x, y; } u2;
/* auxiliary.h:46-56 */
static void getRect(real px, real py, int max_radius, u2* rmin, u2* rmax, unsigned gx,
                    unsigned gy) {
    int a = f2i_sat((px - (real)max_radius) / (real)BLOCK_X);
    int b = f2i_sat((py - (real)max_radius) / (real)BLOCK_Y);
    int c = f2i_sat((((px + (real)max_radius) + (real)BLOCK_X) - 1.0f) / (real)BLOCK_X);
    int d = f2i_sat((((py + (real)max_radius) + (real)BLOCK_Y) - 1.0f) / (real)BLOCK_Y);
    a = a > 0 ? a : 0; b = b > 0 ? b : 0; c = c > 0 ? c : 0; d = d > 0 ? d : 0;
    rmin->x = (unsigned)a < gx ? (unsigned)a : gx;
    rmin->y = (unsigned)b < gy ? (unsigned)b : gy;
    rmax->x = (unsigned)c < gx ? (unsigned)c : gx;
    rmax->y = (unsigned)d < gy ? (unsigned)d : gy;
}

/* auxiliary.h:58-87 */
static v3 transformPoint4x3(v3 p, const real* m) {
    return v3_mk(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                 m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                 m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
static void transformPoint4x4(v3 p, const real* m, real out[4]) {
    out[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    out[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    out[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    out[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}
/* auxiliary.h:89-97 */
static v3 transformVec4x3Transpose(v3 p, const real* m) {
    return v3_mk(m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
                 m[8] * p.x + m[9] * p.y + m[10] * p.z);
}
/* auxiliary.h:107-117 */
static v3 dnormvdv(v3 v, v3 dv) {
    real sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    real invsum32 = 1.0f / sqrt(sum2 * sum2 * sum2);
    v3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* State                                                                                      */
/* ------------------------------------------------------------------------------------------ */
struct oracle_state {
    int P, M, D, W, H, prefiltered, include_feature;
    unsigned gx, gy;
    real scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    real bg[3], view[16], proj[16], campos[3];
    float viewf[16]; /* the float32 view matrix (the depth-sort key, below) */
    /* inputs (borrowed: the caller keeps them alive between forward and backward) */
    const float *means3D, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp, *sh,
        *sh_language, *lang_precomp, *confidence;
    /* geometry (GeometryState, rasterizer_impl.h:21-37) */
    real* depths;
    float* depth_key; /* the reference's float32 view-space z: the depth-sort key */
    unsigned char* clamped; /* [P*3] */
    int* radii;
    real* means2D;       /* [P*2] */
    real* cov3D;         /* [P*6] */
    real* conic_opacity; /* [P*4] (opacity already multiplied by confidence) */
    real* rgb;           /* [P*3] */
    real* feat;          /* [P*3] */
    unsigned* tiles_touched;
    /* binning */
    int R;
    unsigned* point_list;
    unsigned* ranges; /* [tiles*2] */
    /* image */
    real* final_T;
    unsigned* n_contrib;
    real* margin; /* [H*W] test-side diagnostic, see oracle_get_margin */
    /* decision lock (oracle_use_decisions): per pixel, another evaluation's blend decisions --
     * its n_contrib and, over list positions [0, n_contrib), the bitset of the splats it blended
     * (lock_offs[pix] = the pixel's first 32-bit word) -- replace this build's own alpha >= 1/255,
     * power <= 0 and T < 1e-4 tests in the blends.  NULL = no lock. */
    unsigned* lock_nc;
    uint64_t* lock_offs;
    unsigned* lock_words;
    /* colour-clamp lock (oracle_use_clamp): another evaluation's SH colour clamp bits [P*3]
     * replace this build's own result < 0 tests (forward.cu:67-69; the backward's dL/dRGB mask,
     * backward.cu:390-391).  NULL = no lock. */
    unsigned char* clamp_lock;
};

/* forward.cu:20-71 computeColorFromSH */
static v3 color_from_sh(int idx, int deg, int max_coeffs, const float* means, const real* campos,
                        const float* shs, unsigned char* clamped, const unsigned char* lock) {
    v3 pos = v3_mk(means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]);
    v3 dir = v3_sub(pos, v3_mk(campos[0], campos[1], campos[2]));
    real len = sqrt(v3_dot(dir, dir));
    dir = v3_mk(dir.x / len, dir.y / len, dir.z / len);
    const float* s = shs + (size_t)idx * max_coeffs * 3;
#define SH(k) v3_mk(s[3 * (k)], s[3 * (k) + 1], s[3 * (k) + 2])
    v3 result = v3_muls(SH_C0, SH(0));
    if (deg > 0) {
        real x = dir.x, y = dir.y, z = dir.z;
        result = v3_sub(v3_add(v3_sub(result, v3_muls(SH_C1 * y, SH(1))), v3_muls(SH_C1 * z, SH(2))),
                        v3_muls(SH_C1 * x, SH(3)));
        if (deg > 1) {
            real xx = x * x, yy = y * y, zz = z * z;
            real xy = x * y, yz = y * z, xz = x * z;
            result = v3_add(result, v3_muls(SH_C2[0] * xy, SH(4)));
            result = v3_add(result, v3_muls(SH_C2[1] * yz, SH(5)));
            result = v3_add(result, v3_muls(SH_C2[2] * (2.0f * zz - xx - yy), SH(6)));
            result = v3_add(result, v3_muls(SH_C2[3] * xz, SH(7)));
            result = v3_add(result, v3_muls(SH_C2[4] * (xx - yy), SH(8)));
            if (deg > 2) {
                result = v3_add(result, v3_muls(SH_C3[0] * y * (3.0f * xx - yy), SH(9)));
                result = v3_add(result, v3_muls(SH_C3[1] * xy * z, SH(10)));
                result = v3_add(result, v3_muls(SH_C3[2] * y * (4.0f * zz - xx - yy), SH(11)));
                result = v3_add(result,
                                v3_muls(SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), SH(12)));
                result = v3_add(result, v3_muls(SH_C3[4] * x * (4.0f * zz - xx - yy), SH(13)));
                result = v3_add(result, v3_muls(SH_C3[5] * z * (xx - yy), SH(14)));
                result = v3_add(result, v3_muls(SH_C3[6] * x * (xx - 3.0f * yy), SH(15)));
            }
        }
    }
#undef SH
    result = v3_mk(result.x + 0.5f, result.y + 0.5f, result.z + 0.5f);
    clamped[3 * idx + 0] = result.x < 0;
    clamped[3 * idx + 1] = result.y < 0;
    clamped[3 * idx + 2] = result.z < 0;
    if (lock) { /* oracle_use_clamp: the other evaluation's decisions, colour and mask alike */
        clamped[3 * idx + 0] = lock[3 * idx + 0];
        clamped[3 * idx + 1] = lock[3 * idx + 1];
        clamped[3 * idx + 2] = lock[3 * idx + 2];
        return v3_mk(clamped[3 * idx + 0] ? 0 : result.x, clamped[3 * idx + 1] ? 0 : result.y,
                     clamped[3 * idx + 2] ? 0 : result.z);
    }
    return v3_mk(fmaxf_cuda(result.x, 0.0f), fmaxf_cuda(result.y, 0.0f), fmaxf_cuda(result.z, 0.0f));
}

/* forward.cu:74-113 computeCov2D */
static void cov2d(v3 mean, real fx, real fy, real tanx, real tany, const real* c3,
                  const real* view, real out[3]) {
    v3 t = transformPoint4x3(mean, view);
    const real limx = 1.3f * tanx;
    const real limy = 1.3f * tany;
    const real txtz = t.x / t.z;
    const real tytz = t.y / t.z;
    t.x = fminf_cuda(limx, fmaxf_cuda(-limx, txtz)) * t.z;
    t.y = fminf_cuda(limy, fmaxf_cuda(-limy, tytz)) * t.z;
    m3 J = m3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z,
                   -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    m3 W = m3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6],
                   view[10]);
    m3 T = m3_mul(W, J);
    m3 Vrk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    m3 cov = m3_mul(m3_mul(m3_T(T), m3_T(Vrk)), T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out[0] = cov.m[0][0];
    out[1] = cov.m[0][1];
    out[2] = cov.m[1][1];
}

/* forward.cu:118-152 computeCov3D (no quaternion normalisation, :127) */
static void cov3d(const float* scale, real mod, const float* rot, real* out) {
    m3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    real r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    m3 R = m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    m3 M = m3_mul(S, R);
    m3 Sigma = m3_mul(m3_T(M), M);
    out[0] = Sigma.m[0][0];
    out[1] = Sigma.m[0][1];
    out[2] = Sigma.m[0][2];
    out[3] = Sigma.m[1][1];
    out[4] = Sigma.m[1][2];
    out[5] = Sigma.m[2][2];
}

/* auxiliary.h:139-164 in_frustum (near-plane test only) */
static int in_frustum(int idx, const float* pts, const real* view, v3* p_view) {
    v3 p = v3_mk(pts[3 * idx], pts[3 * idx + 1], pts[3 * idx + 2]);
    *p_view = transformPoint4x3(p, view);
    return !(p_view->z <= 0.2f);
}

int oracle_mark_visible(int P, const float* means3D, const float* viewmatrix,
                        const float* projmatrix, unsigned char* present) {
    (void)projmatrix; /* in_frustum computes p_proj but only uses p_view (auxiliary.h:149-154) */
    real view[16];
    for (int k = 0; k < 16; k++) view[k] = viewmatrix[k];
    for (int i = 0; i < P; i++) {
        v3 pv;
        present[i] = (unsigned char)in_frustum(i, means3D, view, &pv);
    }
    return 0;
}

typedef struct { uint64_t key; uint32_t seq; uint32_t val; } inst_t;
static int inst_cmp(const void* a, const void* b) {
    const inst_t* x = (const inst_t*)a;
    const inst_t* y = (const inst_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->seq < y->seq ? -1 : (x->seq > y->seq ? 1 : 0); /* stable: SortPairs is stable */
}

static void* xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

/* ------------------------------------------------------------------------------------------ */
/* Host threads, for the full-size parity tests and the CPU baseline (oracle_set_threads).    */
/* With 1 thread (the default) every loop runs in the reference's sequential order.  With n:  */
/* the per-Gaussian and per-pixel-row loops run as n contiguous static chunks (each element is */
/* computed by the same code, so the forward is bit-identical); the instance sort sorts n runs */
/* and merges them (the comparator is a total order, so the order is identical); the backward */
/* blend sums each chunk's contributions into private accumulators, added in chunk order      */
/* afterwards (deterministic for a given n; the sums differ from the sequential ones only by   */
/* float association, as the reference's own atomics do).                                     */
/* ------------------------------------------------------------------------------------------ */
#define ORACLE_MAX_THREADS 256
static int g_threads = 1;
void oracle_set_threads(int n) {
    g_threads = n < 1 ? 1 : (n > ORACLE_MAX_THREADS ? ORACLE_MAX_THREADS : n);
}
int oracle_get_threads(void) { return g_threads; }

typedef void (*range_fn)(void* ctx, long lo, long hi, int chunk);
typedef struct { range_fn fn; void* ctx; long lo, hi; int chunk; } par_job;
static void* par_entry(void* p) {
    par_job* j = (par_job*)p;
    j->fn(j->ctx, j->lo, j->hi, j->chunk);
    return NULL;
}
/* Chunk count par_for(n, ...) uses. */
static int par_chunks(long n) {
    int nt = g_threads;
    if ((long)nt > n) nt = n > 0 ? (int)n : 1;
    return nt;
}
/* fn over [0, n) in par_chunks(n) contiguous chunks, chunk c on its own thread. */
static void par_for(long n, range_fn fn, void* ctx) {
    const int nt = par_chunks(n);
    if (nt <= 1) { fn(ctx, 0, n, 0); return; }
    pthread_t th[ORACLE_MAX_THREADS];
    par_job job[ORACLE_MAX_THREADS];
    int started[ORACLE_MAX_THREADS];
    const long base = n / nt, rem = n % nt;
    for (int c = 0; c < nt; c++) {
        job[c].fn = fn; job[c].ctx = ctx; job[c].chunk = c;
        job[c].lo = c * base + (c < rem ? c : rem);
        job[c].hi = job[c].lo + base + (c < rem ? 1 : 0);
    }
    for (int c = 1; c < nt; c++) started[c] = pthread_create(&th[c], NULL, par_entry, &job[c]) == 0;
    par_entry(&job[0]);
    for (int c = 1; c < nt; c++) {
        if (started[c]) pthread_join(th[c], NULL);
        else par_entry(&job[c]); /* could not start a thread: run the chunk here */
    }
}

/* ---- preprocessCUDA, forward.cu:155-256 (one Gaussian) ---- */
static void preprocess_one(oracle_state* st, int idx) {
    const float* means3D = st->means3D;
    const int W = st->W, H = st->H;
    st->radii[idx] = 0;
    st->tiles_touched[idx] = 0;
    v3 p_view;
    if (!in_frustum(idx, means3D, st->view, &p_view)) return;
    v3 p_orig = v3_mk(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    real p_hom[4];
    transformPoint4x4(p_orig, st->proj, p_hom);
    real p_w = 1.0f / (p_hom[3] + 0.0000001f);
    real p_proj_x = p_hom[0] * p_w, p_proj_y = p_hom[1] * p_w;
    /* cov3D_precomp was converted into st->cov3D by oracle_forward */
    if (!st->cov3D_precomp)
        cov3d(st->scales + 3 * (size_t)idx, st->scale_modifier, st->rotations + 4 * (size_t)idx,
              st->cov3D + (size_t)idx * 6);
    const real* c3 = st->cov3D + (size_t)idx * 6;
    real cov[3];
    cov2d(p_orig, st->focal_x, st->focal_y, st->tan_fovx, st->tan_fovy, c3, st->view, cov);
    real det = (cov[0] * cov[2] - cov[1] * cov[1]);
    if (det == 0.0f) return;
    real det_inv = 1.f / det;
    real conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
    real mid = 0.5f * (cov[0] + cov[2]);
    real lambda1 = mid + sqrt(fmaxf_cuda(0.1f, mid * mid - det));
    real lambda2 = mid - sqrt(fmaxf_cuda(0.1f, mid * mid - det));
    real my_radius = ceil(3.f * sqrt(fmaxf_cuda(lambda1, lambda2)));
    real pix_x = ndc2Pix(p_proj_x, W), pix_y = ndc2Pix(p_proj_y, H);
    u2 rmin, rmax;
    getRect(pix_x, pix_y, f2i_sat(my_radius), &rmin, &rmax, st->gx, st->gy);
    if ((rmax.x - rmin.x) * (rmax.y - rmin.y) == 0) return;
    if (!st->colors_precomp) {
        v3 c = color_from_sh(idx, st->D, st->M, means3D, st->campos, st->sh, st->clamped,
                             st->clamp_lock);
        st->rgb[3 * idx + 0] = c.x;
        st->rgb[3 * idx + 1] = c.y;
        st->rgb[3 * idx + 2] = c.z;
    }
    st->depths[idx] = p_view.z;
    {   /* forward.cu:227 depths[idx] = p_view.z in float32 (auxiliary.h:58-64): the key bits the
         * binning sorts by (rasterizer_impl.cu:95), so the float64 build orders every tile's list
         * exactly as the float32 one -- near-equal depths would otherwise swap */
        const float* m = st->viewf;
        const float px = means3D[3 * idx], py = means3D[3 * idx + 1], pz = means3D[3 * idx + 2];
        st->depth_key[idx] = m[2] * px + m[6] * py + m[10] * pz + m[14];
    }
    st->radii[idx] = f2i_sat(my_radius);
    st->means2D[2 * idx] = pix_x;
    st->means2D[2 * idx + 1] = pix_y;
    real op = st->opacities[idx];
    if (st->confidence) op = op * st->confidence[idx]; /* confidence = opacity multiplier */
    st->conic_opacity[4 * idx + 0] = conic[0];
    st->conic_opacity[4 * idx + 1] = conic[1];
    st->conic_opacity[4 * idx + 2] = conic[2];
    st->conic_opacity[4 * idx + 3] = op;
    st->tiles_touched[idx] = (rmax.y - rmin.y) * (rmax.x - rmin.x);
    if (st->include_feature) { /* language feature channels */
        if (st->lang_precomp) {
            for (int k = 0; k < 3; k++) st->feat[3 * idx + k] = st->lang_precomp[3 * idx + k];
        } else if (st->sh_language) {
            const float* l = st->sh_language;
            real u0 = SH_C0 * l[3 * idx], u1 = SH_C0 * l[3 * idx + 1], u2v = SH_C0 * l[3 * idx + 2];
            real n = sqrt(u0 * u0 + u1 * u1 + u2v * u2v);
            real den = n + 1e-9f;
            st->feat[3 * idx + 0] = u0 / den;
            st->feat[3 * idx + 1] = u1 / den;
            st->feat[3 * idx + 2] = u2v / den;
        }
    }
}
static void preprocess_range(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    for (long i = lo; i < hi; i++) preprocess_one((oracle_state*)ctx, (int)i);
}

/* ---- stable sort of the instances: per-chunk qsort + pairwise merges (same total order) ---- */
typedef struct { inst_t* a; const long* b; } sort_ctx;
static void sort_runs(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    sort_ctx* c = (sort_ctx*)ctx;
    for (long r = lo; r < hi; r++)
        qsort(c->a + c->b[r], (size_t)(c->b[r + 1] - c->b[r]), sizeof(inst_t), inst_cmp);
}
typedef struct { const inst_t* src; inst_t* dst; const long* b; int nruns; } merge_ctx;
static void merge_runs(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    merge_ctx* m = (merge_ctx*)ctx;
    for (long k = lo; k < hi; k++) {
        const long r = 2 * k;
        const long s0 = m->b[r], e0 = m->b[r + 1];
        const long e1 = (r + 2 <= m->nruns) ? m->b[r + 2] : e0;
        long i = s0, j = e0, o = s0;
        while (i < e0 && j < e1) m->dst[o++] = inst_cmp(&m->src[j], &m->src[i]) < 0 ? m->src[j++] : m->src[i++];
        while (i < e0) m->dst[o++] = m->src[i++];
        while (j < e1) m->dst[o++] = m->src[j++];
    }
}
static void sort_instances(inst_t* a, long n) {
    int nruns = par_chunks(n);
    inst_t* tmp = (nruns > 1 && n >= 4096) ? (inst_t*)malloc(sizeof(inst_t) * (size_t)n) : NULL;
    if (!tmp) {
        qsort(a, (size_t)n, sizeof(inst_t), inst_cmp);
        return;
    }
    long b[ORACLE_MAX_THREADS + 1];
    const long base = n / nruns, rem = n % nruns;
    for (int r = 0; r <= nruns; r++) b[r] = r * base + (r < rem ? r : rem);
    sort_ctx sc = {a, b};
    par_for(nruns, sort_runs, &sc);
    inst_t *src = a, *dst = tmp;
    while (nruns > 1) {
        const long npairs = (nruns + 1) / 2;
        merge_ctx mc = {src, dst, b, nruns};
        par_for(npairs, merge_runs, &mc);
        for (long k = 0; k < npairs; k++) b[k] = b[2 * k];
        b[npairs] = n;
        nruns = (int)npairs;
        inst_t* t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, sizeof(inst_t) * (size_t)n);
    free(tmp);
}

/* ---- renderCUDA (fwd), forward.cu:261-374, extended to NCH channels; rows [lo, hi) ---- */
typedef struct {
    oracle_state* st;
    const float* background;
    real *out_color, *out_depth, *out_alpha, *out_feature;
} blend_fwd_ctx;
static void blend_fwd_rows(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    const blend_fwd_ctx* c = (const blend_fwd_ctx*)ctx;
    oracle_state* st = c->st;
    const int W = st->W, H = st->H;
    const unsigned gx = st->gx;
    const real* feat_ptr = st->rgb; /* colors_precomp converted into rgb by oracle_forward */
    const int nch = st->include_feature ? NCH : 5;
    for (long py = lo; py < hi; py++)
        for (int px = 0; px < W; px++) {
            const unsigned tile = (unsigned)(py / BLOCK_Y) * gx + (unsigned)(px / BLOCK_X);
            const unsigned rs = st->ranges[2 * tile], re = st->ranges[2 * tile + 1];
            const real pfx = (real)px, pfy = (real)py;
            real T = 1.0f;
            unsigned contributor = 0, last_contributor = 0;
            real C[NCH] = {0};
            real margin = 1.0f;
            const size_t lpix = (size_t)py * W + px;
            const unsigned lock_nc = st->lock_nc ? st->lock_nc[lpix] : 0;
            const unsigned* lock_w = st->lock_nc ? st->lock_words + st->lock_offs[lpix] : NULL;
            for (unsigned k = rs; k < re; k++) {
                contributor++;
                if (lock_w && contributor > lock_nc) break; /* the locked evaluation stopped here */
                const unsigned g = st->point_list[k];
                const real dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                const real* co = st->conic_opacity + 4 * (size_t)g;
                real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                const unsigned q = contributor - 1;
                const int lock_take = lock_w ? (int)((lock_w[q >> 5] >> (q & 31)) & 1u) : -1;
                if (fabs(power) < 1e-6f) margin = 0.0f;
                if (lock_take == 0 || (lock_take < 0 && power > 0.0f)) continue;
                real alpha = fminf_cuda(0.99f, co[3] * blend_exp(power));
                margin = fmin(margin, fabs(alpha * 255.0f - 1.0f));
                if (lock_take < 0 && alpha < 1.0f / 255.0f) continue;
                real test_T = T * (1 - alpha);
                margin = fmin(margin, fabs(test_T * 1e4f - 1.0f));
                if (lock_take < 0 && test_T < 0.0001f) break; /* done: nothing later changes this pixel */
                real v[NCH];
                v[0] = feat_ptr[3 * g]; v[1] = feat_ptr[3 * g + 1]; v[2] = feat_ptr[3 * g + 2];
                v[3] = st->depths[g]; v[4] = 1.0f;
                v[5] = st->feat[3 * g]; v[6] = st->feat[3 * g + 1]; v[7] = st->feat[3 * g + 2];
                for (int ch = 0; ch < nch; ch++) C[ch] += v[ch] * alpha * T;
                T = test_T;
                last_contributor = contributor;
            }
            const size_t pix = (size_t)py * W + px, HW = (size_t)W * H;
            st->final_T[pix] = T;
            st->n_contrib[pix] = last_contributor;
            st->margin[pix] = margin;
            for (int ch = 0; ch < 3; ch++) c->out_color[ch * HW + pix] = C[ch] + T * c->background[ch];
            if (c->out_depth) c->out_depth[pix] = C[3];
            if (c->out_alpha) c->out_alpha[pix] = C[4];
            if (c->out_feature)
                for (int ch = 0; ch < 3; ch++)
                    c->out_feature[ch * HW + pix] = st->include_feature ? C[5 + ch] : 0.0f;
        }
}

/* oracle_use_lists: the next oracle_forward on this thread takes these instance lists instead of
 * binning itself (the float64 build run on the float32 build's lists, so that both blend the
 * same instances in the same order even where a radius rounds to another integer). */
static _Thread_local struct { const unsigned *point_list, *ranges; int R; } g_lists;
void oracle_use_lists(const unsigned* point_list, int R, const unsigned* ranges) {
    g_lists.point_list = point_list;
    g_lists.R = R;
    g_lists.ranges = ranges;
}

/* oracle_use_decisions: the next oracle_forward on this thread blends with another evaluation's
 * per-pixel decisions (oracle_accept_bits of a float32 run) instead of its own threshold tests --
 * the float64 build then sums exactly the terms float32 summed, so every remaining difference is
 * rounding (tests/f64_ref.py).  The arrays are copied into the state. */
static _Thread_local struct { const unsigned *nc, *words; const uint64_t* offs; } g_lock;
void oracle_use_decisions(const unsigned* n_contrib, const uint64_t* word_offsets,
                          const unsigned* words) {
    g_lock.nc = n_contrib;
    g_lock.offs = word_offsets;
    g_lock.words = words;
}

/* oracle_use_clamp: the next oracle_forward on this thread takes another evaluation's SH colour
 * clamp bits (oracle_get_clamped, [P*3]) instead of its own result < 0 tests (copied). */
static _Thread_local const unsigned char* g_clamp;
void oracle_use_clamp(const unsigned char* clamped) { g_clamp = clamped; }

/* oracle_use_geometry: the next oracle_forward on this thread blends with another evaluation's
 * projected splats -- screen means [P*2] and conic + opacity [P*4] (oracle_get_means2D /
 * oracle_get_conic_opacity, float32) -- instead of its own preprocess's (float64 parity: the
 * float32 pixel coordinates carry ~1e-4 px of rounding at x ~ 1500, which the Gaussian's falloff
 * turns into ~1e-4 relative changes of G at the splat's edge; with the float32 geometry the
 * float64 blend sums exactly the float32 terms).  The arrays are read during that call. */
static _Thread_local struct { const float *means2D, *conic_opacity; } g_geom;
void oracle_use_geometry(const float* means2D, const float* conic_opacity) {
    g_geom.means2D = means2D;
    g_geom.conic_opacity = conic_opacity;
}

/* The blend decisions of a forward: per pixel the 32-bit word offset of its bitset (offs[H*W+1],
 * a prefix sum of ceil(n_contrib / 32)) and, when words != NULL, the bitset of the list positions
 * [0, n_contrib) it blended (power <= 0 and alpha >= 1/255, recomputed with the forward's own
 * arithmetic).  Returns the number of words. */
long oracle_accept_bits(const oracle_state* st, uint64_t* offs, unsigned* words) {
    const int W = st->W, H = st->H;
    const size_t HW = (size_t)W * H;
    uint64_t o = 0;
    for (size_t pix = 0; pix < HW; pix++) {
        offs[pix] = o;
        o += (st->n_contrib[pix] + 31u) / 32u;
    }
    offs[HW] = o;
    if (!words) return (long)o;
    memset(words, 0, sizeof(unsigned) * (size_t)o);
    for (int py = 0; py < H; py++)
        for (int px = 0; px < W; px++) {
            const size_t pix = (size_t)py * W + px;
            const unsigned tile = (unsigned)(py / BLOCK_Y) * st->gx + (unsigned)(px / BLOCK_X);
            const unsigned rs = st->ranges[2 * tile], nc = st->n_contrib[pix];
            const real pfx = (real)px, pfy = (real)py;
            for (unsigned q = 0; q < nc; q++) {
                const unsigned g = st->point_list[rs + q];
                const real dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                const real* co = st->conic_opacity + 4 * (size_t)g;
                const real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (power > 0.0f) continue;
                if (fminf_cuda(0.99f, co[3] * blend_exp(power)) < 1.0f / 255.0f) continue;
                words[offs[pix] + (q >> 5)] |= 1u << (q & 31);
            }
        }
    return (long)o;
}

oracle_state* oracle_forward(int P, int M, const float* background, const float* means3D,
                             const float* colors_precomp, const float* opacities,
                             const float* scales, const float* rotations, float scale_modifier,
                             const float* cov3D_precomp, const float* viewmatrix,
                             const float* projmatrix, float tan_fovx, float tan_fovy,
                             int image_height, int image_width, const float* sh, int degree,
                             const float* campos, int prefiltered, const float* sh_language,
                             const float* language_feature_precomp, const float* confidence,
                             int include_feature, real* out_color, real* out_depth,
                             real* out_alpha, real* out_feature, int* radii_out,
                             int* num_rendered) {
    if (P < 0 || image_height <= 0 || image_width <= 0) return NULL;
    if (!colors_precomp && !sh) return NULL;
    if (!cov3D_precomp && (!scales || !rotations)) return NULL;
    oracle_state* st = (oracle_state*)calloc(1, sizeof(oracle_state));
    const int W = image_width, H = image_height;
    st->P = P; st->M = M; st->D = degree; st->W = W; st->H = H;
    st->prefiltered = prefiltered; st->include_feature = include_feature;
    st->scale_modifier = scale_modifier; st->tan_fovx = tan_fovx; st->tan_fovy = tan_fovy;
    /* rasterizer_impl.cu:222-223 */
    st->focal_y = (real)H / (2.0f * tan_fovy);
    st->focal_x = (real)W / (2.0f * tan_fovx);
    for (int k = 0; k < 3; k++) st->bg[k] = background[k];
    for (int k = 0; k < 16; k++) st->view[k] = viewmatrix[k];
    memcpy(st->viewf, viewmatrix, sizeof(st->viewf));
    for (int k = 0; k < 16; k++) st->proj[k] = projmatrix[k];
    for (int k = 0; k < 3; k++) st->campos[k] = campos[k];
    st->means3D = means3D; st->colors_precomp = colors_precomp; st->opacities = opacities;
    st->scales = scales; st->rotations = rotations; st->cov3D_precomp = cov3D_precomp;
    st->sh = sh; st->sh_language = sh_language; st->lang_precomp = language_feature_precomp;
    st->confidence = confidence;
    /* rasterizer_impl.cu:234 */
    st->gx = (unsigned)((W + BLOCK_X - 1) / BLOCK_X);
    st->gy = (unsigned)((H + BLOCK_Y - 1) / BLOCK_Y);
    const unsigned gx = st->gx, gy = st->gy;

    st->depths = (real*)xcalloc(P, sizeof(real));
    st->depth_key = (float*)xcalloc(P, sizeof(float));
    st->clamped = (unsigned char*)xcalloc((size_t)P * 3, 1);
    if (g_clamp) { /* oracle_use_clamp: copied, applied by the preprocess below */
        st->clamp_lock = (unsigned char*)xcalloc((size_t)P * 3, 1);
        memcpy(st->clamp_lock, g_clamp, (size_t)P * 3);
        g_clamp = NULL;
    }
    st->radii = (int*)xcalloc(P, sizeof(int));
    st->means2D = (real*)xcalloc((size_t)P * 2, sizeof(real));
    st->cov3D = (real*)xcalloc((size_t)P * 6, sizeof(real));
    st->conic_opacity = (real*)xcalloc((size_t)P * 4, sizeof(real));
    st->rgb = (real*)xcalloc((size_t)P * 3, sizeof(real));
    st->feat = (real*)xcalloc((size_t)P * 3, sizeof(real));
    st->tiles_touched = (unsigned*)xcalloc(P, sizeof(unsigned));

    /* ---- preprocessCUDA, forward.cu:155-256 ---- */
    /* precomputed colours / covariances in the arithmetic type (exact for float) */
    if (colors_precomp)
        for (size_t i = 0; i < (size_t)P * 3; i++) st->rgb[i] = colors_precomp[i];
    if (cov3D_precomp)
        for (size_t i = 0; i < (size_t)P * 6; i++) st->cov3D[i] = cov3D_precomp[i];
    par_for(P, preprocess_range, st);
    if (radii_out) memcpy(radii_out, st->radii, sizeof(int) * (size_t)P);
    if (g_geom.means2D) { /* oracle_use_geometry: another evaluation's projected splats */
        for (size_t i = 0; i < (size_t)P * 2; i++) st->means2D[i] = g_geom.means2D[i];
        for (size_t i = 0; i < (size_t)P * 4; i++) st->conic_opacity[i] = g_geom.conic_opacity[i];
        g_geom.means2D = NULL;
        g_geom.conic_opacity = NULL;
    }

    /* ---- scan + duplicateWithKeys + stable SortPairs, rasterizer_impl.cu:70-111, 277-308 ---- */
    const unsigned ntiles = gx * gy;
    if (g_lists.point_list) { /* oracle_use_lists: another evaluation's binning, as given */
        const int R = g_lists.R;
        st->R = R;
        st->point_list = (unsigned*)xcalloc((size_t)R, sizeof(unsigned));
        memcpy(st->point_list, g_lists.point_list, sizeof(unsigned) * (size_t)R);
        st->ranges = (unsigned*)xcalloc((size_t)ntiles * 2, sizeof(unsigned));
        memcpy(st->ranges, g_lists.ranges, sizeof(unsigned) * 2 * (size_t)ntiles);
        if (num_rendered) *num_rendered = R;
        goto blend;
    }
    {
    uint64_t R64 = 0;
    for (int i = 0; i < P; i++) R64 += st->tiles_touched[i];
    int R = (int)R64;
    st->R = R;
    inst_t* inst = (inst_t*)xcalloc((size_t)R, sizeof(inst_t));
    uint32_t off = 0;
    for (int idx = 0; idx < P; idx++) {
        if (st->radii[idx] > 0) {
            u2 rmin, rmax;
            getRect(st->means2D[2 * idx], st->means2D[2 * idx + 1], st->radii[idx], &rmin, &rmax,
                    gx, gy);
            uint32_t dbits;
            memcpy(&dbits, &st->depth_key[idx], 4);
            for (unsigned y = rmin.y; y < rmax.y; y++)
                for (unsigned x = rmin.x; x < rmax.x; x++) {
                    uint64_t key = (uint64_t)(y * gx + x);
                    key <<= 32;
                    key |= dbits;
                    inst[off].key = key;
                    inst[off].seq = off;
                    inst[off].val = (uint32_t)idx;
                    off++;
                }
        }
    }
    sort_instances(inst, R);
    st->point_list = (unsigned*)xcalloc((size_t)R, sizeof(unsigned));
    for (int i = 0; i < R; i++) st->point_list[i] = inst[i].val;
    /* identifyTileRanges, rasterizer_impl.cu:116-138 (ranges zeroed first, :310) */
    st->ranges = (unsigned*)xcalloc((size_t)ntiles * 2, sizeof(unsigned));
    for (int i = 0; i < R; i++) {
        unsigned cur = (unsigned)(inst[i].key >> 32);
        if (i == 0) st->ranges[2 * cur] = 0;
        else {
            unsigned prev = (unsigned)(inst[i - 1].key >> 32);
            if (cur != prev) {
                st->ranges[2 * prev + 1] = (unsigned)i;
                st->ranges[2 * cur] = (unsigned)i;
            }
        }
        if (i == R - 1) st->ranges[2 * cur + 1] = (unsigned)R;
    }
    free(inst);
    if (num_rendered) *num_rendered = R;
    }

blend:
    if (g_lock.nc) { /* oracle_use_decisions: copied, so the lock outlives the caller's arrays */
        const size_t HW = (size_t)W * H;
        const uint64_t nw = g_lock.offs[HW];
        st->lock_nc = (unsigned*)xcalloc(HW, sizeof(unsigned));
        st->lock_offs = (uint64_t*)xcalloc(HW + 1, sizeof(uint64_t));
        st->lock_words = (unsigned*)xcalloc((size_t)nw, sizeof(unsigned));
        memcpy(st->lock_nc, g_lock.nc, sizeof(unsigned) * HW);
        memcpy(st->lock_offs, g_lock.offs, sizeof(uint64_t) * (HW + 1));
        memcpy(st->lock_words, g_lock.words, sizeof(unsigned) * (size_t)nw);
    }
    /* ---- renderCUDA (fwd), forward.cu:261-374, extended to NCH channels ---- */
    st->final_T = (real*)xcalloc((size_t)W * H, sizeof(real));
    st->n_contrib = (unsigned*)xcalloc((size_t)W * H, sizeof(unsigned));
    st->margin = (real*)xcalloc((size_t)W * H, sizeof(real));
    blend_fwd_ctx bc = {st, background, out_color, out_depth, out_alpha, out_feature};
    par_for(H, blend_fwd_rows, &bc);
    return st;
}

/* backward.cu:20-139 computeColorFromSH (bwd) */
static void sh_backward(int idx, int deg, int max_coeffs, const float* means, const real* campos,
                        const float* shs, const unsigned char* clamped, const real* dL_dcolor,
                        real* dL_dmeans, real* dL_dshs) {
    v3 pos = v3_mk(means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]);
    v3 dir_orig = v3_sub(pos, v3_mk(campos[0], campos[1], campos[2]));
    real len = sqrt(v3_dot(dir_orig, dir_orig));
    v3 dir = v3_mk(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    const float* s = shs + (size_t)idx * max_coeffs * 3;
#define SH(k) v3_mk(s[3 * (k)], s[3 * (k) + 1], s[3 * (k) + 2])
    v3 dL_dRGB = v3_mk(dL_dcolor[3 * idx], dL_dcolor[3 * idx + 1], dL_dcolor[3 * idx + 2]);
    dL_dRGB.x *= clamped[3 * idx + 0] ? 0 : 1;
    dL_dRGB.y *= clamped[3 * idx + 1] ? 0 : 1;
    dL_dRGB.z *= clamped[3 * idx + 2] ? 0 : 1;
    v3 dRGBdx = v3_mk(0, 0, 0), dRGBdy = v3_mk(0, 0, 0), dRGBdz = v3_mk(0, 0, 0);
    real x = dir.x, y = dir.y, z = dir.z;
    real* d = dL_dshs + (size_t)idx * max_coeffs * 3;
#define PUT(k, v) do { v3 _t = (v); d[3 * (k)] = _t.x; d[3 * (k) + 1] = _t.y; d[3 * (k) + 2] = _t.z; } while (0)
    real dRGBdsh0 = SH_C0;
    PUT(0, v3_muls(dRGBdsh0, dL_dRGB));
    if (deg > 0) {
        real dRGBdsh1 = -SH_C1 * y;
        real dRGBdsh2 = SH_C1 * z;
        real dRGBdsh3 = -SH_C1 * x;
        PUT(1, v3_muls(dRGBdsh1, dL_dRGB));
        PUT(2, v3_muls(dRGBdsh2, dL_dRGB));
        PUT(3, v3_muls(dRGBdsh3, dL_dRGB));
        dRGBdx = v3_muls(-SH_C1, SH(3));
        dRGBdy = v3_muls(-SH_C1, SH(1));
        dRGBdz = v3_muls(SH_C1, SH(2));
        if (deg > 1) {
            real xx = x * x, yy = y * y, zz = z * z;
            real xy = x * y, yz = y * z, xz = x * z;
            real dRGBdsh4 = SH_C2[0] * xy;
            real dRGBdsh5 = SH_C2[1] * yz;
            real dRGBdsh6 = SH_C2[2] * (2.f * zz - xx - yy);
            real dRGBdsh7 = SH_C2[3] * xz;
            real dRGBdsh8 = SH_C2[4] * (xx - yy);
            PUT(4, v3_muls(dRGBdsh4, dL_dRGB));
            PUT(5, v3_muls(dRGBdsh5, dL_dRGB));
            PUT(6, v3_muls(dRGBdsh6, dL_dRGB));
            PUT(7, v3_muls(dRGBdsh7, dL_dRGB));
            PUT(8, v3_muls(dRGBdsh8, dL_dRGB));
            v3 tx = v3_add(v3_add(v3_add(v3_muls(SH_C2[0] * y, SH(4)), v3_muls(SH_C2[2] * 2.f * -x, SH(6))),
                                  v3_muls(SH_C2[3] * z, SH(7))),
                           v3_muls(SH_C2[4] * 2.f * x, SH(8)));
            v3 ty = v3_add(v3_add(v3_add(v3_muls(SH_C2[0] * x, SH(4)), v3_muls(SH_C2[1] * z, SH(5))),
                                  v3_muls(SH_C2[2] * 2.f * -y, SH(6))),
                           v3_muls(SH_C2[4] * 2.f * -y, SH(8)));
            v3 tz = v3_add(v3_add(v3_muls(SH_C2[1] * y, SH(5)), v3_muls(SH_C2[2] * 2.f * 2.f * z, SH(6))),
                           v3_muls(SH_C2[3] * x, SH(7)));
            dRGBdx = v3_add(dRGBdx, tx);
            dRGBdy = v3_add(dRGBdy, ty);
            dRGBdz = v3_add(dRGBdz, tz);
            if (deg > 2) {
                real dRGBdsh9 = SH_C3[0] * y * (3.f * xx - yy);
                real dRGBdsh10 = SH_C3[1] * xy * z;
                real dRGBdsh11 = SH_C3[2] * y * (4.f * zz - xx - yy);
                real dRGBdsh12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                real dRGBdsh13 = SH_C3[4] * x * (4.f * zz - xx - yy);
                real dRGBdsh14 = SH_C3[5] * z * (xx - yy);
                real dRGBdsh15 = SH_C3[6] * x * (xx - 3.f * yy);
                PUT(9, v3_muls(dRGBdsh9, dL_dRGB));
                PUT(10, v3_muls(dRGBdsh10, dL_dRGB));
                PUT(11, v3_muls(dRGBdsh11, dL_dRGB));
                PUT(12, v3_muls(dRGBdsh12, dL_dRGB));
                PUT(13, v3_muls(dRGBdsh13, dL_dRGB));
                PUT(14, v3_muls(dRGBdsh14, dL_dRGB));
                PUT(15, v3_muls(dRGBdsh15, dL_dRGB));
                /* backward.cu:99-122: (scalar*vec3) then chained vec3*scalar products */
                v3 ax = v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[0], SH(9)), 3.f), 2.f), xy);
                ax = v3_add(ax, v3_mul_s(v3_muls(SH_C3[1], SH(10)), yz));
                ax = v3_add(ax, v3_mul_s(v3_mul_s(v3_muls(SH_C3[2], SH(11)), -2.f), xy));
                ax = v3_add(ax, v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[3], SH(12)), -3.f), 2.f), xz));
                ax = v3_add(ax, v3_mul_s(v3_muls(SH_C3[4], SH(13)), (-3.f * xx + 4.f * zz - yy)));
                ax = v3_add(ax, v3_mul_s(v3_mul_s(v3_muls(SH_C3[5], SH(14)), 2.f), xz));
                ax = v3_add(ax, v3_mul_s(v3_mul_s(v3_muls(SH_C3[6], SH(15)), 3.f), (xx - yy)));
                v3 ay = v3_mul_s(v3_mul_s(v3_muls(SH_C3[0], SH(9)), 3.f), (xx - yy));
                ay = v3_add(ay, v3_mul_s(v3_muls(SH_C3[1], SH(10)), xz));
                ay = v3_add(ay, v3_mul_s(v3_muls(SH_C3[2], SH(11)), (-3.f * yy + 4.f * zz - xx)));
                ay = v3_add(ay, v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[3], SH(12)), -3.f), 2.f), yz));
                ay = v3_add(ay, v3_mul_s(v3_mul_s(v3_muls(SH_C3[4], SH(13)), -2.f), xy));
                ay = v3_add(ay, v3_mul_s(v3_mul_s(v3_muls(SH_C3[5], SH(14)), -2.f), yz));
                ay = v3_add(ay, v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[6], SH(15)), -3.f), 2.f), xy));
                v3 az = v3_mul_s(v3_muls(SH_C3[1], SH(10)), xy);
                az = v3_add(az, v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[2], SH(11)), 4.f), 2.f), yz));
                az = v3_add(az, v3_mul_s(v3_mul_s(v3_muls(SH_C3[3], SH(12)), 3.f), (2.f * zz - xx - yy)));
                az = v3_add(az, v3_mul_s(v3_mul_s(v3_mul_s(v3_muls(SH_C3[4], SH(13)), 4.f), 2.f), xz));
                az = v3_add(az, v3_mul_s(v3_muls(SH_C3[5], SH(14)), (xx - yy)));
                dRGBdx = v3_add(dRGBdx, ax);
                dRGBdy = v3_add(dRGBdy, ay);
                dRGBdz = v3_add(dRGBdz, az);
            }
        }
    }
#undef PUT
#undef SH
    v3 dL_ddir = v3_mk(v3_dot(dRGBdx, dL_dRGB), v3_dot(dRGBdy, dL_dRGB), v3_dot(dRGBdz, dL_dRGB));
    v3 dm = dnormvdv(dir_orig, dL_ddir);
    dL_dmeans[3 * idx + 0] += dm.x;
    dL_dmeans[3 * idx + 1] += dm.y;
    dL_dmeans[3 * idx + 2] += dm.z;
}

/* backward.cu:144-274 computeCov2DCUDA (per Gaussian) */
static void cov2d_backward(int idx, const float* means, const real* cov3D, real h_x, real h_y,
                           real tan_fovx, real tan_fovy, const real* view,
                           const real* dL_dconics, real* dL_dmeans, real* dL_dcov) {
    const real* c3 = cov3D + 6 * (size_t)idx;
    v3 mean = v3_mk(means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]);
    real dcx = dL_dconics[4 * idx], dcy = dL_dconics[4 * idx + 1], dcz = dL_dconics[4 * idx + 3];
    v3 t = transformPoint4x3(mean, view);
    const real limx = 1.3f * tan_fovx;
    const real limy = 1.3f * tan_fovy;
    const real txtz = t.x / t.z;
    const real tytz = t.y / t.z;
    t.x = fminf_cuda(limx, fmaxf_cuda(-limx, txtz)) * t.z;
    t.y = fminf_cuda(limy, fmaxf_cuda(-limy, tytz)) * t.z;
    const real x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const real y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    m3 J = m3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z,
                   -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
    m3 Wm = m3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6],
                    view[10]);
    m3 Vrk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    m3 T = m3_mul(Wm, J);
    m3 cov2D = m3_mul(m3_mul(m3_T(T), m3_T(Vrk)), T);
    real a = cov2D.m[0][0] += 0.3f;
    real b = cov2D.m[0][1];
    real c = cov2D.m[1][1] += 0.3f;
    real denom = a * c - b * b;
    real dL_da = 0, dL_db = 0, dL_dc = 0;
    real denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    real* dc = dL_dcov + 6 * (size_t)idx;
#define Tm(cc, rr) T.m[cc][rr]
#define V(cc, rr) Vrk.m[cc][rr]
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
        dL_dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
        dL_db = denom2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
        dc[0] = (Tm(0, 0) * Tm(0, 0) * dL_da + Tm(0, 0) * Tm(1, 0) * dL_db + Tm(1, 0) * Tm(1, 0) * dL_dc);
        dc[3] = (Tm(0, 1) * Tm(0, 1) * dL_da + Tm(0, 1) * Tm(1, 1) * dL_db + Tm(1, 1) * Tm(1, 1) * dL_dc);
        dc[5] = (Tm(0, 2) * Tm(0, 2) * dL_da + Tm(0, 2) * Tm(1, 2) * dL_db + Tm(1, 2) * Tm(1, 2) * dL_dc);
        dc[1] = 2 * Tm(0, 0) * Tm(0, 1) * dL_da + (Tm(0, 0) * Tm(1, 1) + Tm(0, 1) * Tm(1, 0)) * dL_db +
                2 * Tm(1, 0) * Tm(1, 1) * dL_dc;
        dc[2] = 2 * Tm(0, 0) * Tm(0, 2) * dL_da + (Tm(0, 0) * Tm(1, 2) + Tm(0, 2) * Tm(1, 0)) * dL_db +
                2 * Tm(1, 0) * Tm(1, 2) * dL_dc;
        dc[4] = 2 * Tm(0, 2) * Tm(0, 1) * dL_da + (Tm(0, 1) * Tm(1, 2) + Tm(0, 2) * Tm(1, 1)) * dL_db +
                2 * Tm(1, 1) * Tm(1, 2) * dL_dc;
    } else {
        for (int i = 0; i < 6; i++) dc[i] = 0;
    }
    real dL_dT00 = 2 * (Tm(0, 0) * V(0, 0) + Tm(0, 1) * V(0, 1) + Tm(0, 2) * V(0, 2)) * dL_da +
                    (Tm(1, 0) * V(0, 0) + Tm(1, 1) * V(0, 1) + Tm(1, 2) * V(0, 2)) * dL_db;
    real dL_dT01 = 2 * (Tm(0, 0) * V(1, 0) + Tm(0, 1) * V(1, 1) + Tm(0, 2) * V(1, 2)) * dL_da +
                    (Tm(1, 0) * V(1, 0) + Tm(1, 1) * V(1, 1) + Tm(1, 2) * V(1, 2)) * dL_db;
    real dL_dT02 = 2 * (Tm(0, 0) * V(2, 0) + Tm(0, 1) * V(2, 1) + Tm(0, 2) * V(2, 2)) * dL_da +
                    (Tm(1, 0) * V(2, 0) + Tm(1, 1) * V(2, 1) + Tm(1, 2) * V(2, 2)) * dL_db;
    real dL_dT10 = 2 * (Tm(1, 0) * V(0, 0) + Tm(1, 1) * V(0, 1) + Tm(1, 2) * V(0, 2)) * dL_dc +
                    (Tm(0, 0) * V(0, 0) + Tm(0, 1) * V(0, 1) + Tm(0, 2) * V(0, 2)) * dL_db;
    real dL_dT11 = 2 * (Tm(1, 0) * V(1, 0) + Tm(1, 1) * V(1, 1) + Tm(1, 2) * V(1, 2)) * dL_dc +
                    (Tm(0, 0) * V(1, 0) + Tm(0, 1) * V(1, 1) + Tm(0, 2) * V(1, 2)) * dL_db;
    real dL_dT12 = 2 * (Tm(1, 0) * V(2, 0) + Tm(1, 1) * V(2, 1) + Tm(1, 2) * V(2, 2)) * dL_dc +
                    (Tm(0, 0) * V(2, 0) + Tm(0, 1) * V(2, 1) + Tm(0, 2) * V(2, 2)) * dL_db;
#undef Tm
#undef V
    real dL_dJ00 = Wm.m[0][0] * dL_dT00 + Wm.m[0][1] * dL_dT01 + Wm.m[0][2] * dL_dT02;
    real dL_dJ02 = Wm.m[2][0] * dL_dT00 + Wm.m[2][1] * dL_dT01 + Wm.m[2][2] * dL_dT02;
    real dL_dJ11 = Wm.m[1][0] * dL_dT10 + Wm.m[1][1] * dL_dT11 + Wm.m[1][2] * dL_dT12;
    real dL_dJ12 = Wm.m[2][0] * dL_dT10 + Wm.m[2][1] * dL_dT11 + Wm.m[2][2] * dL_dT12;
    real tz = 1.f / t.z;
    real tz2 = tz * tz;
    real tz3 = tz2 * tz;
    real dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    real dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    real dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                   (2 * h_y * t.y) * tz3 * dL_dJ12;
    v3 dm = transformVec4x3Transpose(v3_mk(dL_dtx, dL_dty, dL_dtz), view);
    dL_dmeans[3 * idx + 0] = dm.x; /* assigned, backward.cu:273 */
    dL_dmeans[3 * idx + 1] = dm.y;
    dL_dmeans[3 * idx + 2] = dm.z;
}

/* backward.cu:278-341 computeCov3D (bwd) */
static void cov3d_backward(int idx, const float* scale, real mod, const float* rot,
                           const real* dL_dcov3Ds, real* dL_dscales, real* dL_drots) {
    real r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    m3 R = m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    m3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    v3 s = v3_muls(mod, v3_mk(scale[0], scale[1], scale[2]));
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    m3 M = m3_mul(S, R);
    const real* g = dL_dcov3Ds + 6 * (size_t)idx;
    m3 dL_dSigma = m3_cols(g[0], 0.5f * g[1], 0.5f * g[2], 0.5f * g[1], g[3], 0.5f * g[4],
                           0.5f * g[2], 0.5f * g[4], g[5]);
    m3 dL_dM = m3_mul(m3_scale(2.0f, M), dL_dSigma);
    m3 Rt = m3_T(R);
    m3 dL_dMt = m3_T(dL_dM);
    real* ds = dL_dscales + 3 * (size_t)idx;
    for (int k = 0; k < 3; k++) {
        v3 a = v3_mk(Rt.m[k][0], Rt.m[k][1], Rt.m[k][2]);
        v3 b = v3_mk(dL_dMt.m[k][0], dL_dMt.m[k][1], dL_dMt.m[k][2]);
        ds[k] = v3_dot(a, b);
    }
    for (int w = 0; w < 3; w++) {
        dL_dMt.m[0][w] *= s.x;
        dL_dMt.m[1][w] *= s.y;
        dL_dMt.m[2][w] *= s.z;
    }
#define D(cc, rr) dL_dMt.m[cc][rr]
    real* dq = dL_drots + 4 * (size_t)idx;
    dq[0] = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    dq[1] = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) -
            4 * x * (D(2, 2) + D(1, 1));
    dq[2] = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) -
            4 * y * (D(2, 2) + D(0, 0));
    dq[3] = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) -
            4 * z * (D(1, 1) + D(0, 0));
#undef D
}

/* ---- renderCUDA (bwd), backward.cu:399-557, per pixel, extended to NCH channels ---- */
/* Gradient accumulators of one chunk of pixel rows: the caller's arrays (one chunk) or the     */
/* chunk's private block [colors 3P | depth P | feat 3P | means2D 3P | conic 4P | opacity P].     */
enum { ACC_COL = 0, ACC_DEP = 3, ACC_FEAT = 4, ACC_M2D = 7, ACC_CON = 10, ACC_OP = 14, ACC_ROW = 15 };
typedef struct {
    oracle_state* st;
    const float *dc, *dd, *da, *df;
    real* priv;                                        /* private blocks, or NULL */
    real *dcolors, *ddepth, *dfeat, *dmeans2D, *dconic, *dopacity; /* shared targets */
    int mass; /* oracle_blend_rows(mass = 1): sums of the terms' absolute values instead */
} blend_bwd_ctx;
static void blend_bwd_rows(void* ctx, long lo, long hi, int chunk) {
    const blend_bwd_ctx* c = (const blend_bwd_ctx*)ctx;
    oracle_state* st = c->st;
    const size_t P = (size_t)st->P;
    real *dL_dcolors, *ddepth, *dfeat, *dL_dmeans2D, *dconic, *dL_dopacity;
    if (c->priv) {
        real* b = c->priv + (size_t)chunk * ACC_ROW * P;
        dL_dcolors = b + ACC_COL * P; ddepth = b + ACC_DEP * P; dfeat = b + ACC_FEAT * P;
        dL_dmeans2D = b + ACC_M2D * P; dconic = b + ACC_CON * P; dL_dopacity = b + ACC_OP * P;
    } else {
        dL_dcolors = c->dcolors; ddepth = c->ddepth; dfeat = c->dfeat;
        dL_dmeans2D = c->dmeans2D; dconic = c->dconic; dL_dopacity = c->dopacity;
    }
    const int W = st->W, H = st->H;
    const size_t HW = (size_t)W * H;
    const unsigned gx = st->gx;
    const real* color_ptr = st->rgb; /* colors_precomp converted into rgb by oracle_forward */
    const int nch = st->include_feature ? NCH : 5;
    const real ddelx_dx = (real)(0.5 * W);
    const real ddely_dy = (real)(0.5 * H);
    for (long py = lo; py < hi; py++)
        for (int px = 0; px < W; px++) {
            const unsigned tile = (unsigned)(py / BLOCK_Y) * gx + (unsigned)(px / BLOCK_X);
            const unsigned rs = st->ranges[2 * tile], re = st->ranges[2 * tile + 1];
            const size_t pix = (size_t)py * W + px;
            const real pfx = (real)px, pfy = (real)py;
            const real T_final = st->final_T[pix];
            real T = T_final;
            unsigned contributor = re - rs;
            const unsigned last_contributor = st->n_contrib[pix];
            real accum_rec[NCH] = {0}, last_color[NCH] = {0}, dL_dpixel[NCH] = {0};
            for (int i = 0; i < 3; i++) dL_dpixel[i] = c->dc[i * HW + pix];
            dL_dpixel[3] = c->dd ? c->dd[pix] : 0.0f;
            dL_dpixel[4] = c->da ? c->da[pix] : 0.0f;
            for (int i = 0; i < 3; i++) dL_dpixel[5 + i] = c->df ? c->df[i * HW + pix] : 0.0f;
            real last_alpha = 0;
            const unsigned* lock_w = st->lock_nc ? st->lock_words + st->lock_offs[pix] : NULL;
            /* mass mode: the float32 chain length of T at each splat -- the forward's product over
             * the pixel's contributors, then one division per splat replayed -- weights the terms
             * (T, and with it every term, carries ~ one rounding per link of that chain) */
            real chain = 0;
            if (c->mass) {
                unsigned pos = 0;
                for (unsigned k = rs; k < re && pos < last_contributor; k++, pos++) {
                    if (lock_w) {
                        chain += (real)((lock_w[pos >> 5] >> (pos & 31)) & 1u);
                        continue;
                    }
                    const unsigned g = st->point_list[k];
                    const real dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                    const real* co = st->conic_opacity + 4 * (size_t)g;
                    const real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    if (fminf_cuda(0.99f, co[3] * blend_exp(power)) < 1.0f / 255.0f) continue;
                    chain += 1;
                }
            }
            for (unsigned k = re; k-- > rs;) {
                contributor--;
                if (contributor >= last_contributor) continue;
                const int lock_take =
                    lock_w ? (int)((lock_w[contributor >> 5] >> (contributor & 31)) & 1u) : -1;
                if (lock_take == 0) continue;
                const unsigned g = st->point_list[k];
                const real dx = st->means2D[2 * g] - pfx, dy = st->means2D[2 * g + 1] - pfy;
                const real* co = st->conic_opacity + 4 * (size_t)g;
                const real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (lock_take < 0 && power > 0.0f) continue;
                const real G = blend_exp(power);
                const real alpha = fminf_cuda(0.99f, co[3] * G);
                if (lock_take < 0 && alpha < 1.0f / 255.0f) continue;
                T = T / (1.f - alpha);
                const real dchannel_dcolor = alpha * T;
                real dL_dalpha = 0.0f;
                real amass = 0.0f; /* mass mode: the absolute values of dL_dalpha's terms */
                real v[NCH];
                v[0] = color_ptr[3 * g]; v[1] = color_ptr[3 * g + 1]; v[2] = color_ptr[3 * g + 2];
                v[3] = st->depths[g]; v[4] = 1.0f;
                v[5] = st->feat[3 * g]; v[6] = st->feat[3 * g + 1]; v[7] = st->feat[3 * g + 2];
                for (int ch = 0; ch < nch; ch++) {
                    const real cv = v[ch];
                    accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                    last_color[ch] = cv;
                    const real dL_dchannel = dL_dpixel[ch];
                    dL_dalpha += (cv - accum_rec[ch]) * dL_dchannel;
                    if (c->mass) amass += (fabs(cv) + fabs(accum_rec[ch])) * fabs(dL_dchannel);
                    const real gv = c->mass ? fabs(dchannel_dcolor * dL_dchannel) * (2 + chain)
                                            : dchannel_dcolor * dL_dchannel;
                    if (ch < 3) dL_dcolors[3 * (size_t)g + ch] += gv;
                    else if (ch == 3) ddepth[g] += gv;
                    else if (ch >= 5) dfeat[3 * (size_t)g + ch - 5] += gv;
                }
                dL_dalpha *= T;
                last_alpha = alpha;
                real bg_dot_dpixel = 0;
                for (int i = 0; i < 3; i++) bg_dot_dpixel += st->bg[i] * dL_dpixel[i];
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                if (c->mass) {
                    chain += 1;
                    real bgm = 0;
                    for (int i = 0; i < 3; i++) bgm += fabs(st->bg[i] * dL_dpixel[i]);
                    const real am = (amass * T + T_final / (1.f - alpha) * bgm) * (1 + chain);
                    const real gm = co[3] * am;
                    const real ax = fabs(G * dx), ay = fabs(G * dy);
                    dL_dmeans2D[3 * (size_t)g + 0] += gm * (ax * fabs(co[0]) + ay * fabs(co[1])) * ddelx_dx;
                    dL_dmeans2D[3 * (size_t)g + 1] += gm * (ay * fabs(co[2]) + ax * fabs(co[1])) * ddely_dy;
                    dconic[4 * (size_t)g + 0] += 0.5f * ax * fabs(dx) * gm;
                    dconic[4 * (size_t)g + 1] += 0.5f * ax * fabs(dy) * gm;
                    dconic[4 * (size_t)g + 3] += 0.5f * ay * fabs(dy) * gm;
                    dL_dopacity[g] += G * am;
                    continue;
                }
                const real dL_dG = co[3] * dL_dalpha;
                const real gdx = G * dx;
                const real gdy = G * dy;
                const real dG_ddelx = -gdx * co[0] - gdy * co[1];
                const real dG_ddely = -gdy * co[2] - gdx * co[1];
                dL_dmeans2D[3 * (size_t)g + 0] += dL_dG * dG_ddelx * ddelx_dx;
                dL_dmeans2D[3 * (size_t)g + 1] += dL_dG * dG_ddely * ddely_dy;
                dconic[4 * (size_t)g + 0] += -0.5f * gdx * dx * dL_dG;
                dconic[4 * (size_t)g + 1] += -0.5f * gdx * dy * dL_dG;
                dconic[4 * (size_t)g + 3] += -0.5f * gdy * dy * dL_dG;
                dL_dopacity[g] += G * dL_dalpha;
            }
        }
}
/* target[i] = sum over chunks (in chunk order) of private slot `slot0`+.. element i */
typedef struct { const real* priv; int nchunks; size_t P; size_t slot; real* dst; } reduce_ctx;
static void reduce_range(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    const reduce_ctx* r = (const reduce_ctx*)ctx;
    for (long i = lo; i < hi; i++) {
        real s = 0.0f;
        for (int c = 0; c < r->nchunks; c++) s += r->priv[(size_t)c * ACC_ROW * r->P + r->slot * r->P + i];
        r->dst[i] = s;
    }
}

/* ---- BACKWARD::preprocess, backward.cu:559-622, per Gaussian ---- */
typedef struct {
    oracle_state* st;
    const real* cov3D_ptr;
    real *dL_dmeans2D, *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales,
        *dL_drotations, *dL_dsh_language, *dL_dlanguage_feature, *dconic, *ddepth, *dfeat;
} pre_bwd_ctx;
static void cov2d_bwd_range(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    const pre_bwd_ctx* c = (const pre_bwd_ctx*)ctx;
    oracle_state* st = c->st;
    for (long i = lo; i < hi; i++) {
        const int idx = (int)i;
        if (!(st->radii[idx] > 0)) continue;
        cov2d_backward(idx, st->means3D, c->cov3D_ptr, st->focal_x, st->focal_y, st->tan_fovx,
                       st->tan_fovy, st->view, c->dconic, c->dL_dmeans3D, c->dL_dcov3D);
    }
}
static void pre_bwd_range(void* ctx, long lo, long hi, int chunk) {
    (void)chunk;
    const pre_bwd_ctx* c = (const pre_bwd_ctx*)ctx;
    oracle_state* st = c->st;
    const real* proj = st->proj;
    for (long i = lo; i < hi; i++) {
        const int idx = (int)i;
        if (!(st->radii[idx] > 0)) continue;
        /* backward.cu:370-387 */
        v3 m = v3_mk(st->means3D[3 * idx], st->means3D[3 * idx + 1], st->means3D[3 * idx + 2]);
        real m_hom[4];
        transformPoint4x4(m, proj, m_hom);
        real m_w = 1.0f / (m_hom[3] + 0.0000001f);
        real mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        real mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        const real gx2 = c->dL_dmeans2D[3 * idx], gy2 = c->dL_dmeans2D[3 * idx + 1];
        v3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * gx2 + (proj[1] * m_w - proj[3] * mul2) * gy2;
        dm.y = (proj[4] * m_w - proj[7] * mul1) * gx2 + (proj[5] * m_w - proj[7] * mul2) * gy2;
        dm.z = (proj[8] * m_w - proj[11] * mul1) * gx2 + (proj[9] * m_w - proj[11] * mul2) * gy2;
        c->dL_dmeans3D[3 * idx + 0] += dm.x;
        c->dL_dmeans3D[3 * idx + 1] += dm.y;
        c->dL_dmeans3D[3 * idx + 2] += dm.z;
        if (st->sh && c->dL_dsh)
            sh_backward(idx, st->D, st->M, st->means3D, st->campos, st->sh, st->clamped,
                        c->dL_dcolors, c->dL_dmeans3D, c->dL_dsh);
        if (st->scales && c->dL_dscales && c->dL_drotations)
            cov3d_backward(idx, st->scales + 3 * (size_t)idx, st->scale_modifier,
                           st->rotations + 4 * (size_t)idx, c->dL_dcov3D, c->dL_dscales,
                           c->dL_drotations);
        /* depth channel -> view-space z = view[2]x + view[6]y + view[10]z + view[14] */
        const real dz = c->ddepth[idx];
        c->dL_dmeans3D[3 * idx + 0] += dz * st->view[2];
        c->dL_dmeans3D[3 * idx + 1] += dz * st->view[6];
        c->dL_dmeans3D[3 * idx + 2] += dz * st->view[10];
        /* confidence is an opacity multiplier */
        if (st->confidence) c->dL_dopacity[idx] = c->dL_dopacity[idx] * st->confidence[idx];
        if (st->include_feature) {
            const real* gf = c->dfeat + 3 * (size_t)idx;
            if (st->lang_precomp) {
                if (c->dL_dlanguage_feature)
                    for (int k = 0; k < 3; k++) c->dL_dlanguage_feature[3 * idx + k] = gf[k];
            } else if (st->sh_language && c->dL_dsh_language) {
                /* f = u / (|u| + 1e-9), u = SH_C0 * l */
                const float* l = st->sh_language + 3 * (size_t)idx;
                real u0 = SH_C0 * l[0], u1 = SH_C0 * l[1], u2v = SH_C0 * l[2];
                real n = sqrt(u0 * u0 + u1 * u1 + u2v * u2v);
                real den = n + 1e-9f;
                real ug = u0 * gf[0] + u1 * gf[1] + u2v * gf[2];
                real k2 = n > 0.0f ? ug / (den * den * n) : 0.0f;
                c->dL_dsh_language[3 * idx + 0] = SH_C0 * (gf[0] / den - u0 * k2);
                c->dL_dsh_language[3 * idx + 1] = SH_C0 * (gf[1] / den - u1 * k2);
                c->dL_dsh_language[3 * idx + 2] = SH_C0 * (gf[2] / den - u2v * k2);
            }
        }
    }
}

/* The blend backward's per-Gaussian sums (renderCUDA bwd) into `rows`, the ACC block
 * [colors 3P | depth P | feat 3P | means2D 3P | conic 4P | opacity P] (zeroed here); mass: the sums
 * of the terms' absolute values (oracle_blend_rows). */
static void blend_backward(oracle_state* st, const float* dL_dout_color, const float* dL_dout_depth,
                           const float* dL_dout_alpha, const float* dL_dout_feature, int mass,
                           real* rows) {
    const size_t P = (size_t)st->P;
    const int H = st->H;
    memset(rows, 0, sizeof(real) * ACC_ROW * P);
    blend_bwd_ctx bc = {st, dL_dout_color, dL_dout_depth, dL_dout_alpha, dL_dout_feature, NULL,
                        rows + ACC_COL * P, rows + ACC_DEP * P, rows + ACC_FEAT * P,
                        rows + ACC_M2D * P, rows + ACC_CON * P, rows + ACC_OP * P, mass};
    const int nchunks = par_chunks(H);
    if (nchunks > 1) bc.priv = (real*)calloc((size_t)nchunks * ACC_ROW * P, sizeof(real));
    if (bc.priv) par_for(H, blend_bwd_rows, &bc);
    else blend_bwd_rows(&bc, 0, H, 0); /* one chunk straight into the rows */
    if (bc.priv) {
        for (size_t s = 0; s < ACC_ROW; s++) {
            reduce_ctx rc = {bc.priv, nchunks, P, s, rows + s * P};
            par_for((long)P, reduce_range, &rc);
        }
        free(bc.priv);
    }
}

/* BACKWARD::preprocess (backward.cu:559-622) from the blend's rows (ACC block, read-only). */
static void backward_from_rows(oracle_state* st, const real* rows, real* dL_dmeans2D,
                               real* dL_dcolors, real* dL_dopacity, real* dL_dmeans3D,
                               real* dL_dcov3D, real* dL_dsh, real* dL_dscales,
                               real* dL_drotations, real* dL_dsh_language,
                               real* dL_dlanguage_feature) {
    const size_t P = (size_t)st->P, M = (size_t)st->M;
    /* rasterize_points.cu:151-159 zero-initialised grads */
    memset(dL_dmeans3D, 0, sizeof(real) * 3 * P);
    memset(dL_dcov3D, 0, sizeof(real) * 6 * P);
    if (dL_dsh) memset(dL_dsh, 0, sizeof(real) * 3 * P * M);
    if (dL_dscales) memset(dL_dscales, 0, sizeof(real) * 3 * P);
    if (dL_drotations) memset(dL_drotations, 0, sizeof(real) * 4 * P);
    if (dL_dsh_language) memset(dL_dsh_language, 0, sizeof(real) * 3 * P);
    if (dL_dlanguage_feature) memset(dL_dlanguage_feature, 0, sizeof(real) * 3 * P);
    memcpy(dL_dmeans2D, rows + ACC_M2D * P, sizeof(real) * 3 * P);
    memcpy(dL_dcolors, rows + ACC_COL * P, sizeof(real) * 3 * P);
    memcpy(dL_dopacity, rows + ACC_OP * P, sizeof(real) * P);
    real* priv = (real*)xcalloc(8 * P, sizeof(real)); /* conic 4P | depth P | feat 3P */
    memcpy(priv, rows + ACC_CON * P, sizeof(real) * 4 * P);
    memcpy(priv + 4 * P, rows + ACC_DEP * P, sizeof(real) * P);
    memcpy(priv + 5 * P, rows + ACC_FEAT * P, sizeof(real) * 3 * P);
    pre_bwd_ctx pc = {st, st->cov3D, dL_dmeans2D,
                      dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                      dL_drotations, dL_dsh_language, dL_dlanguage_feature, priv, priv + 4 * P,
                      priv + 5 * P};
    par_for((long)P, cov2d_bwd_range, &pc);
    par_for((long)P, pre_bwd_range, &pc);
    /* invisible Gaussians: the grads of the colour channels etc. are already zero. */
    free(priv);
}

int oracle_backward(oracle_state* st, const float* dL_dout_color, const float* dL_dout_depth,
                    const float* dL_dout_alpha, const float* dL_dout_feature, real* dL_dmeans2D,
                    real* dL_dcolors, real* dL_dopacity, real* dL_dmeans3D, real* dL_dcov3D,
                    real* dL_dsh, real* dL_dscales, real* dL_drotations,
                    real* dL_dsh_language, real* dL_dlanguage_feature) {
    if (!st) return 1;
    real* rows = (real*)xcalloc((size_t)ACC_ROW * st->P, sizeof(real));
    /* ---- renderCUDA (bwd), backward.cu:399-557 ---- */
    blend_backward(st, dL_dout_color, dL_dout_depth, dL_dout_alpha, dL_dout_feature, 0, rows);
    /* ---- BACKWARD::preprocess, backward.cu:559-622 ---- */
    backward_from_rows(st, rows, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                       dL_dsh, dL_dscales, dL_drotations, dL_dsh_language, dL_dlanguage_feature);
    free(rows);
    return 0;
}

int oracle_blend_rows(oracle_state* st, const float* dL_dout_color, const float* dL_dout_depth,
                      const float* dL_dout_alpha, const float* dL_dout_feature, int mass,
                      real* rows) {
    if (!st || !rows) return 1;
    blend_backward(st, dL_dout_color, dL_dout_depth, dL_dout_alpha, dL_dout_feature, mass, rows);
    return 0;
}

int oracle_backward_rows(oracle_state* st, const real* rows, real* dL_dmeans2D, real* dL_dcolors,
                         real* dL_dopacity, real* dL_dmeans3D, real* dL_dcov3D, real* dL_dsh,
                         real* dL_dscales, real* dL_drotations, real* dL_dsh_language,
                         real* dL_dlanguage_feature) {
    if (!st || !rows) return 1;
    backward_from_rows(st, rows, dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
                       dL_dsh, dL_dscales, dL_drotations, dL_dsh_language, dL_dlanguage_feature);
    return 0;
}

void oracle_free(oracle_state* st) {
    if (!st) return;
    free(st->depths); free(st->depth_key); free(st->clamped); free(st->radii); free(st->means2D); free(st->cov3D);
    free(st->conic_opacity); free(st->rgb); free(st->feat); free(st->tiles_touched);
    free(st->point_list); free(st->ranges); free(st->final_T); free(st->n_contrib); free(st->margin);
    free(st->lock_nc); free(st->lock_offs); free(st->lock_words); free(st->clamp_lock);
    free(st);
}

/* The reference's instance list (point_list, ranges) with the instances the exact tile cull
 * drops removed; order otherwise unchanged.  Returns the number of instances kept. */
int oracle_cut_lists(const oracle_state* st, unsigned* point_list_out, unsigned* ranges_out) {
    const unsigned ntiles = st->gx * st->gy;
    unsigned n = 0;
    for (unsigned t = 0; t < ntiles; t++) {
        const unsigned rs = st->ranges[2 * t], re = st->ranges[2 * t + 1];
        const unsigned tx = t % st->gx, ty = t / st->gx;
        const unsigned start = n;
        for (unsigned k = rs; k < re; k++) {
            const unsigned g = st->point_list[k];
            /* the cut is float-defined (gsr_device.h): float values of the record */
            const real* cr = st->conic_opacity + 4 * (size_t)g;
            const float co[4] = {(float)cr[0], (float)cr[1], (float)cr[2], (float)cr[3]};
            const float mx = (float)st->means2D[2 * (size_t)g], my = (float)st->means2D[2 * (size_t)g + 1];
            u2 rmin, rmax;
            getRect(mx, my, st->radii[g], &rmin, &rmax, st->gx, st->gy);
            const band_cut c = make_band_cut(mx, my, co[0], co[1], co[2], cut_q(co[0], co[1], co[2], co[3]));
            unsigned a, b;
            band_row_range(&c, ty, rmin.x, rmax.x, &a, &b);
            if (tx >= a && tx < b) point_list_out[n++] = g;
        }
        ranges_out[2 * t] = n > start ? start : 0;
        ranges_out[2 * t + 1] = n > start ? n : 0;
    }
    return (int)n;
}

int oracle_get_point_list(const oracle_state* st, unsigned* out) { memcpy(out, st->point_list, sizeof(unsigned) * (size_t)st->R); return st->R; }
int oracle_get_ranges(const oracle_state* st, unsigned* out) { memcpy(out, st->ranges, sizeof(unsigned) * 2 * (size_t)st->gx * st->gy); return 0; }
static void to_float(float* out, const real* in, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = (float)in[i];
}
int oracle_get_final_T(const oracle_state* st, float* out) { to_float(out, st->final_T, (size_t)st->W * st->H); return 0; }
int oracle_get_n_contrib(const oracle_state* st, unsigned* out) { memcpy(out, st->n_contrib, sizeof(unsigned) * (size_t)st->W * st->H); return 0; }
int oracle_get_margin(const oracle_state* st, float* out) { to_float(out, st->margin, (size_t)st->W * st->H); return 0; }
int oracle_get_means2D(const oracle_state* st, float* out) { to_float(out, st->means2D, 2 * (size_t)st->P); return 0; }
int oracle_get_conic_opacity(const oracle_state* st, float* out) { to_float(out, st->conic_opacity, 4 * (size_t)st->P); return 0; }
int oracle_get_depths(const oracle_state* st, float* out) { to_float(out, st->depths, (size_t)st->P); return 0; }
int oracle_get_rgb(const oracle_state* st, float* out) { to_float(out, st->rgb, 3 * (size_t)st->P); return 0; }
int oracle_get_tiles_touched(const oracle_state* st, unsigned* out) { memcpy(out, st->tiles_touched, sizeof(unsigned) * (size_t)st->P); return 0; }
int oracle_get_clamped(const oracle_state* st, unsigned char* out) { memcpy(out, st->clamped, 3 * (size_t)st->P); return 0; }
/* The preprocess outputs at the build's own precision, [P][13] doubles in the GPU splat record's
 * order (gsr_preprocess.hip): x_px, y_px, conic a, b, c, opacity, depth, r, g, b, f0, f1, f2
 * (tests/test_pre_f64_parity.py; the float getters above round the float64 build to float). */
int oracle_get_preprocess_f64(const oracle_state* st, double* out) {
    for (long i = 0; i < st->P; i++) {
        double* o = out + 13 * i;
        o[0] = st->means2D[2 * i]; o[1] = st->means2D[2 * i + 1];
        for (int k = 0; k < 4; k++) o[2 + k] = st->conic_opacity[4 * i + k];
        o[6] = st->depths[i];
        for (int k = 0; k < 3; k++) o[7 + k] = st->rgb[3 * i + k];
        for (int k = 0; k < 3; k++) o[10 + k] = st->feat[3 * i + k];
    }
    return 0;
}
int oracle_get_cov3D(const oracle_state* st, float* out) { to_float(out, st->cov3D, 6 * (size_t)st->P); return 0; }

// gsr_loss.hip -- the training losses either side of the rasterizer.
//
// Reference (utils/loss_utils.py, train.py:99-130):
//   Ll1  = l1_loss(image, gt)                         mean |x - y|                     (:106-107)
//   loss = (1 - lambda) Ll1 + lambda (1 - ssim(image, gt))                              (train.py:100)
//   ssim: 11x11 Gaussian window (sigma 1.5), zero padding, five depthwise F.conv2d        (:119-162)
//         (mu_x, mu_y, E[x^2], E[y^2], E[xy]), C1 = 0.01^2, C2 = 0.03^2, mean of the map
//   depth: 1 - pearson_corrcoef(...) (torchmetrics), min over two variants      (train.py:126-129)
//
// SSIM here: one tiled kernel per pass instead of five convolutions + ~20 element-wise kernels +
// autograd through all of them.  A workgroup owns a 32x32 output tile of one channel: both
// images' (32+10)x(32+10) halo tiles go to LDS, a horizontal pass blurs the five moments with the
// separable 1-D window, a vertical pass finishes them, and the map value, |x - y| and the three
// per-pixel backward coefficients
//     A = dm/dmu1 - 2 mu1 dm/dsigma1^2 - mu2 dm/dsigma12,  B = dm/dsigma1^2,  C = dm/dsigma12
// are produced in registers.  The backward blurs A, B, C the same way (the window is symmetric)
// and forms dm_total/dx(p) = blur(A) + 2 x(p) blur(B) + y(p) blur(C).  Partial sums per workgroup
// are reduced in a fixed order (deterministic).  HBM: forward reads 8 B and writes 12 B per
// pixel-channel, backward reads 20 B and writes 4 B.
//
// Pearson: per column of [N, K] inputs, torchmetrics' two-pass form (means, then centred sums
// var_x, var_y, cov, each divided by N - 1; r = cov / sqrt(var_x var_y), clamped to [-1, 1]),
// with the reductions in double.
#include <math.h>

#include "gsr_internal.h"
#include "../../include/gsr_loss.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kR = 5;                 // window radius (window_size 11)
constexpr int kW = 2 * kR + 1;
#ifndef GSR_SSIM_TY
#define GSR_SSIM_TY 32
#endif
constexpr int kTX = 32, kTY = GSR_SSIM_TY;  // output tile
constexpr int kIX = kTX + 2 * kR;     // 42
constexpr int kIY = kTY + 2 * kR;     // 42
// Register blocking of the two blur passes: a thread of the horizontal pass produces kHS
// consecutive outputs of one row from kHS + 10 inputs held in registers (one LDS read per input
// instead of one per tap), a thread of the vertical pass kVS consecutive outputs of one column.
// Every output still sums its 11 taps in tap order, so the blurred values are those of the
// one-output-per-thread form.
constexpr int kSX = 44;               // LDS row stride of the halo tiles (16-B aligned rows)
constexpr int kHS = 8, kHN = kHS + 2 * kR;   // 18 inputs per horizontal task
constexpr int kVS = kTY / 8, kVN = kVS + 2 * kR;  // 14 inputs per vertical task at kTY = 32
static_assert(kIY * (kTX / kHS) <= kThreads, "one horizontal task per thread");
static_assert(kTX * (kTY / kVS) == kThreads, "one vertical task per thread");

// rows [0, kIY) x columns [0, kIX) of NP planes around (x0 - kR, y0 - kR), zero outside: every
// load of the thread is issued before the first LDS store, so the tile's global reads overlap
template <int NP>
__device__ __forceinline__ void load_halo(const float* const (&src)[NP], size_t plane, int x0,
                                          int y0, int H, int W, float (*dst)[kIY][kSX]) {
  constexpr int kIt = (kIX * kIY + kThreads - 1) / kThreads;
  float v[NP][kIt];
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    const int e = (int)threadIdx.x + it * kThreads;
    const int r = e / kIX, q = e - r * kIX;
    const int gy = y0 + r - kR, gx = x0 + q - kR;
    const bool in = e < kIX * kIY && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const size_t o = in ? plane + (size_t)gy * W + gx : 0;
#pragma unroll
    for (int p = 0; p < NP; p++) v[p][it] = in ? src[p][o] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    const int e = (int)threadIdx.x + it * kThreads;
    const int r = e / kIX, q = e - r * kIX;
    if (e < kIX * kIY)
#pragma unroll
      for (int p = 0; p < NP; p++) dst[p][r][q] = v[p][it];
  }
}

// kHN consecutive floats of an LDS row starting at a multiple of 8 (16-B aligned)
__device__ __forceinline__ void row_span(const float* row, float (&v)[kHN]) {
  const float4* p = reinterpret_cast<const float4*>(row);
#pragma unroll
  for (int i = 0; i < kHN / 4; i++) {
    const float4 t = p[i];
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
  const float2 t = reinterpret_cast<const float2*>(row)[kHN / 2 - 1];
  v[kHN - 2] = t.x;
  v[kHN - 1] = t.y;
}

struct Window {
  float w[kW];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// workgroup sum of two floats -> out[0], out[1] (thread 0)
__device__ __forceinline__ void block_sum2(float a, float b, float* out) {
  __shared__ float s[2][kThreads / 64];
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    s[0][w] = a;
    s[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = (s[0][0] + s[0][1]) + (s[0][2] + s[0][3]);
    out[1] = (s[1][0] + s[1][1]) + (s[1][2] + s[1][3]);
  }
}

struct SsimArgs {
  int C, H, W;
  const float *x, *y;     // [C,H,W]
  float *A, *B, *Cc;      // [C,H,W] backward coefficients (may be null: no grad needed)
  float* parts;           // [blocks][2]: sum of the map, sum of |x - y|
  Window win;
  float c1, c2;
};

// one 32x32 output tile (bx, by) of channel c; its partial sums go to parts[2 * b]
__device__ __forceinline__ void ssim_fwd_tile(const SsimArgs& a, int bx, int by, int c, size_t b) {
  // the blurs are explicit FMA chains and nothing else contracts: every kernel that inlines this
  // tile (the photometric loss, the training views' loss) computes the same bits (the reference's
  // conv2d fixes no evaluation order; parity is against float64, tests/test_losses.py)
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float sxy[2][kIY][kSX];
  __shared__ float h[5][kIY][kTX];
  float (*sx)[kSX] = sxy[0];
  float (*sy)[kSX] = sxy[1];
  const int x0 = bx * kTX, y0 = by * kTY;
  const size_t plane = (size_t)c * a.H * a.W;
  {
    const float* const src[2] = {a.x, a.y};
    load_halo<2>(src, plane, x0, y0, a.H, a.W, sxy);
  }
  __syncthreads();
  if (threadIdx.x < kIY * (kTX / kHS)) {
    const int r = (int)threadIdx.x / (kTX / kHS), q0 = ((int)threadIdx.x % (kTX / kHS)) * kHS;
    float u[kHN], v[kHN];
    row_span(&sx[r][q0], u);
    row_span(&sy[r][q0], v);
#pragma unroll
    for (int j = 0; j < kHS; j++) {
      float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
      for (int k = 0; k < kW; k++) {
        const float uk = u[j + k], vk = v[j + k], w = a.win.w[k];
        m1 = __builtin_fmaf(w, uk, m1);
        m2 = __builtin_fmaf(w, vk, m2);
        e11 = __builtin_fmaf(w, uk * uk, e11);
        e22 = __builtin_fmaf(w, vk * vk, e22);
        e12 = __builtin_fmaf(w, uk * vk, e12);
      }
      h[0][r][q0 + j] = m1;
      h[1][r][q0 + j] = m2;
      h[2][r][q0 + j] = e11;
      h[3][r][q0 + j] = e22;
      h[4][r][q0 + j] = e12;
    }
  }
  __syncthreads();
  float msum = 0.f, l1sum = 0.f;
  const int q = (int)threadIdx.x % kTX, r0 = ((int)threadIdx.x / kTX) * kVS;
  const int gx = x0 + q;
  float col[5][kVN];
#pragma unroll
  for (int m = 0; m < 5; m++)
#pragma unroll
    for (int i = 0; i < kVN; i++) col[m][i] = h[m][r0 + i][q];
#pragma unroll
  for (int i = 0; i < kVS; i++) {
    const int r = r0 + i, gy = y0 + r;
    if (gy >= a.H || gx >= a.W) continue;
    float mu1 = 0.f, mu2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int k = 0; k < kW; k++) {
      const float w = a.win.w[k];
      mu1 = __builtin_fmaf(w, col[0][i + k], mu1);
      mu2 = __builtin_fmaf(w, col[1][i + k], mu2);
      e11 = __builtin_fmaf(w, col[2][i + k], e11);
      e22 = __builtin_fmaf(w, col[3][i + k], e22);
      e12 = __builtin_fmaf(w, col[4][i + k], e12);
    }
    // _ssim (loss_utils.py:143-162), same expression order
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
    const float s1 = e11 - mu1_sq, s2 = e22 - mu2_sq, s12 = e12 - mu1_mu2;
    const float a1 = 2.f * mu1_mu2 + a.c1, a2 = 2.f * s12 + a.c2;
    const float b1 = (mu1_sq + mu2_sq) + a.c1, b2 = (s1 + s2) + a.c2;
    const float den = b1 * b2;
    const float m = (a1 * a2) / den;
    msum += m;
    const float xv = sx[r + kR][q + kR], yv = sy[r + kR][q + kR];
    l1sum += fabsf(xv - yv);
    if (a.A) {
      const float dmu1 = (2.f * mu2 * a2) / den - m * (2.f * mu1) / b1;
      const float ds1 = -m / b2;
      const float ds12 = (2.f * a1) / den;
      const size_t o = plane + (size_t)gy * a.W + gx;
      a.A[o] = dmu1 - 2.f * mu1 * ds1 - mu2 * ds12;
      a.B[o] = ds1;
      a.Cc[o] = ds12;
    }
  }
  block_sum2(msum, l1sum, a.parts + 2 * b);
}

__global__ __launch_bounds__(kThreads) void ssim_fwd_kernel(SsimArgs a) {
  ssim_fwd_tile(a, blockIdx.x, blockIdx.y, blockIdx.z,
                ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
}

// parts [n][2] -> out: loss, l1 mean, ssim mean (double accumulation, fixed order)
__global__ __launch_bounds__(kThreads) void ssim_reduce_kernel(const float* __restrict__ parts,
                                                               int n, double inv_count,
                                                               float lambda,
                                                               float* __restrict__ out) {
  __shared__ double s[2][kThreads];
  double m = 0.0, l = 0.0;
  for (int i = threadIdx.x; i < n; i += kThreads) {
    m += (double)parts[2 * i];
    l += (double)parts[2 * i + 1];
  }
  s[0][threadIdx.x] = m;
  s[1][threadIdx.x] = l;
  __syncthreads();
  for (int d = kThreads / 2; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d) {
      s[0][threadIdx.x] += s[0][threadIdx.x + d];
      s[1][threadIdx.x] += s[1][threadIdx.x + d];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float ssim = (float)(s[0][0] * inv_count), l1 = (float)(s[1][0] * inv_count);
    out[0] = (1.0f - lambda) * l1 + lambda * (1.0f - ssim);
    out[1] = l1;
    out[2] = ssim;
  }
}

struct SsimBwdArgs {
  int C, H, W;
  const float *x, *y, *A, *B, *Cc;
  const float *g_loss, *g_l1, *g_ssim;  // device scalars (null = 0)
  float lambda, inv_count;
  float* dx;
  Window win;
};

__device__ __forceinline__ void ssim_bwd_tile(const SsimBwdArgs& a, int bx, int by, int c) {
#pragma clang fp contract(off)  // explicit FMA blurs, as ssim_fwd_tile
  __shared__ __attribute__((aligned(16))) float s[3][kIY][kSX];
  __shared__ float h[3][kIY][kTX];
  const int x0 = bx * kTX, y0 = by * kTY;
  const size_t plane = (size_t)c * a.H * a.W;
  // d loss / d ssim_mean and d loss / d l1_mean for the three outputs (loss, l1, ssim)
  const float gl = a.g_loss ? *a.g_loss : 0.f;
  const float k_ssim = (-a.lambda * gl + (a.g_ssim ? *a.g_ssim : 0.f)) * a.inv_count;
  const float k_l1 = ((1.0f - a.lambda) * gl + (a.g_l1 ? *a.g_l1 : 0.f)) * a.inv_count;
  {
    const float* const src[3] = {a.A, a.B, a.Cc};
    load_halo<3>(src, plane, x0, y0, a.H, a.W, s);
  }
  __syncthreads();
  if (threadIdx.x < kIY * (kTX / kHS)) {
    const int r = (int)threadIdx.x / (kTX / kHS), q0 = ((int)threadIdx.x % (kTX / kHS)) * kHS;
#pragma unroll
    for (int m = 0; m < 3; m++) {
      float v[kHN];
      row_span(&s[m][r][q0], v);
#pragma unroll
      for (int j = 0; j < kHS; j++) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < kW; k++) acc = __builtin_fmaf(a.win.w[k], v[j + k], acc);
        h[m][r][q0 + j] = acc;
      }
    }
  }
  __syncthreads();
  const int q = (int)threadIdx.x % kTX, r0 = ((int)threadIdx.x / kTX) * kVS;
  const int gx = x0 + q;
  float col[3][kVN];
#pragma unroll
  for (int m = 0; m < 3; m++)
#pragma unroll
    for (int i = 0; i < kVN; i++) col[m][i] = h[m][r0 + i][q];
#pragma unroll
  for (int i = 0; i < kVS; i++) {
    const int gy = y0 + r0 + i;
    if (gy >= a.H || gx >= a.W) continue;
    float u0 = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll
    for (int k = 0; k < kW; k++) {
      const float w = a.win.w[k];
      u0 = __builtin_fmaf(w, col[0][i + k], u0);
      u1 = __builtin_fmaf(w, col[1][i + k], u1);
      u2 = __builtin_fmaf(w, col[2][i + k], u2);
    }
    const size_t o = plane + (size_t)gy * a.W + gx;
    const float xv = a.x[o], yv = a.y[o];
    const float dm = u0 + 2.f * xv * u1 + yv * u2;
    const float d = xv - yv;
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch.abs backward: sign
    a.dx[o] = k_ssim * dm + k_l1 * sgn;
  }
}

__global__ __launch_bounds__(kThreads) void ssim_bwd_kernel(SsimBwdArgs a) {
  ssim_bwd_tile(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---- Pearson -------------------------------------------------------------------------------------
// Column k of x (and of the transformed variant xt = 1 / (offset - x) when `variants` = 2) against
// column k of y; stats[k]: {sum x, sum y} then {Sxx, Syy, Sxy}; two passes.
struct PearsonArgs {
  int64_t N;
  int K;
  const float *x, *y;  // [N, K]
  double* acc;         // [variants][K][8]: sx, sy, sxx, syy, sxy
  double* parts;       // [variants][K][nblocks][3] per-workgroup partial sums
  int nblocks;
  int variants;
  float offset;
};

__device__ __forceinline__ float variant_x(float x, int v, float offset) {
  return v == 0 ? x : 1.0f / (-x + offset);  // train.py:128: 1 / (-depth_mono + 200)
}

__device__ double wave_sum_d(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Partial sums per workgroup, written to their own slots: no same-address atomics (on MI355X
// those serialise at device scope across the 8 XCDs' L2s), and a fixed reduction order.
template <int PASS>
__global__ __launch_bounds__(kThreads) void pearson_kernel(PearsonArgs a) {
  __shared__ double s[3][kThreads / 64];
  const int k = blockIdx.y, v = blockIdx.z;
  const double* acc = a.acc + ((size_t)v * a.K + k) * 8;
  double t0 = 0.0, t1 = 0.0, t2 = 0.0;
  double mx = 0.0, my = 0.0;
  if (PASS == 1) {
    mx = acc[0] / (double)a.N;
    my = acc[1] / (double)a.N;
  }
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.N;
       i += (int64_t)gridDim.x * kThreads) {
    const double xv = (double)variant_x(a.x[i * a.K + k], v, a.offset);
    const double yv = (double)a.y[i * a.K + k];
    if (PASS == 0) {
      t0 += xv;
      t1 += yv;
    } else {
      const double dx = xv - mx, dy = yv - my;
      t0 += dx * dx;
      t1 += dy * dy;
      t2 += dx * dy;
    }
  }
  t0 = wave_sum_d(t0);
  t1 = wave_sum_d(t1);
  t2 = wave_sum_d(t2);
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    s[0][w] = t0;
    s[1][w] = t1;
    s[2][w] = t2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int j = threadIdx.x;
    double* p = a.parts + (((size_t)v * a.K + k) * a.nblocks + blockIdx.x) * 3;
    p[j] = (s[j][0] + s[j][1]) + (s[j][2] + s[j][3]);
  }
}

// acc[v][k][PASS ? 2..4 : 0..1] = sum over the workgroup partials (grid: K x variants)
template <int PASS>
__global__ __launch_bounds__(kThreads) void pearson_reduce_kernel(PearsonArgs a) {
  __shared__ double s[3][kThreads];
  const int k = blockIdx.x, v = blockIdx.y;
  const double* p = a.parts + ((size_t)v * a.K + k) * a.nblocks * 3;
  double t[3] = {0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < a.nblocks; b += kThreads)
#pragma unroll
    for (int j = 0; j < 3; j++) t[j] += p[3 * b + j];
#pragma unroll
  for (int j = 0; j < 3; j++) s[j][threadIdx.x] = t[j];
  __syncthreads();
  for (int d = kThreads / 2; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d)
#pragma unroll
      for (int j = 0; j < 3; j++) s[j][threadIdx.x] += s[j][threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* acc = a.acc + ((size_t)v * a.K + k) * 8;
    if (PASS == 0) {
      acc[0] = s[0][0];
      acc[1] = s[1][0];
    } else {
      acc[2] = s[0][0];
      acc[3] = s[1][0];
      acc[4] = s[2][0];
    }
  }
}

// r per (variant, column); out_r[v*K + k]; loss = min over variants of 1 - r (first wins ties),
// out_sel[k] = chosen variant
__global__ void pearson_finish_kernel(PearsonArgs a, float* __restrict__ out_r,
                                      float* __restrict__ out_loss, int32_t* __restrict__ out_sel) {
  const int k = threadIdx.x;
  if (k >= a.K) return;
  float best = 0.f;
  int sel = 0;
  for (int v = 0; v < a.variants; v++) {
    const double* acc = a.acc + ((size_t)v * a.K + k) * 8;
    const double nb = (double)(a.N - 1);
    const double vx = acc[2] / nb, vy = acc[3] / nb, cxy = acc[4] / nb;
    float r = (float)(cxy / sqrt(vx * vy));
    if (r == r) r = fminf(fmaxf(r, -1.0f), 1.0f);  // torch.clamp keeps NaN
    out_r[v * a.K + k] = r;
    const float l = 1.0f - r;
    if (v == 0 || l < best) {  // Python min(a, b): b only if b < a
      best = l;
      sel = v;
    }
  }
  if (out_loss) out_loss[k] = best;
  if (out_sel) out_sel[k] = sel;
}

// d(1 - r_sel)/dy_i * g: -g * [ (x_i - mx) / sqrt(Sxx Syy) - r (y_i - my) / Syy ] (0 when clamped)
__global__ __launch_bounds__(kThreads) void pearson_bwd_kernel(PearsonArgs a,
                                                               const int32_t* __restrict__ sel,
                                                               const float* __restrict__ g,
                                                               float* __restrict__ dy,
                                                               float* __restrict__ dx) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.N) return;
  for (int k = 0; k < a.K; k++) {
    const int v = sel ? sel[k] : 0;
    const double* acc = a.acc + ((size_t)v * a.K + k) * 8;
    const double mx = acc[0] / (double)a.N, my = acc[1] / (double)a.N;
    const double sxx = acc[2], syy = acc[3], sxy = acc[4];
    const double rr = sxy / sqrt(sxx * syy);
    const bool pass = rr >= -1.0 && rr <= 1.0;  // clamp backward
    const double gk = pass ? -(double)(g ? g[k] : 1.0f) : 0.0;
    const double xv = (double)variant_x(a.x[i * a.K + k], v, a.offset);
    const double yv = (double)a.y[i * a.K + k];
    const double inv = 1.0 / sqrt(sxx * syy);
    if (dy) dy[i * a.K + k] = (float)(gk * ((xv - mx) * inv - rr * (yv - my) / syy));
    if (dx && v == 0) dx[i * a.K + k] = (float)(gk * ((yv - my) * inv - rr * (xv - mx) / sxx));
  }
}

// ---- one training view's loss in three launches (train.py:99-131, losses.train_view_loss) -------
// photometric (L1 + SSIM of image vs gt) + depth_weight * the Pearson depth term (depth_mono vs
// the rendered depth, min over mono and 1 / (offset - mono)).  Forward: SSIM tiles and the Pearson
// partial sums in ONE grid (the Pearson blocks follow the SSIM tiles), then one workgroup reduces
// both and writes every output including the total; backward: SSIM tiles + Pearson elements in
// one grid.  Pearson here is single-pass: sums of (x - x[0]), (y - y[0]) and their squares and
// product in double (the shift keeps the centred sums free of cancellation), instead of the
// two-pass means-then-centred form of gsr_pearson_loss; same r to double rounding.
constexpr int kViewPearsonSums = 8;  // x0, x0^2, x0 y, x1, x1^2, x1 y, y, y^2 (shifted)
constexpr int kViewPearsonMaxBlocks = 1024;

struct ViewLossArgs {
  SsimArgs ss;
  int nssim;                 // SSIM tiles (grid x of ssim_grid, flattened)
  int gx, gy;                // SSIM tile grid
  int64_t N;                 // depth pixels
  const float *mono, *depth;
  float offset, depth_weight;
  int npb;                   // Pearson partial blocks
  double* pparts;            // [npb][8]
  double* acc;               // [2][8]: the layout pearson_bwd_kernel reads (K = 1, variants = 2)
  int32_t* sel;              // [1]
  float* out;                // [5]: photometric loss, L1, SSIM, depth term, total (copy)
  float* total;              // [1]
  double inv_count;
  float lambda;
};

__device__ double block_sum_d(double v, double* lds) {  // thread 0 gets the workgroup sum
  v = wave_sum_d(v);
  const int w = (int)(threadIdx.x >> 6);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[w] = v;
  __syncthreads();
  return (lds[0] + lds[1]) + (lds[2] + lds[3]);
}

__device__ void view_pearson_partial(const ViewLossArgs& a, int b) {
  __shared__ double lds[kThreads / 64];
  const float x0s = a.mono[0], x1s = variant_x(a.mono[0], 1, a.offset), ys = a.depth[0];
  double t[kViewPearsonSums] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = (int64_t)b * kThreads + threadIdx.x; i < a.N; i += (int64_t)a.npb * kThreads) {
    const float m = a.mono[i];
    const double x0 = (double)m - (double)x0s;
    const double x1 = (double)variant_x(m, 1, a.offset) - (double)x1s;
    const double y = (double)a.depth[i] - (double)ys;
    t[0] += x0; t[1] += x0 * x0; t[2] += x0 * y;
    t[3] += x1; t[4] += x1 * x1; t[5] += x1 * y;
    t[6] += y;  t[7] += y * y;
  }
#pragma unroll
  for (int j = 0; j < kViewPearsonSums; j++) {
    const double v = block_sum_d(t[j], lds);
    if (threadIdx.x == 0) a.pparts[(size_t)b * kViewPearsonSums + j] = v;
  }
}

// (bodies shared by the one-view kernels and the several-views kernels: blk = the workgroup's
// index inside its view's grid)
__device__ __forceinline__ void view_loss_fwd_body(const ViewLossArgs& a, int blk) {
  // the Pearson blocks come first in the grid, so they run beside the SSIM tiles, not after them
  const int b = blk - a.npb;
  if (b >= 0) {
    const int per = a.gx * a.gy;
    const int c = b / per, r = b - c * per;
    ssim_fwd_tile(a.ss, r % a.gx, r / a.gx, c, (size_t)b);
  } else {
    view_pearson_partial(a, blk);
  }
}


__device__ __forceinline__ void view_loss_finish_body(const ViewLossArgs& a) {
  __shared__ double s[2][kThreads];
  __shared__ double q[kViewPearsonSums][kThreads / 64];
  // SSIM / L1 means exactly as ssim_reduce_kernel
  double m = 0.0, l = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < a.nssim; i += kThreads) {
    m += (double)a.ss.parts[2 * i];
    l += (double)a.ss.parts[2 * i + 1];
  }
  s[0][threadIdx.x] = m;
  s[1][threadIdx.x] = l;
  __syncthreads();
  for (int d = kThreads / 2; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d) {
      s[0][threadIdx.x] += s[0][threadIdx.x + d];
      s[1][threadIdx.x] += s[1][threadIdx.x + d];
    }
    __syncthreads();
  }
  // Pearson sums over the partial blocks, fixed order
  double t[kViewPearsonSums] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int i = threadIdx.x; i < a.npb; i += kThreads)
#pragma unroll
    for (int j = 0; j < kViewPearsonSums; j++) t[j] += a.pparts[(size_t)i * kViewPearsonSums + j];
  const int w = (int)(threadIdx.x >> 6);
#pragma unroll
  for (int j = 0; j < kViewPearsonSums; j++) {
    const double v = wave_sum_d(t[j]);
    if ((threadIdx.x & 63) == 0) q[j][w] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float ssim = (float)(s[0][0] * a.inv_count), l1 = (float)(s[1][0] * a.inv_count);
  const float photo = (1.0f - a.lambda) * l1 + a.lambda * (1.0f - ssim);
  double S[kViewPearsonSums];
#pragma unroll
  for (int j = 0; j < kViewPearsonSums; j++) S[j] = (q[j][0] + q[j][1]) + (q[j][2] + q[j][3]);
  const double n = (double)a.N;
  const float x0s = a.mono[0], x1s = variant_x(a.mono[0], 1, a.offset), ys = a.depth[0];
  const double syy = S[7] - S[6] * S[6] / n;
  float best = 0.f;
  int sel = 0;
  for (int v = 0; v < 2; v++) {
    const double sx = S[3 * v], sxx = S[3 * v + 1] - sx * sx / n, sxy = S[3 * v + 2] - sx * S[6] / n;
    double* acc = a.acc + (size_t)v * 8;  // pearson_bwd_kernel: mean = acc[0..1] / N, centred sums
    acc[0] = ((double)(v == 0 ? x0s : x1s) + sx / n) * n;
    acc[1] = ((double)ys + S[6] / n) * n;
    acc[2] = sxx;
    acc[3] = syy;
    acc[4] = sxy;
    float r = (float)(sxy / sqrt(sxx * syy));
    if (r == r) r = fminf(fmaxf(r, -1.0f), 1.0f);  // torch.clamp keeps NaN
    const float lv = 1.0f - r;
    if (v == 0 || lv < best) {  // Python min(a, b): b only if b < a
      best = lv;
      sel = v;
    }
  }
  *a.sel = sel;
  const float total = photo + a.depth_weight * best;  // torch.add(photo, depth, alpha=w)
  a.out[0] = photo;
  a.out[1] = l1;
  a.out[2] = ssim;
  a.out[3] = best;
  a.out[4] = total;
  *a.total = total;
}


struct ViewLossBwdArgs {
  SsimBwdArgs ss;
  int nssim, gx, gy;
  int npe;         // Pearson element blocks, first in the grid
  PearsonArgs pa;  // N, K = 1, x = mono, y = depth, variants = 2, acc
  const int32_t* sel;
  const float* g_total;
  float depth_weight;
  float* dd;
};

__device__ __forceinline__ void view_loss_bwd_body(const ViewLossBwdArgs& a, int blk) {
  const int b = blk - a.npe;
  if (b >= 0) {
    const int per = a.gx * a.gy;
    const int c = b / per, r = b - c * per;
    ssim_bwd_tile(a.ss, r % a.gx, r / a.gx, c);
    return;
  }
  // pearson_bwd_kernel's element work with grad_loss = g_total * depth_weight (as torch's g * w)
  const int64_t i = (int64_t)blk * kThreads + threadIdx.x;
  if (i >= a.pa.N) return;
  const int v = *a.sel;
  const double* acc = a.pa.acc + (size_t)v * 8;
  const double mx = acc[0] / (double)a.pa.N, my = acc[1] / (double)a.pa.N;
  const double sxx = acc[2], syy = acc[3], sxy = acc[4];
  const double rr = sxy / sqrt(sxx * syy);
  const bool pass = rr >= -1.0 && rr <= 1.0;
  const float gq = *a.g_total * a.depth_weight;
  const double gk = pass ? -(double)gq : 0.0;
  const double xv = (double)variant_x(a.pa.x[i], v, a.pa.offset);
  const double yv = (double)a.pa.y[i];
  const double inv = 1.0 / sqrt(sxx * syy);
  a.dd[i] = (float)(gk * ((xv - mx) * inv - rr * (yv - my) / syy));
}


// Several training views' losses per launch (the multi-view training step, losses.train_views_loss):
// workgroup b belongs to view k with first[k] <= b < first[k + 1]; per view exactly the one-view
// kernels' arithmetic, so every view's outputs and gradients are bitwise those of gsr_view_loss.
constexpr int kMaxLossViews = 8;
struct ViewLossViews {
  ViewLossArgs v[kMaxLossViews];
  uint32_t first[kMaxLossViews + 1];
  int V;
};
struct ViewLossBwdViews {
  ViewLossBwdArgs v[kMaxLossViews];
  uint32_t first[kMaxLossViews + 1];
  int V;
};
static_assert(sizeof(ViewLossViews) <= 4096 && sizeof(ViewLossBwdViews) <= 4096,
              "kernel argument size");
__device__ __forceinline__ int loss_view(const uint32_t* first, int V, uint32_t b) {
  int k = 0;
  while (k + 1 < V && b >= first[k + 1]) k++;
  return k;
}
__global__ __launch_bounds__(kThreads) void view_loss_fwd_views_kernel(ViewLossViews m) {
  const int k = loss_view(m.first, m.V, blockIdx.x);
  view_loss_fwd_body(m.v[k], (int)(blockIdx.x - m.first[k]));
}
__global__ __launch_bounds__(kThreads) void view_loss_finish_views_kernel(ViewLossViews m) {
  view_loss_finish_body(m.v[blockIdx.x]);  // one workgroup per view
}
__global__ __launch_bounds__(kThreads) void view_loss_bwd_views_kernel(ViewLossBwdViews m) {
  const int k = loss_view(m.first, m.V, blockIdx.x);
  view_loss_bwd_body(m.v[k], (int)(blockIdx.x - m.first[k]));
}

}  // namespace
}  // namespace gsr

using namespace gsr;

namespace {

Window make_window() {
  // loss_utils.py:119-121: exp(-(x - 5)^2 / (2 sigma^2)) in double, stored as float32, then
  // normalised in float32
  Window w;
  float g[kW], sum = 0.f;
  for (int x = 0; x < kW; x++) {
    g[x] = (float)exp(-(double)((x - kR) * (x - kR)) / (2.0 * 1.5 * 1.5));
    sum += g[x];
  }
  for (int x = 0; x < kW; x++) w.w[x] = g[x] / sum;
  return w;
}

dim3 ssim_grid(int C, int H, int W) {
  return dim3((unsigned)((W + kTX - 1) / kTX), (unsigned)((H + kTY - 1) / kTY), (unsigned)C);
}

size_t ssim_blocks(int C, int H, int W) {
  const dim3 g = ssim_grid(C, H, W);
  return (size_t)g.x * g.y * g.z;
}

}  // namespace

extern "C" size_t gsr_photometric_scratch_bytes(int C, int H, int W) {
  if (C <= 0 || H <= 0 || W <= 0) return 0;
  Carver c(nullptr);
  c.take<float>((size_t)C * H * W * 3);
  c.take<float>(2 * ssim_blocks(C, H, W));
  return c.size();
}

static void carve_photometric(void* scratch, int C, int H, int W, float** A, float** B, float** Cc,
                              float** parts) {
  Carver c((char*)scratch);
  const size_t n = (size_t)C * H * W;
  float* abc = c.take<float>(n * 3);
  *A = abc;
  *B = abc + n;
  *Cc = abc + 2 * n;
  *parts = c.take<float>(2 * ssim_blocks(C, H, W));
}

extern "C" int gsr_photometric_loss(int C, int H, int W, const float* image, const float* gt,
                                    float lambda_dssim, int need_grad, float* out,
                                    void* scratch, void* stream) {
  if (C <= 0 || H <= 0 || W <= 0 || !image || !gt || !out || !scratch) return 1;
  SsimArgs a{};
  a.C = C; a.H = H; a.W = W;
  a.x = image; a.y = gt;
  float *A, *B, *Cc, *parts;
  carve_photometric(scratch, C, H, W, &A, &B, &Cc, &parts);
  a.A = need_grad ? A : nullptr;
  a.B = need_grad ? B : nullptr;
  a.Cc = need_grad ? Cc : nullptr;
  a.parts = parts;
  a.win = make_window();
  a.c1 = (float)(0.01 * 0.01);
  a.c2 = (float)(0.03 * 0.03);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ssim_fwd_kernel, ssim_grid(C, H, W), dim3(kThreads), 0, s, a);
  const double inv = 1.0 / ((double)C * H * W);
  hipLaunchKernelGGL(ssim_reduce_kernel, dim3(1), dim3(kThreads), 0, s, parts,
                     (int)ssim_blocks(C, H, W), inv, lambda_dssim, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_photometric_loss_backward(int C, int H, int W, const float* image,
                                             const float* gt, float lambda_dssim,
                                             const float* grad_loss, const float* grad_l1,
                                             const float* grad_ssim, float* grad_image,
                                             void* scratch, void* stream) {
  if (C <= 0 || H <= 0 || W <= 0 || !image || !gt || !grad_image || !scratch) return 1;
  SsimBwdArgs a{};
  a.C = C; a.H = H; a.W = W;
  a.x = image; a.y = gt;
  float *A, *B, *Cc, *parts;
  carve_photometric(scratch, C, H, W, &A, &B, &Cc, &parts);
  a.A = A; a.B = B; a.Cc = Cc;
  a.g_loss = grad_loss; a.g_l1 = grad_l1; a.g_ssim = grad_ssim;
  a.lambda = lambda_dssim;
  a.inv_count = (float)(1.0 / ((double)C * H * W));
  a.dx = grad_image;
  a.win = make_window();
  hipLaunchKernelGGL(ssim_bwd_kernel, ssim_grid(C, H, W), dim3(kThreads), 0, (hipStream_t)stream,
                     a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static unsigned pearson_blocks(int64_t N) {
  const int64_t b = (N + kThreads * 8 - 1) / (kThreads * 8);
  return (unsigned)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

extern "C" size_t gsr_pearson_scratch_bytes(int K, int variants) {
  if (K <= 0 || variants < 1 || variants > 2) return 0;
  Carver c(nullptr);
  c.take<double>((size_t)variants * K * 8);
  c.take<float>((size_t)variants * K);
  c.take<int32_t>((size_t)K);
  c.take<double>((size_t)variants * K * 1024 * 3);
  return c.size();
}

static void carve_pearson(void* scratch, int K, int variants, double** acc, float** r,
                          int32_t** sel, double** parts) {
  Carver c((char*)scratch);
  *acc = c.take<double>((size_t)variants * K * 8);
  *r = c.take<float>((size_t)variants * K);
  *sel = c.take<int32_t>((size_t)K);
  *parts = c.take<double>((size_t)variants * K * 1024 * 3);
}

extern "C" int gsr_pearson_loss(int64_t N, int K, const float* x, const float* y, int variants,
                                float offset, float* out_r, float* out_loss, void* scratch,
                                void* stream) {
  if (N < 2 || K < 1 || K > 256 || variants < 1 || variants > 2 || !x || !y || !scratch)
    return 1;
  hipStream_t s = (hipStream_t)stream;
  PearsonArgs a{};
  a.N = N; a.K = K; a.x = x; a.y = y; a.variants = variants; a.offset = offset;
  a.nblocks = (int)pearson_blocks(N);
  float* r;
  int32_t* sel;
  carve_pearson(scratch, K, variants, &a.acc, &r, &sel, &a.parts);
  const dim3 grid((unsigned)a.nblocks, (unsigned)K, (unsigned)variants);
  const dim3 rgrid((unsigned)K, (unsigned)variants);
  hipLaunchKernelGGL(pearson_kernel<0>, grid, dim3(kThreads), 0, s, a);
  hipLaunchKernelGGL(pearson_reduce_kernel<0>, rgrid, dim3(kThreads), 0, s, a);
  hipLaunchKernelGGL(pearson_kernel<1>, grid, dim3(kThreads), 0, s, a);
  hipLaunchKernelGGL(pearson_reduce_kernel<1>, rgrid, dim3(kThreads), 0, s, a);
  hipLaunchKernelGGL(pearson_finish_kernel, dim3(1), dim3(256), 0, s, a, r, out_loss, sel);
  if (out_r &&
      hipMemcpyAsync(out_r, r, (size_t)variants * K * sizeof(float), hipMemcpyDeviceToDevice, s) !=
          hipSuccess)
    return 2;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_pearson_loss_backward(int64_t N, int K, const float* x, const float* y,
                                         int variants, float offset, const float* grad_loss,
                                         float* grad_y, float* grad_x, void* scratch,
                                         void* stream) {
  if (N < 2 || K < 1 || K > 256 || variants < 1 || variants > 2 || !x || !y || !scratch ||
      (grad_x && variants != 1))
    return 1;
  PearsonArgs a{};
  a.N = N; a.K = K; a.x = x; a.y = y; a.variants = variants; a.offset = offset;
  float* r;
  int32_t* sel;
  carve_pearson(scratch, K, variants, &a.acc, &r, &sel, &a.parts);
  hipLaunchKernelGGL(pearson_bwd_kernel, dim3((unsigned)((N + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, (hipStream_t)stream, a, sel, grad_loss, grad_y, grad_x);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static size_t view_pearson_bytes() {
  Carver c(nullptr);
  c.take<double>(2 * 8);
  c.take<int32_t>(4);
  c.take<double>((size_t)kViewPearsonMaxBlocks * kViewPearsonSums);
  return c.size();
}

extern "C" size_t gsr_view_loss_scratch_bytes(int C, int H, int W) {
  const size_t p = gsr_photometric_scratch_bytes(C, H, W);
  return p ? ((p + 255) & ~(size_t)255) + view_pearson_bytes() : 0;
}

static void carve_view(void* scratch, int C, int H, int W, float** A, float** B, float** Cc,
                       float** parts, double** acc, int32_t** sel, double** pparts) {
  carve_photometric(scratch, C, H, W, A, B, Cc, parts);
  const size_t p = (gsr_photometric_scratch_bytes(C, H, W) + 255) & ~(size_t)255;
  Carver c((char*)scratch + p);
  *acc = c.take<double>(2 * 8);
  *sel = c.take<int32_t>(4);
  *pparts = c.take<double>((size_t)kViewPearsonMaxBlocks * kViewPearsonSums);
}

static ViewLossArgs view_loss_args(int C, int H, int W, const float* image, const float* gt,
                                   float lambda_dssim, int64_t N, const float* depth,
                                   const float* depth_mono, float offset, float depth_weight,
                                   int need_grad, float* out, float* total, void* scratch) {
  ViewLossArgs a{};
  a.ss.C = C; a.ss.H = H; a.ss.W = W;
  a.ss.x = image; a.ss.y = gt;
  float *A, *B, *Cc;
  carve_view(scratch, C, H, W, &A, &B, &Cc, &a.ss.parts, &a.acc, &a.sel, &a.pparts);
  a.ss.A = need_grad ? A : nullptr;
  a.ss.B = need_grad ? B : nullptr;
  a.ss.Cc = need_grad ? Cc : nullptr;
  a.ss.win = make_window();
  a.ss.c1 = (float)(0.01 * 0.01);
  a.ss.c2 = (float)(0.03 * 0.03);
  const dim3 g = ssim_grid(C, H, W);
  a.gx = (int)g.x; a.gy = (int)g.y;
  a.nssim = (int)ssim_blocks(C, H, W);
  a.N = N; a.mono = depth_mono; a.depth = depth;
  a.offset = offset; a.depth_weight = depth_weight;
  a.npb = (int)pearson_blocks(N);
  a.out = out; a.total = total;
  a.inv_count = 1.0 / ((double)C * H * W);
  a.lambda = lambda_dssim;
  return a;
}

extern "C" int gsr_view_loss(int C, int H, int W, const float* image, const float* gt,
                             float lambda_dssim, int64_t N, const float* depth,
                             const float* depth_mono, float offset, float depth_weight,
                             int need_grad, float* out, float* total, void* scratch,
                             void* stream) {
  if (C <= 0 || H <= 0 || W <= 0 || N < 2 || !image || !gt || !depth || !depth_mono || !out ||
      !total || !scratch)
    return 1;
  // the several-views kernels with one view: the single-view and the multi-view training steps
  // run the same compiled code (the SSIM tiles contract to FMA per instance), so their losses and
  // gradients agree bit for bit
  ViewLossViews m{};
  m.V = 1;
  m.v[0] = view_loss_args(C, H, W, image, gt, lambda_dssim, N, depth, depth_mono, offset,
                          depth_weight, need_grad, out, total, scratch);
  m.first[0] = 0;
  m.first[1] = (uint32_t)(m.v[0].nssim + m.v[0].npb);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(view_loss_fwd_views_kernel, dim3(m.first[1]), dim3(kThreads), 0, s, m);
  hipLaunchKernelGGL(view_loss_finish_views_kernel, dim3(1), dim3(kThreads), 0, s, m);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static ViewLossBwdArgs view_loss_bwd_args(int C, int H, int W, const float* image,
                                          const float* gt, float lambda_dssim, int64_t N,
                                          const float* depth, const float* depth_mono,
                                          float offset, float depth_weight,
                                          const float* grad_total, float* grad_image,
                                          float* grad_depth, void* scratch) {
  ViewLossBwdArgs a{};
  a.ss.C = C; a.ss.H = H; a.ss.W = W;
  a.ss.x = image; a.ss.y = gt;
  float *A, *B, *Cc, *parts;
  double *acc, *pparts;
  int32_t* sel;
  carve_view(scratch, C, H, W, &A, &B, &Cc, &parts, &acc, &sel, &pparts);
  a.ss.A = A; a.ss.B = B; a.ss.Cc = Cc;
  a.ss.g_loss = grad_total; a.ss.g_l1 = nullptr; a.ss.g_ssim = nullptr;
  a.ss.lambda = lambda_dssim;
  a.ss.inv_count = (float)(1.0 / ((double)C * H * W));
  a.ss.dx = grad_image;
  a.ss.win = make_window();
  const dim3 g = ssim_grid(C, H, W);
  a.gx = (int)g.x; a.gy = (int)g.y;
  a.nssim = (int)ssim_blocks(C, H, W);
  a.pa.N = N; a.pa.K = 1; a.pa.x = depth_mono; a.pa.y = depth; a.pa.variants = 2;
  a.pa.offset = offset; a.pa.acc = acc;
  a.sel = sel;
  a.g_total = grad_total;
  a.depth_weight = depth_weight;
  a.dd = grad_depth;
  a.npe = (int)((N + kThreads - 1) / kThreads);
  return a;
}

extern "C" int gsr_view_loss_backward(int C, int H, int W, const float* image, const float* gt,
                                      float lambda_dssim, int64_t N, const float* depth,
                                      const float* depth_mono, float offset, float depth_weight,
                                      const float* grad_total, float* grad_image,
                                      float* grad_depth, void* scratch, void* stream) {
  if (C <= 0 || H <= 0 || W <= 0 || N < 2 || !image || !gt || !depth || !depth_mono ||
      !grad_total || !grad_image || !grad_depth || !scratch)
    return 1;
  ViewLossBwdViews m{};  // (one view: see gsr_view_loss)
  m.V = 1;
  m.v[0] = view_loss_bwd_args(C, H, W, image, gt, lambda_dssim, N, depth, depth_mono, offset,
                              depth_weight, grad_total, grad_image, grad_depth, scratch);
  m.first[0] = 0;
  m.first[1] = (uint32_t)(m.v[0].nssim + m.v[0].npe);
  hipLaunchKernelGGL(view_loss_bwd_views_kernel, dim3(m.first[1]), dim3(kThreads), 0,
                     (hipStream_t)stream, m);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// V views back to back: images [V][C][H][W], depths [V][N], grads alike; gts / depth_monos one
// pointer per view; out [V][5], total [V]; scratch V x gsr_view_loss_scratch_bytes(C, H, W).
extern "C" int gsr_view_loss_views(int V, int C, int H, int W, const float* images,
                                   const float* const* gts, float lambda_dssim, int64_t N,
                                   const float* depths, const float* const* depth_monos,
                                   float offset, float depth_weight, int need_grad, float* out,
                                   float* total, void* scratch, void* stream) {
  if (V <= 0 || V > kMaxLossViews || C <= 0 || H <= 0 || W <= 0 || N < 2 || !images || !gts ||
      !depths || !depth_monos || !out || !total || !scratch)
    return 1;
  const size_t sb = gsr_view_loss_scratch_bytes(C, H, W);
  const size_t img = (size_t)C * H * W;
  ViewLossViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    if (!gts[k] || !depth_monos[k]) return 1;
    m.v[k] = view_loss_args(C, H, W, images + (size_t)k * img, gts[k], lambda_dssim, N,
                            depths + (size_t)k * N, depth_monos[k], offset, depth_weight,
                            need_grad, out + 5 * k, total + k, (char*)scratch + (size_t)k * sb);
    m.first[k + 1] = m.first[k] + (uint32_t)(m.v[k].nssim + m.v[k].npb);
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(view_loss_fwd_views_kernel, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  hipLaunchKernelGGL(view_loss_finish_views_kernel, dim3((unsigned)V), dim3(kThreads), 0, s, m);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_view_loss_views_backward(int V, int C, int H, int W, const float* images,
                                            const float* const* gts, float lambda_dssim,
                                            int64_t N, const float* depths,
                                            const float* const* depth_monos, float offset,
                                            float depth_weight, const float* grad_total,
                                            float* grad_images, float* grad_depths,
                                            void* scratch, void* stream) {
  if (V <= 0 || V > kMaxLossViews || C <= 0 || H <= 0 || W <= 0 || N < 2 || !images || !gts ||
      !depths || !depth_monos || !grad_total || !grad_images || !grad_depths || !scratch)
    return 1;
  const size_t sb = gsr_view_loss_scratch_bytes(C, H, W);
  const size_t img = (size_t)C * H * W;
  ViewLossBwdViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    if (!gts[k] || !depth_monos[k]) return 1;
    m.v[k] = view_loss_bwd_args(C, H, W, images + (size_t)k * img, gts[k], lambda_dssim, N,
                                depths + (size_t)k * N, depth_monos[k], offset, depth_weight,
                                grad_total + k, grad_images + (size_t)k * img,
                                grad_depths + (size_t)k * N, (char*)scratch + (size_t)k * sb);
    m.first[k + 1] = m.first[k] + (uint32_t)(m.v[k].nssim + m.v[k].npe);
  }
  hipLaunchKernelGGL(view_loss_bwd_views_kernel, dim3(m.first[V]), dim3(kThreads), 0,
                     (hipStream_t)stream, m);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

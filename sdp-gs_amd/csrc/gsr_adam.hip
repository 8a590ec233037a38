// gsr_adam.hip -- fused multi-tensor Adam step for the Gaussian parameters.
//
// Reference: GaussianModel.training_setup builds torch.optim.Adam(param_groups, lr=0.0,
// eps=1e-15) over _xyz, _features_dc, _features_rest, _opacity, _scaling, _rotation (and
// _language_feature), one tensor per group with its own learning rate
// (scene/gaussian_model.py:217-271), and train.py steps it after every backward
// (train.py:229-231).  PyTorch's default CUDA/HIP Adam is the foreach implementation: per group
// 8+ element-wise passes over the parameter, gradient and both moments.  Here one launch updates
// every tensor of every group in a single streaming pass: per element read p, g, m, v and write
// p, m, v (28 bytes), HBM-bound.
//
// Arithmetic follows torch.optim.adam._multi_tensor_adam (non-capturable, no amsgrad):
//   g' = g + wd * p                       (weight_decay != 0, L2 form)
//   m  = lerp(m, g', 1 - beta1)           (torch's lerp: a + w (b - a) for w < 0.5)
//   v  = v * beta2 + (1 - beta2) * g' * g'
//   p  = p + step_size * (m / (sqrt(v) / bc2_sqrt + eps)),  step_size = -lr / (1 - beta1^t)
// with the per-tensor scalars computed on the host in double, as PyTorch does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>

#include "../../include/gsr_optim.h"

namespace gsr {
uint32_t* forward_faults_word();  // gsr_sort.hip: sticky fault word of failed rasterizer forwards
}

namespace {

constexpr int kThreads = 256;
constexpr int kVecPerThread = 4;                       // float4s per thread per workgroup
constexpr int kBlockElems = kThreads * kVecPerThread * 4;  // 4096 floats per workgroup

struct AdamArgs {
  int n;  // tensors
  float* p[GSR_ADAM_MAX_TENSORS];
  const float* g[GSR_ADAM_MAX_TENSORS];
  float* m[GSR_ADAM_MAX_TENSORS];
  float* v[GSR_ADAM_MAX_TENSORS];
  int64_t numel[GSR_ADAM_MAX_TENSORS];
  uint32_t block0[GSR_ADAM_MAX_TENSORS + 1];  // first workgroup of each tensor
  float step_size[GSR_ADAM_MAX_TENSORS];     // -lr / (1 - beta1^t)
  float bc2_sqrt[GSR_ADAM_MAX_TENSORS];      // sqrt(1 - beta2^t)
  float wd[GSR_ADAM_MAX_TENSORS];
  uint32_t vec_ok;                           // bit t: all four arrays of tensor t 16-B aligned
  float w1, beta2, one_m_beta2, eps;
  // the step's skip decision, read once per workgroup from one float written before this
  // launch (step_guard_kernel's snapshot of the device's forward fault word, or that snapshot
  // SUM-all-reduced over the ranks): != 0 = some forward of the step failed (its gradients are
  // NaN), so every parameter and moment stays untouched (include/gsr_optim.h)
  const float* skip;
  uint32_t* host_skipped;  // pinned host word: 1 = this step was skipped, 0 = applied (or NULL)
};

__device__ __forceinline__ float lerp_torch(float a, float b, float w) {
  return w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float wd,
                                         float w1, float beta2, float one_m_beta2, float eps,
                                         float step_size, float bc2_sqrt) {
  if (wd != 0.0f) g = g + p * wd;
  m = lerp_torch(m, g, w1);
  v = v * beta2;
  v = v + one_m_beta2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + step_size * (m / denom);
}

// Every element is touched once per step and the step's 1.7 GB (1M Gaussians) dwarfs the caches:
// 2 = every load and store nontemporal (`nt`: no cache allocation), 0.327 -> 0.295 ms at 1M
// (5.3 -> 5.9 TB/s, scripts/adam_bench.py); 1 = only g loaded and p, m, v stored nontemporally
// (0.302 ms); 0 = plain vector accesses
#ifndef GSR_ADAM_NT
#define GSR_ADAM_NT 2
#endif
template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
  if (NT) {
    const float* f = reinterpret_cast<const float*>(p);
    return make_float4(__builtin_nontemporal_load(f), __builtin_nontemporal_load(f + 1),
                       __builtin_nontemporal_load(f + 2), __builtin_nontemporal_load(f + 3));
  }
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(float4* p, float4 v) {
  if (NT) {
    float* f = reinterpret_cast<float*>(p);
    __builtin_nontemporal_store(v.x, f);
    __builtin_nontemporal_store(v.y, f + 1);
    __builtin_nontemporal_store(v.z, f + 2);
    __builtin_nontemporal_store(v.w, f + 3);
    return;
  }
  *p = v;
}

// One lane: slot[0] = (the device's sticky forward fault word != 0) ? 1 : 0.  Every workgroup of
// the Adam launch behind it reads this one snapshot, so a forward failing on another stream while
// Adam runs cannot leave some tensors updated and others not.
__global__ void step_guard_kernel(const uint32_t* __restrict__ fault, float* __restrict__ slot) {
  if (threadIdx.x == 0)
    slot[0] = (fault && __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1.0f
                                                                                                : 0.0f;
}

__global__ __launch_bounds__(kThreads) void adam_kernel(AdamArgs a) {
  const bool skipped = !(*a.skip == 0.0f);  // workgroup-uniform; NaN counts as a failure
  if (a.host_skipped && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.host_skipped, skipped ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (skipped) return;
  const uint32_t b = blockIdx.x;
  int t = 0;
  while (t + 1 < a.n && b >= a.block0[t + 1]) t++;  // workgroup-uniform, <= 16 tensors
  const int64_t base = (int64_t)(b - a.block0[t]) * kBlockElems;
  const int64_t n = a.numel[t];
  float* __restrict__ P = a.p[t];
  const float* __restrict__ G = a.g[t];
  float* __restrict__ M = a.m[t];
  float* __restrict__ V = a.v[t];
  const float ss = a.step_size[t], bc = a.bc2_sqrt[t], wd = a.wd[t];
  if (((a.vec_ok >> t) & 1u) && base + kBlockElems <= n) {
    // full workgroup, 16-byte vectors, all loads of a lane in flight before the math
    float4 pv[kVecPerThread], gv[kVecPerThread], mv[kVecPerThread], vv[kVecPerThread];
#pragma unroll
    for (int u = 0; u < kVecPerThread; u++) {
      const int64_t q = (base >> 2) + (int64_t)u * kThreads + threadIdx.x;
      pv[u] = ld4<GSR_ADAM_NT == 2>(reinterpret_cast<const float4*>(P) + q);
      gv[u] = ld4<GSR_ADAM_NT >= 1>(reinterpret_cast<const float4*>(G) + q);
      mv[u] = ld4<GSR_ADAM_NT == 2>(reinterpret_cast<const float4*>(M) + q);
      vv[u] = ld4<GSR_ADAM_NT == 2>(reinterpret_cast<const float4*>(V) + q);
    }
#pragma unroll
    for (int u = 0; u < kVecPerThread; u++) {
      adam_one(pv[u].x, gv[u].x, mv[u].x, vv[u].x, wd, a.w1, a.beta2, a.one_m_beta2, a.eps, ss, bc);
      adam_one(pv[u].y, gv[u].y, mv[u].y, vv[u].y, wd, a.w1, a.beta2, a.one_m_beta2, a.eps, ss, bc);
      adam_one(pv[u].z, gv[u].z, mv[u].z, vv[u].z, wd, a.w1, a.beta2, a.one_m_beta2, a.eps, ss, bc);
      adam_one(pv[u].w, gv[u].w, mv[u].w, vv[u].w, wd, a.w1, a.beta2, a.one_m_beta2, a.eps, ss, bc);
      const int64_t q = (base >> 2) + (int64_t)u * kThreads + threadIdx.x;
      st4<GSR_ADAM_NT >= 1>(reinterpret_cast<float4*>(P) + q, pv[u]);
      st4<GSR_ADAM_NT >= 1>(reinterpret_cast<float4*>(M) + q, mv[u]);
      st4<GSR_ADAM_NT >= 1>(reinterpret_cast<float4*>(V) + q, vv[u]);
    }
    return;
  }
  // tail workgroup of a tensor (or unaligned tensor): scalar, coalesced
  const int64_t end = base + kBlockElems < n ? base + kBlockElems : n;
  for (int64_t i = base + threadIdx.x; i < end; i += kThreads) {
    float p = P[i], m = M[i], v = V[i];
    adam_one(p, G[i], m, v, wd, a.w1, a.beta2, a.one_m_beta2, a.eps, ss, bc);
    P[i] = p;
    M[i] = m;
    V[i] = v;
  }
}

bool aligned(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// One float per device for the guard snapshot of a step without a caller-provided skip slot.
float* device_guard_slot() {
  constexpr int kMaxDev = 64;
  static std::atomic<float*> cache[kMaxDev];
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  float* s = cache[dev].load(std::memory_order_acquire);
  if (s) return s;
  std::lock_guard<std::mutex> lock(mu);
  s = cache[dev].load(std::memory_order_relaxed);
  if (!s) {
    void* p = nullptr;
    if (hipMalloc(&p, 256) != hipSuccess) return nullptr;
    s = (float*)p;
    cache[dev].store(s, std::memory_order_release);
  }
  return s;
}

}  // namespace

extern "C" int gsr_step_guard(float* slot, void* stream) {
  if (!slot) return 1;
  hipLaunchKernelGGL(step_guard_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     gsr::forward_faults_word(), slot);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int gsr_adam_step(int n_tensors, float* const* params, const float* const* grads,
                             float* const* exp_avg, float* const* exp_avg_sq,
                             const int64_t* numel, const double* lr, const double* weight_decay,
                             const double* step, double beta1, double beta2, double eps,
                             void* stream) {
  return gsr_adam_step_guarded(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, lr,
                               weight_decay, step, beta1, beta2, eps, nullptr, nullptr, stream);
}

extern "C" int gsr_adam_step_guarded(int n_tensors, float* const* params, const float* const* grads,
                                     float* const* exp_avg, float* const* exp_avg_sq,
                                     const int64_t* numel, const double* lr,
                                     const double* weight_decay, const double* step, double beta1,
                                     double beta2, double eps, const float* skip,
                                     uint32_t* host_skipped, void* stream) {
  if (n_tensors < 0 || n_tensors > GSR_ADAM_MAX_TENSORS) return 1;
  if (n_tensors == 0) return 0;
  AdamArgs a{};
  a.n = n_tensors;
  uint32_t blocks = 0;
  for (int t = 0; t < n_tensors; t++) {
    if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t] || numel[t] < 0 || step[t] < 1)
      return 1;
    a.p[t] = params[t]; a.g[t] = grads[t]; a.m[t] = exp_avg[t]; a.v[t] = exp_avg_sq[t];
    a.numel[t] = numel[t];
    a.block0[t] = blocks;
    const int64_t nb = (numel[t] + kBlockElems - 1) / kBlockElems;
    if ((int64_t)blocks + nb > 0x7fffffffLL) return 1;
    blocks += (uint32_t)nb;
    // torch: bias_correction = 1 - beta ** step in double; step_size = (lr / bc1) * -1;
    // bias_correction2_sqrt = bc2 ** 0.5 -- scalars reach the kernels as float
    const double bc1 = 1.0 - __builtin_pow(beta1, step[t]);
    const double bc2 = 1.0 - __builtin_pow(beta2, step[t]);
    a.step_size[t] = (float)((lr[t] / bc1) * -1.0);
    a.bc2_sqrt[t] = (float)__builtin_sqrt(bc2);
    a.wd[t] = (float)weight_decay[t];
    if (aligned(params[t]) && aligned(grads[t]) && aligned(exp_avg[t]) && aligned(exp_avg_sq[t]))
      a.vec_ok |= 1u << t;
  }
  a.block0[n_tensors] = blocks;
  a.w1 = (float)(1.0 - beta1);
  a.beta2 = (float)beta2;
  a.one_m_beta2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  if (blocks == 0) return 0;
  if (!skip) {  // snapshot the device's fault word into this device's guard slot first
    float* slot = device_guard_slot();
    if (!slot) return 2;
    if (gsr_step_guard(slot, stream) != 0) return 2;
    skip = slot;
  }
  a.skip = skip;
  a.host_skipped = host_skipped;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

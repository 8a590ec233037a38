// gsr_api.cpp -- host orchestration behind the C ABI (include/gsr.h).
//
// Sequence per view (reference: Rasterizer::forward, cuda_rasterizer/rasterizer_impl.cu:198-336):
//   preprocess -> stable depth sort of the P splats -> inclusive scan of tile counts in depth
//   order -> 8-byte readback of the instance count R (+ error flag) -> duplicate tile ids in depth
//   order -> stable radix sort of the R tile ids over ceil(log2(tiles)) bits -> tile ranges ->
//   blend.  Backward (rasterizer_impl.cu:340-434): zero the accumulators -> backward blend ->
//   fused per-Gaussian backward.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_testing.h"
#include "gsr_internal.h"

namespace gsr {

GeomState carve_geom(char* base, size_t P) {
  Carver c(base);
  GeomState g{};
  g.flags = c.take<uint32_t>(4);
  g.dkey_a = c.take<uint32_t>(P);
  g.dval_a = c.take<uint32_t>(P);
  g.dkey_b = c.take<uint32_t>(P);
  g.dval_b = c.take<uint32_t>(P);
  g.dkey_c = c.take<uint32_t>(P);
  g.dval_c = c.take<uint32_t>(P);
  g.clamped = c.take<uint8_t>(P);
  g.radii = c.take<int32_t>(P);
  g.rec = c.take<float4>(4 * P);
  g.bword = c.take<uint2>(P);
  g.tiles_touched = c.take<uint32_t>(P);
  g.offsets = c.take<uint32_t>(P);
  g.acc = c.take<float>((size_t)kAccFloats * P);
  g.ebeg = c.take<uint32_t>(P);
  g.sort = take_sort_scratch(c, P);
  g.scan_status = c.take<uint64_t>(scan_lb_words(P));
  g.ttot = c.take<uint32_t>(kSortTotTileWords);
  g.scan_parts = c.take<uint32_t>(scan_parts(P) + 1);
  g.pre_parts = c.take<uint32_t>(2 * ((P + 255) / 256) + 1);
  g.bytes = c.size();
  return g;
}

BinState carve_bin(char* base, size_t R, bool rows) {
  Carver c(base);
  BinState b{};
  b.tag = c.take<uint32_t>(4);
  b.tkey_a = c.take<uint32_t>(R);
  b.tval_a = c.take<uint32_t>(R);
  b.tkey_b = c.take<uint32_t>(R);
  b.tval_b = c.take<uint32_t>(R);
  b.sort = take_sort_scratch(c, R);
  if (rows) {
    b.egid = c.take<uint32_t>(R);
    b.partial = c.take<float>(R * kAccFloats);
  }
  b.bytes = c.size();
  return b;
}

ImgState carve_img(char* base, size_t W, size_t H) {
  Carver c(base);
  ImgState s{};
  const size_t gx = (W + kTile - 1) / kTile, gy = (H + kTile - 1) / kTile;
  s.final_T = c.take<float>(W * H);
  s.n_contrib = c.take<uint32_t>(W * H);
  s.ranges = c.take<uint2>(gx * gy);
  s.tile_last = c.take<uint32_t>(gx * gy);
  s.order = c.take<uint32_t>(gx * gy);
  s.status = c.take<uint32_t>(4);
  s.bytes = c.size();
  return s;
}

// Geometry buffers whose gradient accumulator rows were zeroed by their forward's preprocess
// and not yet used by a backward: the backward skips its memset exactly once per forward (a
// second backward through the same graph, retain_graph=True, clears them itself).
namespace {
std::mutex g_acc_mu;
std::vector<const void*> g_acc_clean;
}  // namespace
void acc_mark_clean(const void* geom) {
  std::lock_guard<std::mutex> l(g_acc_mu);
  for (const void* p : g_acc_clean)
    if (p == geom) return;
  // forwards without a backward (inference) leave entries behind: keep the newest few (a
  // dropped entry only costs its backward a memset)
  if (g_acc_clean.size() >= 64) g_acc_clean.erase(g_acc_clean.begin());
  g_acc_clean.push_back(geom);
}
bool acc_take_clean(const void* geom) {
  std::lock_guard<std::mutex> l(g_acc_mu);
  for (size_t i = 0; i < g_acc_clean.size(); i++)
    if (g_acc_clean[i] == geom) {
      g_acc_clean[i] = g_acc_clean.back();
      g_acc_clean.pop_back();
      return true;
    }
  return false;
}

int tile_schedule_mode() {
  static const int mode = [] {
    const char* e = getenv("GSR_TILE_ORDER");
    if (e && strcmp(e, "natural") == 0) return 0;
    if (e && strcmp(e, "xcd") == 0) return 1;
    return 2;  // heaviest first
  }();
  return mode;
}

}  // namespace gsr

using namespace gsr;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define GSR_CHECK(expr)                                                                     \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(GSR_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    if (debug) {                                                                            \
      e_ = hipStreamSynchronize(stream);                                                    \
      if (e_ == hipSuccess) e_ = hipGetLastError();                                         \
      if (e_ != hipSuccess)                                                                 \
        return fail(GSR_ERR_HIP, "[debug] after %s: %s", #expr, hipGetErrorString(e_));     \
    }                                                                                       \
  } while (0)

// Bits needed to hold tile ids 0 .. ntiles-1 (the reference sorts 32 + getHigherMsb(ntiles)
// bits of a 64-bit key, rasterizer_impl.cu:35-50,300; our tile sort only needs the tile part).
int tile_bits(uint32_t ntiles) {
  if (ntiles <= 1) return 0;
  return 32 - __builtin_clz(ntiles - 1);
}

// host time spent waiting for forwards' instance-count read-backs (gsr_test_host_wait_ms)
std::atomic<long long> g_wait_ns{0};
// tile instances the last forward on this host thread actually binned (gsr_last_forward_instances)
thread_local int g_last_instances = 0;

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ---- per-call forward status (the same-call backstop of the sorts' bounded look-back) -----------
// Each forward gets a mailbox: a pinned, device-mapped word the tile-ranges kernel writes the
// call's status into (kStatus* bits; the forward blend or-s in kStatusClamp), and an event
// recorded after the forward blend.  No copy and no host wait is added to the forward.  The
// backward of the same call checks it on entry without blocking (a status already published fails
// that backward); gsr_forward_status / gsr_check_forwards check with or without waiting.  The
// device side poisons the outputs (NaN) and the gradients of a failed call in any case.
constexpr int kMailSlots = 256;
constexpr uint32_t kMailPending = 0xffffffffu;
struct Mailbox {
  const void* key = nullptr;  // the call's image buffer
  hipEvent_t ev = nullptr;
  int dev = -1;
  bool armed = false;
};
std::mutex g_mail_mu;
Mailbox g_mail[kMailSlots];
volatile uint32_t* g_mail_host = nullptr;
int g_mail_next = 0;
std::string g_mail_lost;  // a failed status found when its slot was recycled unchecked

std::string status_message(uint32_t v) {
  std::string m = "forward status 0x" + std::to_string(v) + ":";
  if (v & kStatusDepthSort) m += " depth-sort look-back timed out;";
  if (v & kStatusTileSort) m += " tile-sort look-back timed out;";
  if (v & kStatusClamp) m += " an out-of-range Gaussian id was clamped;";
  return m + " the call's outputs and gradients are invalid (NaN-poisoned)";
}

// caller holds g_mail_mu; returns the final status if known (0 = fine), kMailPending otherwise
uint32_t mail_read(int i, bool wait) {
  Mailbox& m = g_mail[i];
  if (!m.armed) return 0;
  bool complete = false;
  if (wait) complete = hipEventSynchronize(m.ev) == hipSuccess;
  else complete = hipEventQuery(m.ev) == hipSuccess;
  const uint32_t v = g_mail_host[i];
  if (v != 0 && v != kMailPending) {  // a failure is final as soon as it is published
    m.armed = false;
    return v;
  }
  if (complete) {
    m.armed = false;
    return v == kMailPending ? 0u : v;  // an event that completed always saw the kernel write
  }
  return kMailPending;
}

// Arm a mailbox for the forward on image buffer `key`; returns the device-visible status word
// (null if pinned memory is unavailable: the device-side poison still applies).
uint32_t* mail_post(const void* key, int* slot) {
  std::lock_guard<std::mutex> l(g_mail_mu);
  *slot = -1;
  if (!g_mail_host) {
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(uint32_t) * kMailSlots, hipHostMallocCoherent) != hipSuccess)
      return nullptr;
    g_mail_host = (volatile uint32_t*)p;
    for (int i = 0; i < kMailSlots; i++) g_mail_host[i] = 0;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  // retire an older forward on the same buffer and the slot's previous owner without waiting: a
  // failure they already published is kept for gsr_check_forwards (their outputs and gradients
  // were poisoned on the device either way)
  auto retire = [](int j) {
    const uint32_t v = mail_read(j, false);
    if (v && v != kMailPending && g_mail_lost.empty()) g_mail_lost = status_message(v);
    g_mail[j].armed = false;
  };
  for (int j = 0; j < kMailSlots; j++)
    if (g_mail[j].armed && g_mail[j].key == key) retire(j);
  const int i = g_mail_next;
  g_mail_next = (g_mail_next + 1) % kMailSlots;
  Mailbox& m = g_mail[i];
  if (m.armed) retire(i);
  if (m.ev && m.dev != dev) {
    (void)hipEventDestroy(m.ev);
    m.ev = nullptr;
  }
  if (!m.ev && hipEventCreateWithFlags(&m.ev, hipEventDisableTiming) != hipSuccess) {
    m.ev = nullptr;
    return nullptr;
  }
  m.dev = dev;
  m.key = key;
  g_mail_host[i] = kMailPending;
  *slot = i;
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, (void*)(g_mail_host + i), 0) != hipSuccess) return nullptr;
  return (uint32_t*)dptr;
}

hipError_t mail_arm(int slot, hipStream_t s) {
  if (slot < 0) return hipSuccess;
  std::lock_guard<std::mutex> l(g_mail_mu);
  hipError_t e = hipEventRecord(g_mail[slot].ev, s);
  g_mail[slot].armed = e == hipSuccess;
  return e;
}

// 0 = fine or not yet known (wait = 0); else the failing status
uint32_t mail_check(const void* key, bool wait) {
  std::lock_guard<std::mutex> l(g_mail_mu);
  if (!g_mail_host) return 0;
  for (int i = 0; i < kMailSlots; i++)
    if (g_mail[i].armed && g_mail[i].key == key) {
      const uint32_t v = mail_read(i, wait);
      return v == kMailPending ? 0u : v;
    }
  return 0;
}

// ---- optional per-stage hipEvent timing (include/gsr_testing.h) ----------------------------------
struct Profiler {
  std::mutex mu;
  std::atomic<uint32_t> mask{0};
  std::vector<hipEvent_t> pool;
  struct Rec { int stage; hipEvent_t a, b; };
  std::vector<Rec> pending;
  double ms[GSR_NUM_STAGES] = {0};
  long long calls[GSR_NUM_STAGES] = {0};
};
Profiler& prof() {
  static Profiler p;
  return p;
}
hipEvent_t prof_take() {
  Profiler& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  if (!p.pool.empty()) {
    hipEvent_t e = p.pool.back();
    p.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
hipEvent_t prof_begin(int stage, hipStream_t s) {
  if (!((prof().mask.load(std::memory_order_relaxed) >> stage) & 1u)) return nullptr;
  hipEvent_t a = prof_take();
  if (a && hipEventRecord(a, s) != hipSuccess) return nullptr;
  return a;
}
void prof_end(int stage, hipEvent_t a, hipStream_t s) {
  if (!a) return;
  hipEvent_t b = prof_take();
  if (!b || hipEventRecord(b, s) != hipSuccess) return;
  Profiler& p = prof();
  std::lock_guard<std::mutex> g(p.mu);
  p.pending.push_back({stage, a, b});
}
#define PROF_BEGIN(st) hipEvent_t prof_ev_##st = prof_begin(GSR_STAGE_##st, stream)
#define PROF_END(st) prof_end(GSR_STAGE_##st, prof_ev_##st, stream)

const char* kStageNames[GSR_NUM_STAGES] = {"preprocess", "depth_sort", "scan", "duplicate",
                                          "tile_sort", "ranges", "render_fwd", "acc_zero",
                                          "render_bwd", "preprocess_bwd", "sh_precolor",
                                          "sh_flush"};

}  // namespace

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }

int gsr_last_forward_instances(void) { return g_last_instances; }

int gsr_forward_status(const void* image_buffer, int wait) {
  g_err.clear();
  if (const uint32_t v = mail_check(image_buffer, wait != 0))
    return fail(GSR_ERR_SORT, "%s", status_message(v).c_str());
  return GSR_OK;
}

int gsr_check_forwards(int wait) {
  g_err.clear();
  std::lock_guard<std::mutex> l(g_mail_mu);
  if (!g_mail_lost.empty()) {
    g_err = g_mail_lost;
    g_mail_lost.clear();
    return GSR_ERR_SORT;
  }
  if (!g_mail_host) return GSR_OK;
  uint32_t bad = 0;
  for (int i = 0; i < kMailSlots; i++) {
    const uint32_t v = mail_read(i, wait != 0);
    if (v && v != kMailPending && !bad) bad = v;
  }
  if (bad) return fail(GSR_ERR_SORT, "%s", status_message(bad).c_str());
  return GSR_OK;
}
const char* gsr_last_error(void) { return g_err.c_str(); }

size_t gsr_geom_buffer_bytes(int P) { return carve_geom(nullptr, (size_t)(P > 0 ? P : 0)).bytes; }
size_t gsr_binning_buffer_bytes(int R) {
  return carve_bin(nullptr, (size_t)(R > 0 ? R : 0), false).bytes;
}
size_t gsr_binning_buffer_bytes_det(int R) {
  return carve_bin(nullptr, (size_t)(R > 0 ? R : 0), true).bytes;
}
size_t gsr_image_buffer_bytes(int H, int W) {
  return carve_img(nullptr, (size_t)(W > 0 ? W : 0), (size_t)(H > 0 ? H : 0)).bytes;
}

// ---- forward, in two phases per view ----------------------------------------------------------
// The model side of a forward (shared by every view of a multi-view call).  fused != 0:
// opacities / scales / rotations are GaussianModel's raw _opacity / _scaling / _rotation and the
// SH come split as sh_dc + sh_rest (activations in-kernel).
struct FwdModel {
  int P = 0, M = 0;
  const float *background = nullptr, *means3D = nullptr, *colors_precomp = nullptr;
  const float *opacities = nullptr, *scales = nullptr, *rotations = nullptr;
  float scale_modifier = 1.0f;
  const float *cov3D_precomp = nullptr, *sh = nullptr;
  int degree = 0, prefiltered = 0;
  const float *sh_language = nullptr, *lang_precomp = nullptr, *confidence = nullptr;
  int include_feature = 0, fused = 0;
  const float *sh_dc = nullptr, *sh_rest = nullptr;
  int debug = 0;            // bit 0 only (synchronous checks)
  bool det = false, rows = false;
};
// One camera of a forward, and the state its two phases hand over.
struct FwdCam {
  const float *view = nullptr, *proj = nullptr, *campos = nullptr;
  float tanx = 0, tany = 0;
  int W = 0, H = 0;
  const float* pre_color = nullptr;
  const uint8_t* pre_clamp = nullptr;
  float *out_color = nullptr, *out_depth = nullptr, *out_alpha = nullptr, *out_feature = nullptr;
  int* radii = nullptr;
  gsr_alloc_fn alloc = nullptr;
  void* alloc_ctx = nullptr;
  hipStream_t stream = nullptr;
  uint32_t* host = nullptr;    // pinned landing slot of the read-back
  uint32_t* host_dev = nullptr;  // its device pointer (batched binning: the sum kernel stores it)
  hipEvent_t ready = nullptr;  // recorded after the read-back's copy
  // state of the first phase
  char *gbase = nullptr, *ibase = nullptr, *bbase = nullptr;
  GeomState g{};
  ImgState im{};
  int32_t* radii_ptr = nullptr;
  uint32_t gx = 0, gy = 0;
  bool done = false;  // P == 0: outputs written by the first phase
  bool depth_in_b = false;  // which buffer pair holds the depth sort's result
  bool defer_pre = false;  // fwd_prep leaves the preprocess arguments in pa (not launched)
  // buffers already allocated by the caller (the multi-view call allocates a group's buffers in
  // one callback and carves them), else allocated through `alloc`
  char *given_g = nullptr, *given_i = nullptr, *given_b = nullptr;
  SideClear acc_clear{nullptr, 0};  // accumulator rows the forward blend zeroes (multi-view call)
  PreArgs pa{};
  // state of the binning half of the second phase (fwd_bin -> the blend)
  BinState b{};
  RenderArgs ra{};
  int mail_slot = -1;
  // results
  int num_rendered = 0, num_instances = 0;
};

// Argument checks of the model side (the reference's, rasterize_points.cu:57-59 and
// rasterizer_impl.cu:229-232); `sh` is set to sh_dc on the fused path.
static int fwd_check_model(FwdModel& m) {
  if (m.fused && m.P != 0) {  // P = 0: empty tensors have null data (rasterize_points.cu:81)
    if (!m.sh_dc || (m.M > 1 && !m.sh_rest) || !m.scales || !m.rotations)
      return fail(GSR_ERR_ARGUMENT, "fused path needs features_dc/_rest, _scaling, _rotation");
    m.sh = m.sh_dc;  // "SH present" for the checks below; the kernels read sh_dc / sh_rest
  }
  if (m.P < 0) return fail(GSR_ERR_ARGUMENT, "means3D must have dimensions (num_points, 3)");
  if (m.P == 0) return GSR_OK;
  if (!m.background || !m.means3D || !m.opacities)
    return fail(GSR_ERR_ARGUMENT, "background/means3D/opacities/viewmatrix/projmatrix/campos required");
  if ((m.colors_precomp == nullptr) == (m.sh == nullptr))
    return fail(GSR_ERR_ARGUMENT, "Please provide excatly one of either SHs or precomputed colors!");
  if ((m.cov3D_precomp == nullptr) == (m.scales == nullptr || m.rotations == nullptr))
    return fail(GSR_ERR_ARGUMENT,
                "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  if (m.sh) {
    if (m.degree < 0 || m.degree > 3)
      return fail(GSR_ERR_ARGUMENT, "sh_degree must be in [0, 3] (got %d)", m.degree);
    if (m.M > 16)  // the kernels stage at most 16 coefficients per Gaussian in LDS
      return fail(GSR_ERR_ARGUMENT, "sh has M = %d coefficients; at most 16 (degree 3) supported", m.M);
    if ((m.degree + 1) * (m.degree + 1) > m.M)
      return fail(GSR_ERR_ARGUMENT, "sh has %d coefficients but degree %d needs %d", m.M, m.degree,
                  (m.degree + 1) * (m.degree + 1));
  }
  if (m.rotations && !aligned16(m.rotations))
    return fail(GSR_ERR_ARGUMENT, "rotations must be 16-byte aligned");
  if (scan_parts((size_t)m.P) > (size_t)kScanMaxParts)
    return fail(GSR_ERR_TOO_LARGE, "P = %d exceeds the scan capacity", m.P);
  return GSR_OK;
}

// Phase 1a: the call's buffers and the preprocess launch (its per-workgroup instance counts in
// g.pre_parts).
static int fwd_prep(const FwdModel& m, FwdCam& c) {
  const int debug = m.debug;
  hipStream_t stream = c.stream;
  const int W = c.W, H = c.H, P = m.P;
  if ((c.pre_color == nullptr) != (c.pre_clamp == nullptr) || (c.pre_color && !m.fused))
    return fail(GSR_ERR_ARGUMENT, "pre_color / pre_clamp: both or neither, fused path only");
  if (W <= 0 || H <= 0) return fail(GSR_ERR_ARGUMENT, "image size must be positive (got %dx%d)", W, H);
  if (!c.out_color) return fail(GSR_ERR_ARGUMENT, "out_color / num_rendered missing");
  const size_t HW = (size_t)W * H;
  if (P == 0) {
    c.done = true;
    GSR_CHECK(hipMemsetAsync(c.out_color, 0, 3 * HW * sizeof(float), stream));
    if (c.out_depth) GSR_CHECK(hipMemsetAsync(c.out_depth, 0, HW * sizeof(float), stream));
    if (c.out_alpha) GSR_CHECK(hipMemsetAsync(c.out_alpha, 0, HW * sizeof(float), stream));
    if (c.out_feature) GSR_CHECK(hipMemsetAsync(c.out_feature, 0, 3 * HW * sizeof(float), stream));
    return GSR_OK;
  }
  if (!c.view || !c.proj || !c.campos)
    return fail(GSR_ERR_ARGUMENT, "background/means3D/opacities/viewmatrix/projmatrix/campos required");
  if (!c.alloc) return fail(GSR_ERR_ARGUMENT, "allocator callback missing");
  if (!c.host || !c.ready) return fail(GSR_ERR_HIP, "pinned host slot / event creation failed");
  c.gx = (uint32_t)((W + kTile - 1) / kTile);
  c.gy = (uint32_t)((H + kTile - 1) / kTile);

  const size_t gbytes = carve_geom(nullptr, (size_t)P).bytes;
  c.gbase = c.given_g ? c.given_g : (char*)c.alloc(c.alloc_ctx, gbytes, GSR_BUF_GEOM);
  if (!c.gbase) return fail(GSR_ERR_ALLOC, "geometry buffer allocation of %zu bytes failed", gbytes);
  const size_t ibytes = carve_img(nullptr, (size_t)W, (size_t)H).bytes;
  c.ibase = c.given_i ? c.given_i : (char*)c.alloc(c.alloc_ctx, ibytes, GSR_BUF_IMAGE);
  if (!c.ibase) return fail(GSR_ERR_ALLOC, "image buffer allocation of %zu bytes failed", ibytes);
  c.g = carve_geom(c.gbase, (size_t)P);
  c.im = carve_img(c.ibase, (size_t)W, (size_t)H);
  const GeomState& g = c.g;
  c.radii_ptr = c.radii ? c.radii : g.radii;

  // flags[0] (prefiltered violation) is only written -- and only read back -- when prefiltered
  if (m.prefiltered) GSR_CHECK(hipMemsetAsync(g.flags, 0, 4 * sizeof(uint32_t), stream));
  PreArgs pa{};
  pa.P = P; pa.D = m.degree; pa.M = m.M; pa.W = W; pa.H = H; pa.gx = c.gx; pa.gy = c.gy;
  pa.means3D = m.means3D; pa.scales = m.scales; pa.rotations = m.rotations;
  pa.opacities = m.opacities;
  pa.shs = m.sh; pa.cov3D_precomp = m.cov3D_precomp; pa.colors_precomp = m.colors_precomp;
  pa.sh_language = m.sh_language; pa.lang_precomp = m.lang_precomp;
  pa.confidence = m.confidence;
  pa.view = c.view; pa.proj = c.proj; pa.campos = c.campos;
  pa.scale_modifier = m.scale_modifier; pa.tanx = c.tanx; pa.tany = c.tany;
  pa.fy = (float)H / (2.0f * c.tany);  // rasterizer_impl.cu:222-223
  pa.fx = (float)W / (2.0f * c.tanx);
  pa.prefiltered = m.prefiltered; pa.include_feature = m.include_feature;
  pa.radii = c.radii_ptr; pa.g = g;
  pa.fused = m.fused; pa.sh_dc = m.sh_dc; pa.sh_rest = m.sh_rest;
  pa.pre_color = c.pre_color; pa.pre_clamp = c.pre_clamp;
  // the preprocess grid also zeroes the depth sort's scratch, the look-back scan's status words
  // and (acc_zero) the backward's accumulators
  pa.clear = SideClear{g.sort.aux, (size_t)((char*)(g.ttot + kSortTotTileWords) - (char*)g.sort.aux)};
  pa.acc_zero = m.rows ? 0 : 1;  // the rows layout never reads the accumulator rows
  pa.parts = g.pre_parts;
  if (c.defer_pre) {  // the multi-view call launches the views' preprocesses together
    c.pa = pa;
    return GSR_OK;
  }
  PROF_BEGIN(PREPROCESS);
  GSR_CHECK(launch_preprocess(pa, stream));
  PROF_END(PREPROCESS);
  return GSR_OK;
}

// Phase 1: preprocess, the instance counts' read-back (queued, not waited for), depth sort and
// scan.  Nothing here blocks the host.
static int fwd_begin(const FwdModel& m, FwdCam& c) {
  if (int rc = fwd_prep(m, c)) return rc;
  if (c.done) return GSR_OK;
  const int debug = m.debug;
  hipStream_t stream = c.stream;
  const int P = m.P;
  const GeomState& g = c.g;
  // R = total tile count (order-independent): reduced right after the preprocess and read back
  // while the depth sort and the scan are already queued behind it, so the host's wait and the
  // binning-buffer allocation overlap GPU work instead of draining the stream
  // flags[1] = R
  // flags[2] = the reference's num_rendered: the sum of the full 3-sigma tile rectangles
  // (forward.cu:255, rasterizer_impl.cu:281), returned at the boundary; the binning buffer is
  // carved for that many instances, so a backward handed the reference's count re-carves the
  // same offsets
  const size_t pre_blocks = ((size_t)P + 255) / 256;
  GSR_CHECK(sum_u32_parts(g.pre_parts, pre_blocks, g.flags + 1, stream, g.pre_parts + pre_blocks));
  // one read-back: flags[0] (prefiltered violation), R and the reference's count.  The sorts'
  // look-back timeouts are this call's status (mailbox below), not part of this wait.
  GSR_CHECK(hipMemcpyAsync(c.host, g.flags, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  GSR_CHECK(hipEventRecord(c.ready, stream));

  bool in_b = false;
  PROF_BEGIN(DEPTH_SORT);
  // the last pass writes each Gaussian's tile count in place of its sorted key
  // (planned: the passes of constant digits -- typically the exponent byte -- do not run)
  GSR_CHECK(radix_sort_pairs(g.dkey_a, g.dval_a, g.dkey_b, g.dval_b, (size_t)P, 32,
                             g.sort, &in_b, stream, /*sentinel_anywhere=*/true,
                             /*precleared=*/true, /*key_payload=*/g.tiles_touched, g.dkey_c,
                             g.dval_c));
  PROF_END(DEPTH_SORT);
  c.depth_in_b = in_b;
  const uint32_t* counts_sorted = in_b ? g.dkey_b : g.dkey_a;
  PROF_BEGIN(SCAN);
  GSR_CHECK(scan_u32(counts_sorted, nullptr, g.offsets, (size_t)P, true, g.scan_parts, stream));
  PROF_END(SCAN);
  return GSR_OK;
}

// The read-back's values (already landed in c.host) -> the argument checks of
// rasterizer_impl.cu:281-283 and the binning buffer, carved for the reference's count.
static int fwd_bin_alloc(const FwdModel& m, FwdCam& c, bool tag_by_dup = false) {
  const int debug = m.debug;
  hipStream_t stream = c.stream;
  const GeomState& g = c.g;
  uint32_t* host = c.host;
  const uint32_t R = host[1];       // instances binned: tiles that pass the exact cull
  const uint32_t R_ref = host[2];   // the reference's num_rendered (full rectangles), R <= R_ref
  if (m.prefiltered && host[0]) return fail(GSR_ERR_PREFILTERED,
                           "Point is filtered although prefiltered is set. This shouldn't happen!");
  if (R_ref > 0x7fffffffu || R > R_ref)
    return fail(GSR_ERR_TOO_LARGE, "num_rendered = %u exceeds the sort capacity", R_ref);
  if (debug) {
    GSR_CHECK(hipMemcpyAsync(host + 2, g.sort.aux + kSortAuxErr, 4, hipMemcpyDeviceToHost, stream));
    GSR_CHECK(hipStreamSynchronize(stream));
    if (host[2]) return fail(GSR_ERR_HIP, "depth sort look-back timed out");
  }
  const size_t bbytes = carve_bin(nullptr, R_ref, m.rows).bytes;
  c.bbase = c.given_b ? c.given_b : (char*)c.alloc(c.alloc_ctx, bbytes, GSR_BUF_BINNING);
  if (!c.bbase) return fail(GSR_ERR_ALLOC, "binning buffer allocation of %zu bytes failed", bbytes);
  c.b = carve_bin(c.bbase, R_ref, m.rows);  // capacity R_ref, the first R entries used
  // the layout this forward binned with, for a backward that only holds the buffer (the `_C`
  // signature: GSR_DEBUG_LAYOUT_FROM_BUFFER)
  // (tag_by_dup: the duplicate kernel writes it, no fill launch of its own)
  if (!tag_by_dup)
    GSR_CHECK(hipMemsetD32Async((hipDeviceptr_t)c.b.tag, (int)bin_layout_tag(m.det, m.rows), 1, stream));
  c.num_rendered = (int)R_ref;
  c.num_instances = (int)R;
  return GSR_OK;
}

// The blend's arguments of a binned view (left in c.ra).
static void fwd_render_args(const FwdModel& m, FwdCam& c, const uint32_t* point_list,
                            uint32_t* host_status) {
  const ImgState& im = c.im;
  RenderArgs& ra = c.ra;
  ra.W = c.W; ra.H = c.H; ra.gx = c.gx; ra.gy = c.gy;
  ra.ranges = im.ranges; ra.point_list = point_list; ra.rec = c.g.rec; ra.P = (uint32_t)m.P;
  ra.bg = m.background;
  ra.final_T = im.final_T; ra.n_contrib = im.n_contrib; ra.tile_last = im.tile_last;
  ra.out_color = c.out_color; ra.out_depth = c.out_depth; ra.out_alpha = c.out_alpha;
  ra.out_feature = c.out_feature; ra.include_feature = m.include_feature;
  ra.order = im.order; ra.sched = tile_schedule_mode();
  ra.status = im.status; ra.host_status = host_status; ra.fault = forward_faults_word();
}

// Phase 2a: wait for the read-back (the one host synchronisation of a view, as
// rasterizer_impl.cu:281), then duplicate, tile sort and ranges; the blend's arguments are left in
// c.ra (launched by fwd_end, or with other views' by the multi-view call).
static int fwd_bin(const FwdModel& m, FwdCam& c) {
  if (c.done) {
    c.num_rendered = c.num_instances = 0;
    return GSR_OK;
  }
  int debug = m.debug;
  hipStream_t stream = c.stream;
  const int P = m.P;
  const GeomState& g = c.g;
  const ImgState& im = c.im;
  const uint32_t ntiles = c.gx * c.gy;
  const uint32_t* order = c.depth_in_b ? g.dval_b : g.dval_a;
  {
    const auto t0 = std::chrono::steady_clock::now();
    GSR_CHECK(hipEventSynchronize(c.ready));
    g_wait_ns.fetch_add((long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - t0).count(),
                        std::memory_order_relaxed);
  }
  if (int rc = fwd_bin_alloc(m, c)) return rc;
  const uint32_t R = (uint32_t)c.num_instances;
  const BinState& b = c.b;

  PROF_BEGIN(DUPLICATE);
  // the duplicate grid also zeroes the tile sort's scratch and the tile ranges
  const int tbits = tile_bits(ntiles);
  GSR_CHECK(launch_duplicate(P, order, g.offsets, c.radii_ptr, g.rec, c.gx, c.gy, b.tkey_a, b.tval_a,
                             (uint32_t)R, SideClear{b.sort.aux, sort_clear_bytes(b.sort, R, tbits)},
                             SideClear{im.ranges, sizeof(uint2) * ntiles}, stream,
                             m.rows ? b.egid : nullptr, m.rows ? g.ebeg : nullptr, g.bword));
  PROF_END(DUPLICATE);
  bool t_in_b = false;
  PROF_BEGIN(TILE_SORT);
  GSR_CHECK(radix_sort_pairs(b.tkey_a, b.tval_a, b.tkey_b, b.tval_b, R, tbits, b.sort, &t_in_b,
                             stream, false, /*precleared=*/true));
  PROF_END(TILE_SORT);
  if (debug) {
    uint32_t* host = c.host;
    GSR_CHECK(hipMemcpyAsync(host + 2, b.sort.aux + kSortAuxErr, 4, hipMemcpyDeviceToHost, stream));
    GSR_CHECK(hipStreamSynchronize(stream));
    if (host[2]) return fail(GSR_ERR_HIP, "tile sort look-back timed out");
  }
  const uint32_t* tiles_sorted = t_in_b ? b.tkey_b : b.tkey_a;
  const uint32_t* point_list = t_in_b ? b.tval_b : b.tval_a;
  if (m.rows) {  // the sorted values are emission indices: Gaussian ids into the other value array
    uint32_t* pl = t_in_b ? b.tval_a : b.tval_b;
    GSR_CHECK(launch_det_gather(R, point_list, b.egid, pl, stream));
    point_list = pl;
  }
  int mail_slot = -1;
  uint32_t* host_status = mail_post(c.ibase, &mail_slot);
  PROF_BEGIN(RANGES);
  GSR_CHECK(launch_tile_ranges(R, tiles_sorted, im.ranges, ntiles, g.sort.aux + kSortAuxErr,
                               b.sort.aux + kSortAuxErr, im.status, host_status,
                               forward_faults_word(), stream, /*ranges_cleared=*/true));
  PROF_END(RANGES);

  fwd_render_args(m, c, point_list, host_status);
  c.mail_slot = mail_slot;
  return GSR_OK;
}

// After the view's blend has been issued on `stream`: its mailbox event, the debug check, and the
// accumulator rows marked clean for the backward.
static int fwd_blended(const FwdModel& m, FwdCam& c, hipStream_t stream) {
  if (c.done) return GSR_OK;
  const int debug = m.debug;
  GSR_CHECK(mail_arm(c.mail_slot, stream));
  if (debug) {
    const uint32_t v = mail_check(c.ibase, true);
    if (v) return fail(GSR_ERR_SORT, "%s", status_message(v).c_str());
  }
  if (!m.rows) acc_mark_clean(c.gbase);
  return GSR_OK;
}

// Phase 2 of a single view: binning, then its blend on its own stream.
static int fwd_end(const FwdModel& m, FwdCam& c) {
  if (int rc = fwd_bin(m, c)) return rc;
  if (c.done) return GSR_OK;
  const int debug = m.debug;
  hipStream_t stream = c.stream;
  PROF_BEGIN(RENDER_FWD);
  GSR_CHECK(launch_render_forward(c.ra, stream));
  PROF_END(RENDER_FWD);
  return fwd_blended(m, c, stream);
}

// Pinned read-back slots and their events for the views in flight of one host thread (a
// multi-view call has up to kFwdSlots views between their two phases).
constexpr int kFwdSlots = 64;
static uint32_t* pinned_slot(int i) {
  thread_local uint32_t* p = nullptr;
  if (!p) {
    if (hipHostMalloc((void**)&p, 16 * kFwdSlots, hipHostMallocDefault) != hipSuccess) p = nullptr;
  }
  return p ? p + 4 * i : nullptr;
}
static hipEvent_t readback_event(int i) {
  constexpr int kMaxDev = 64;
  thread_local hipEvent_t ev[kMaxDev][kFwdSlots] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  if (!ev[dev][i] && hipEventCreateWithFlags(&ev[dev][i], hipEventDisableTiming) != hipSuccess)
    ev[dev][i] = nullptr;
  return ev[dev][i];
}

static int forward_impl(int P, int M, const float* background, const float* means3D,
                        const float* colors_precomp, const float* opacities, const float* scales,
                        const float* rotations, float scale_modifier, const float* cov3D_precomp,
                        const float* viewmatrix, const float* projmatrix, float tan_fovx,
                        float tan_fovy, int image_height, int image_width, const float* sh,
                        int degree, const float* campos, int prefiltered, const float* sh_language,
                        const float* language_feature_precomp, const float* confidence,
                        int include_feature, float* out_color, float* out_depth, float* out_alpha,
                        float* out_feature, int* radii, int* num_rendered, gsr_alloc_fn alloc,
                        void* alloc_ctx, void* stream_ptr, int debug, int fused,
                        const float* sh_dc, const float* sh_rest,
                        const float* pre_color = nullptr, const uint8_t* pre_clamp = nullptr) {
  g_err.clear();
  FwdModel m;
  m.det = (debug & GSR_DEBUG_DETERMINISTIC) != 0;  // gsr.h: debug bit 1
  m.rows = m.det;  // per-instance gradient rows (binning layout)
  m.debug = debug & 1;
  m.P = P; m.M = M; m.background = background; m.means3D = means3D;
  m.colors_precomp = colors_precomp; m.opacities = opacities; m.scales = scales;
  m.rotations = rotations; m.scale_modifier = scale_modifier; m.cov3D_precomp = cov3D_precomp;
  m.sh = sh; m.degree = degree; m.prefiltered = prefiltered; m.sh_language = sh_language;
  m.lang_precomp = language_feature_precomp; m.confidence = confidence;
  m.include_feature = include_feature; m.fused = fused; m.sh_dc = sh_dc; m.sh_rest = sh_rest;
  if (!num_rendered || !out_color) return fail(GSR_ERR_ARGUMENT, "out_color / num_rendered missing");
  if (image_width <= 0 || image_height <= 0)
    return fail(GSR_ERR_ARGUMENT, "image size must be positive (got %dx%d)", image_width, image_height);
  if (int rc = fwd_check_model(m)) return rc;
  FwdCam c;
  c.view = viewmatrix; c.proj = projmatrix; c.campos = campos; c.tanx = tan_fovx; c.tany = tan_fovy;
  c.W = image_width; c.H = image_height; c.pre_color = pre_color; c.pre_clamp = pre_clamp;
  c.out_color = out_color; c.out_depth = out_depth; c.out_alpha = out_alpha;
  c.out_feature = out_feature; c.radii = radii; c.alloc = alloc; c.alloc_ctx = alloc_ctx;
  c.stream = (hipStream_t)stream_ptr;
  if (P > 0) {
    c.host = pinned_slot(0);
    c.ready = readback_event(0);
  }
  if (int rc = fwd_begin(m, c)) return rc;
  if (int rc = fwd_end(m, c)) return rc;
  *num_rendered = c.num_rendered;
  g_last_instances = c.num_instances;
  return GSR_OK;
}

int gsr_rasterize_gaussians(int P, int M, const float* background, const float* means3D,
                            const float* colors_precomp, const float* opacities,
                            const float* scales, const float* rotations, float scale_modifier,
                            const float* cov3D_precomp, const float* viewmatrix,
                            const float* projmatrix, float tan_fovx, float tan_fovy,
                            int image_height, int image_width, const float* sh, int degree,
                            const float* campos, int prefiltered, const float* sh_language,
                            const float* language_feature_precomp, const float* confidence,
                            int include_feature, float* out_color, float* out_depth,
                            float* out_alpha, float* out_feature, int* radii, int* num_rendered,
                            gsr_alloc_fn alloc, void* alloc_ctx, void* stream_ptr, int debug) {
  return forward_impl(P, M, background, means3D, colors_precomp, opacities, scales, rotations,
                      scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                      image_height, image_width, sh, degree, campos, prefiltered, sh_language,
                      language_feature_precomp, confidence, include_feature, out_color, out_depth,
                      out_alpha, out_feature, radii, num_rendered, alloc, alloc_ctx, stream_ptr,
                      debug, 0, nullptr, nullptr);
}

int gsr_rasterize_gaussians_fused(int P, int M, const float* background, const float* means3D,
                                  const float* features_dc, const float* features_rest,
                                  const float* opacity_raw, const float* scaling_raw,
                                  const float* rotation_raw, float scale_modifier,
                                  const float* viewmatrix, const float* projmatrix, float tan_fovx,
                                  float tan_fovy, int image_height, int image_width, int degree,
                                  const float* campos, int prefiltered,
                                  const float* language_feature, const float* confidence,
                                  int include_feature, float* out_color, float* out_depth,
                                  float* out_alpha, float* out_feature, int* radii,
                                  int* num_rendered, gsr_alloc_fn alloc, void* alloc_ctx,
                                  void* stream_ptr, int debug) {
  return forward_impl(P, M, background, means3D, nullptr, opacity_raw, scaling_raw, rotation_raw,
                      scale_modifier, nullptr, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                      image_height, image_width, nullptr, degree, campos, prefiltered,
                      language_feature, nullptr, confidence, include_feature, out_color, out_depth,
                      out_alpha, out_feature, radii, num_rendered, alloc, alloc_ctx, stream_ptr,
                      debug, 1, features_dc, features_rest);
}

int gsr_rasterize_gaussians_fused_precolor(
    int P, int M, const float* background, const float* means3D, const float* features_dc,
    const float* features_rest, const float* opacity_raw, const float* scaling_raw,
    const float* rotation_raw, float scale_modifier, const float* viewmatrix,
    const float* projmatrix, float tan_fovx, float tan_fovy, int image_height, int image_width,
    int degree, const float* campos, int prefiltered, const float* language_feature,
    const float* confidence, int include_feature, const float* pre_color,
    const uint8_t* pre_clamp, float* out_color, float* out_depth, float* out_alpha,
    float* out_feature, int* radii, int* num_rendered, gsr_alloc_fn alloc, void* alloc_ctx,
    void* stream_ptr, int debug) {
  return forward_impl(P, M, background, means3D, nullptr, opacity_raw, scaling_raw, rotation_raw,
                      scale_modifier, nullptr, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                      image_height, image_width, nullptr, degree, campos, prefiltered,
                      language_feature, nullptr, confidence, include_feature, out_color, out_depth,
                      out_alpha, out_feature, radii, num_rendered, alloc, alloc_ctx, stream_ptr,
                      debug, 1, features_dc, features_rest, pre_color, pre_clamp);
}

// ---- backward, in two parts per view ----------------------------------------------------------
// The blend part (accumulator zeroing + backward blend) and the per-Gaussian part (backward
// preprocess) of one view's backward, with their launch arguments.
struct BwdCall {
  bool done = false;       // P == 0: nothing to do
  bool blend = false;      // R > 0
  bool acc_zero = false;   // the accumulator rows were not zeroed by this buffer's forward
  float* acc = nullptr;
  size_t P = 0;
  int debug = 0;
  RenderBwdArgs rb{};
  BwdPreArgs ba{};
};

static int bwd_setup(
    BwdCall& call, int P, int M, int R, const float* background, const float* means3D, const int* radii,
    const float* colors_precomp, const float* scales, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, float tan_fovx,
    float tan_fovy, int image_height, int image_width, const float* dL_dout_color,
    const float* dL_dout_depth, const float* dL_dout_alpha, const float* dL_dout_feature,
    const float* sh, int degree, const float* campos, const float* sh_language,
    const float* language_feature_precomp, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer, float* dL_dmeans2D,
    float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
    float* dL_dscales, float* dL_drotations, float* dL_dsh_language, float* dL_dlanguage_feature,
    int debug, int fused, const float* sh_dc, const float* sh_rest,
    const float* opacity_raw, float* dL_dsh_rest, int accumulate, float* dRGB_sh,
    const float* pre_jac, bool sh_in_views = false) {
  const bool det = (debug & GSR_DEBUG_DETERMINISTIC) != 0;  // must match the forward's flags
  const bool rows = det;
  debug &= 1;
  call.debug = debug;
  if (fused && P != 0) {
    if (!sh_dc || (M > 1 && !sh_rest) || (M > 1 && !dL_dsh_rest && !dRGB_sh) || !scales ||
        !rotations || !opacity_raw)
      return fail(GSR_ERR_ARGUMENT, "fused backward needs the raw parameters and their grads");
    sh = sh_dc;
  } else if (dRGB_sh) {
    return fail(GSR_ERR_ARGUMENT, "deferred SH gradients are a fused-path mode");
  }
  // pre_jac without dL_dcolor_sh: the multi-view call forms the SH gradients in its per-Gaussian
  // launch (gsr.h gsr_view.pre_jac); a single-view call needs the deferred dL/dRGB plane
  if (pre_jac && !dRGB_sh && !sh_in_views)
    return fail(GSR_ERR_ARGUMENT, "pre_jac needs the deferred SH gradients (dL_dcolor_sh)");
  const int W = image_width, H = image_height;
  if (P < 0 || R < 0 || W <= 0 || H <= 0) return fail(GSR_ERR_ARGUMENT, "invalid sizes");
  if (P == 0) {
    call.done = true;
    return GSR_OK;
  }
  if (!geom_buffer || !image_buffer || (R > 0 && !binning_buffer))
    return fail(GSR_ERR_ARGUMENT, "forward scratch buffers missing");
  // the forward of these buffers failed and has already said so (no wait; the device side
  // poisons the gradients whether or not the host has seen the status yet)
  if (const uint32_t v = mail_check(image_buffer, debug != 0))
    return fail(GSR_ERR_SORT, "%s", status_message(v).c_str());
  if (!dL_dout_color || !dL_dmeans2D || !dL_dopacity || !dL_dmeans3D)
    return fail(GSR_ERR_ARGUMENT, "required gradient buffers missing");
  if (sh && !dL_dsh && !dRGB_sh) return fail(GSR_ERR_ARGUMENT, "dL_dsh required when sh is given");
  if (scales && (!dL_dscales || !dL_drotations || !rotations))
    return fail(GSR_ERR_ARGUMENT, "dL_dscales / dL_drotations required when scales are given");
  if ((rotations && !aligned16(rotations)) || (dL_drotations && !aligned16(dL_drotations)))
    return fail(GSR_ERR_ARGUMENT, "rotations / dL_drotations must be 16-byte aligned");
  if (sh && (degree < 0 || degree > 3 || (degree + 1) * (degree + 1) > M))
    return fail(GSR_ERR_ARGUMENT, "invalid sh degree %d for M = %d", degree, M);
  if (sh && M > 16)  // the backward stages at most 16 coefficients per Gaussian in LDS
    return fail(GSR_ERR_ARGUMENT, "sh has M = %d coefficients; at most 16 (degree 3) supported", M);
  if (dL_dsh_language && !sh_language && !language_feature_precomp && include_feature)
    ;  // nothing to differentiate: zeros are written

  const uint32_t gx = (uint32_t)((W + kTile - 1) / kTile), gy = (uint32_t)((H + kTile - 1) / kTile);
  const uint32_t ntiles = gx * gy;
  GeomState g = carve_geom((char*)geom_buffer, (size_t)P);
  ImgState im = carve_img((char*)image_buffer, (size_t)W, (size_t)H);
  BinState b = carve_bin((char*)binning_buffer, (size_t)R, rows);
  const int passes = sort_passes(tile_bits(ntiles));
  const uint32_t* point_list = (passes & 1) ? b.tval_b : b.tval_a;
  const uint32_t* einst = nullptr;
  if (rows) {  // forward: emission indices sorted in place, Gaussian ids gathered into the other
    einst = point_list;
    point_list = (passes & 1) ? b.tval_a : b.tval_b;
  }
  const int32_t* radii_ptr = radii ? radii : g.radii;

  call.P = (size_t)P;
  call.acc = g.acc;
  call.acc_zero = !rows && !acc_take_clean(geom_buffer);  // not freshly zeroed by its forward
  call.blend = R > 0;
  RenderBwdArgs& rb = call.rb;
  rb.W = W; rb.H = H; rb.gx = gx; rb.gy = gy;
  rb.ranges = im.ranges; rb.point_list = point_list; rb.rec = g.rec; rb.P = (uint32_t)P; rb.bg = background;
  rb.final_T = im.final_T; rb.n_contrib = im.n_contrib; rb.tile_last = im.tile_last;
  rb.dL_dcolor = dL_dout_color; rb.dL_ddepth = dL_dout_depth; rb.dL_dalpha = dL_dout_alpha;
  rb.dL_dfeature = dL_dout_feature; rb.acc = g.acc; rb.include_feature = include_feature;
  rb.order = im.order; rb.sched = tile_schedule_mode();
  rb.einst = einst; rb.partial = rows ? b.partial : nullptr; rb.det = det ? 1 : 0;
  rb.nrows = (uint32_t)R; rb.status = im.status;
  BwdPreArgs& ba = call.ba;
  ba.P = P; ba.D = degree; ba.M = M;
  ba.means3D = means3D; ba.scales = scales; ba.rotations = rotations; ba.shs = sh;
  ba.cov3D = cov3D_precomp; ba.colors_precomp = colors_precomp;
  ba.sh_language = sh_language; ba.lang_precomp = language_feature_precomp;
  ba.confidence = confidence;
  ba.view = viewmatrix; ba.proj = projmatrix; ba.campos = campos;
  ba.scale_modifier = scale_modifier; ba.tanx = tan_fovx; ba.tany = tan_fovy;
  ba.fy = (float)H / (2.0f * tan_fovy);  // rasterizer_impl.cu:380-381
  ba.fx = (float)W / (2.0f * tan_fovx);
  ba.include_feature = include_feature;
  ba.radii = radii_ptr; ba.clamped = g.clamped; ba.acc = g.acc;
  ba.dL_dmeans2D = dL_dmeans2D; ba.dL_dcolors = dL_dcolors; ba.dL_dopacity = dL_dopacity;
  ba.dL_dmeans3D = dL_dmeans3D; ba.dL_dcov3D = dL_dcov3D; ba.dL_dsh = sh ? dL_dsh : nullptr;
  ba.dL_dscales = scales ? dL_dscales : nullptr; ba.dL_drotations = scales ? dL_drotations : nullptr;
  ba.dL_dsh_language = dL_dsh_language; ba.dL_dlanguage_feature = dL_dlanguage_feature;
  ba.fused = fused; ba.accumulate = accumulate; ba.sh_dc = sh_dc; ba.sh_rest = sh_rest;
  ba.opacities_raw = opacity_raw; ba.dL_dsh_rest = dL_dsh_rest;
  ba.dRGB_out = dRGB_sh;
  ba.pre_jac = pre_jac;
  ba.status = im.status;
  // rows layout: each Gaussian sums its instances' rows (emission order, contiguous) itself
  ba.use_rows = rows ? 1 : 0;
  ba.rows = R > 0 && rows ? reinterpret_cast<const float4*>(b.partial) : nullptr;
  ba.ebeg = g.ebeg; ba.count = g.tiles_touched;
  if (dRGB_sh) ba.dL_dsh = ba.dL_dsh_rest = nullptr;
  return GSR_OK;
}

// accumulator zeroing (when needed) + the backward blend
static int bwd_blend(const BwdCall& call, hipStream_t stream) {
  const int debug = call.debug;
  if (call.done) return GSR_OK;
  if (call.acc_zero) {
    PROF_BEGIN(ACC_ZERO);
    GSR_CHECK(hipMemsetAsync(call.acc, 0, sizeof(float) * kAccFloats * call.P, stream));
    PROF_END(ACC_ZERO);
  }
  if (call.blend) {
    PROF_BEGIN(RENDER_BWD);
    GSR_CHECK(launch_render_backward(call.rb, stream));
    PROF_END(RENDER_BWD);
  }
  return GSR_OK;
}

// the fused per-Gaussian backward (computeCov2DCUDA + preprocessCUDA backward + activations)
static int bwd_pre(const BwdCall& call, hipStream_t stream) {
  const int debug = call.debug;
  if (call.done) return GSR_OK;
  PROF_BEGIN(PREPROCESS_BWD);
  GSR_CHECK(launch_preprocess_backward(call.ba, stream));
  PROF_END(PREPROCESS_BWD);
  return GSR_OK;
}

static int backward_impl(
    int P, int M, int R, const float* background, const float* means3D, const int* radii,
    const float* colors_precomp, const float* scales, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, float tan_fovx,
    float tan_fovy, int image_height, int image_width, const float* dL_dout_color,
    const float* dL_dout_depth, const float* dL_dout_alpha, const float* dL_dout_feature,
    const float* sh, int degree, const float* campos, const float* sh_language,
    const float* language_feature_precomp, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer, float* dL_dmeans2D,
    float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
    float* dL_dscales, float* dL_drotations, float* dL_dsh_language, float* dL_dlanguage_feature,
    void* stream_ptr, int debug, int fused, const float* sh_dc, const float* sh_rest,
    const float* opacity_raw, float* dL_dsh_rest, int accumulate, float* dRGB_sh = nullptr,
    const float* pre_jac = nullptr) {
  g_err.clear();
  if (debug & GSR_DEBUG_LAYOUT_FROM_BUFFER) {
    debug &= ~GSR_DEBUG_LAYOUT_FROM_BUFFER;
    if (R > 0 && binning_buffer) {
      // the caller holds only the buffers (the reference's `_C` signature): the forward wrote its
      // layout into the binning buffer's tag word -- one synchronous 4-byte read
      uint32_t tag = 0;
      const BinState hb = carve_bin((char*)binning_buffer, 0, false);
      hipStream_t stream = (hipStream_t)stream_ptr;
      GSR_CHECK(hipMemcpyAsync(&tag, hb.tag, sizeof(tag), hipMemcpyDeviceToHost, stream));
      GSR_CHECK(hipStreamSynchronize(stream));
      const bool det = (tag & 2u) != 0;
      if ((tag & ~3u) != kBinLayoutMagic || ((tag & 1u) != 0) != det)
        return fail(GSR_ERR_ARGUMENT, "binningBuffer does not come from a libgsr forward of this "
                                      "process (layout tag 0x%08x)", tag);
      debug = (debug & ~GSR_DEBUG_DETERMINISTIC) | (det ? GSR_DEBUG_DETERMINISTIC : 0);
    }
  }
  BwdCall call;
  if (int rc = bwd_setup(call, P, M, R, background, means3D, radii, colors_precomp, scales,
                         rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                         tan_fovx, tan_fovy, image_height, image_width, dL_dout_color,
                         dL_dout_depth, dL_dout_alpha, dL_dout_feature, sh, degree, campos,
                         sh_language, language_feature_precomp, confidence, include_feature,
                         geom_buffer, binning_buffer, image_buffer, dL_dmeans2D, dL_dcolors,
                         dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations,
                         dL_dsh_language, dL_dlanguage_feature, debug, fused, sh_dc, sh_rest,
                         opacity_raw, dL_dsh_rest, accumulate, dRGB_sh, pre_jac))
    return rc;
  hipStream_t stream = (hipStream_t)stream_ptr;
  if (int rc = bwd_blend(call, stream)) return rc;
  return bwd_pre(call, stream);
}

int gsr_rasterize_gaussians_backward(
    int P, int M, int R, const float* background, const float* means3D, const int* radii,
    const float* colors_precomp, const float* scales, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, float tan_fovx,
    float tan_fovy, int image_height, int image_width, const float* dL_dout_color,
    const float* dL_dout_depth, const float* dL_dout_alpha, const float* dL_dout_feature,
    const float* sh, int degree, const float* campos, const float* sh_language,
    const float* language_feature_precomp, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer, float* dL_dmeans2D,
    float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
    float* dL_dscales, float* dL_drotations, float* dL_dsh_language, float* dL_dlanguage_feature,
    void* stream_ptr, int debug) {
  return backward_impl(P, M, R, background, means3D, radii, colors_precomp, scales, rotations,
                       scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                       image_height, image_width, dL_dout_color, dL_dout_depth, dL_dout_alpha,
                       dL_dout_feature, sh, degree, campos, sh_language, language_feature_precomp,
                       confidence, include_feature, geom_buffer, binning_buffer, image_buffer,
                       dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh,
                       dL_dscales, dL_drotations, dL_dsh_language, dL_dlanguage_feature, stream_ptr,
                       debug, 0, nullptr, nullptr, nullptr, nullptr, 0);
}

int gsr_rasterize_gaussians_fused_backward(
    int P, int M, int R, const float* background, const float* means3D, const int* radii,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    const float* viewmatrix, const float* projmatrix, float tan_fovx, float tan_fovy,
    int image_height, int image_width, const float* dL_dout_color, const float* dL_dout_depth,
    const float* dL_dout_alpha, const float* dL_dout_feature, int degree, const float* campos,
    const float* language_feature, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer, float* dL_dmeans2D,
    float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest, float* dL_dopacity_raw,
    float* dL_dscaling_raw, float* dL_drotation_raw, float* dL_dlanguage_feature, int accumulate,
    void* stream_ptr, int debug) {
  return gsr_rasterize_gaussians_fused_backward_deferred(
      P, M, R, background, means3D, radii, features_dc, features_rest, opacity_raw, scaling_raw,
      rotation_raw, scale_modifier, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
      image_width, dL_dout_color, dL_dout_depth, dL_dout_alpha, dL_dout_feature, degree, campos,
      language_feature, confidence, include_feature, geom_buffer, binning_buffer, image_buffer,
      dL_dmeans2D, dL_dmeans3D, dL_dfeatures_dc, dL_dfeatures_rest, dL_dopacity_raw,
      dL_dscaling_raw, dL_drotation_raw, dL_dlanguage_feature, nullptr, nullptr, accumulate,
      stream_ptr, debug);
}

int gsr_rasterize_gaussians_fused_backward_deferred(
    int P, int M, int R, const float* background, const float* means3D, const int* radii,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    const float* viewmatrix, const float* projmatrix, float tan_fovx, float tan_fovy,
    int image_height, int image_width, const float* dL_dout_color, const float* dL_dout_depth,
    const float* dL_dout_alpha, const float* dL_dout_feature, int degree, const float* campos,
    const float* language_feature, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer, float* dL_dmeans2D,
    float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest, float* dL_dopacity_raw,
    float* dL_dscaling_raw, float* dL_drotation_raw, float* dL_dlanguage_feature,
    float* dL_dcolor_sh, const float* pre_jac, int accumulate, void* stream_ptr, int debug) {
  return backward_impl(P, M, R, background, means3D, radii, nullptr, scaling_raw, rotation_raw,
                       scale_modifier, nullptr, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                       image_height, image_width, dL_dout_color, dL_dout_depth, dL_dout_alpha,
                       dL_dout_feature, nullptr, degree, campos, language_feature, nullptr,
                       confidence, include_feature, geom_buffer, binning_buffer, image_buffer,
                       dL_dmeans2D, nullptr, dL_dopacity_raw, dL_dmeans3D, nullptr,
                       dL_dfeatures_dc, dL_dscaling_raw, dL_drotation_raw, dL_dlanguage_feature,
                       nullptr, stream_ptr, debug, 1, features_dc, features_rest, opacity_raw,
                       dL_dfeatures_rest, accumulate, dL_dcolor_sh, pre_jac);
}

// ---- multi-view calls --------------------------------------------------------------------------
namespace {
// per host thread: events joining the views' streams with the call's stream
hipEvent_t join_event(int i) {
  constexpr int kMaxDev = 64;
  thread_local hipEvent_t ev[kMaxDev][kFwdSlots + 1] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  // stream-to-stream ordering only: a device-scope release, no system fence (no host reads)
  if (!ev[dev][i] &&
      hipEventCreateWithFlags(&ev[dev][i], hipEventDisableTiming | hipEventDisableSystemFence) !=
          hipSuccess)
    ev[dev][i] = nullptr;
  return ev[dev][i];
}

// Coherent, device-mapped pinned words (4 per view) that the batched sums store each view's
// read-back into: no copy launch, one event per group.
uint32_t* batch_slot(int i, uint32_t** dev_ptr) {
  constexpr int kMaxDev = 64;
  thread_local uint32_t* host[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  if (!host[dev]) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 16 * kFwdSlots, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      return nullptr;
    host[dev] = (uint32_t*)p;
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host[dev] + 4 * i, 0) != hipSuccess) return nullptr;
  *dev_ptr = (uint32_t*)d;
  return host[dev] + 4 * i;
}

// debug builds of the batched path: a sort's look-back error word, synchronously
int check_sort_err(const uint32_t* err, hipStream_t stream, const char* what) {
  const int debug = 1;
  uint32_t v = 0;
  GSR_CHECK(hipMemcpyAsync(&v, err, 4, hipMemcpyDeviceToHost, stream));
  GSR_CHECK(hipStreamSynchronize(stream));
  if (v) return fail(GSR_ERR_HIP, "%s look-back timed out", what);
  return GSR_OK;
}

// Batched binning.  The views are split into `ng` groups, group g on the g-th distinct view
// stream (group 0 on the call's stream, so its preprocess follows the caller's last kernel -- the
// colour pre-pass -- on the same queue without a cross-stream wait); inside a group every stage
// after the preprocess is ONE launch for all the group's views -- the preprocesses, the
// instance-count sums (which also store the read-back into pinned words), each depth-sort pass,
// the scan, the duplication, each tile-sort pass, the ranges, the schedules and the blend.  A
// view's binning alone is a chain of ~14 small launches whose latency, not HBM, sets its time
// (0.20 ms per view at 1 stream); batched, each launch is as wide as the group.  Every kernel sees
// exactly its one-view arguments (own totals, tickets, look-back words), so the results are
// bit-identical to the per-view path.  The host waits once per group, for its read-back, while the
// group's depth sort and scan run; group g's blend then overlaps group g + 1's binning on the other
// stream.  Each group's first phase is queued before the first wait.  The views' backward
// accumulator rows are zeroed by the forward blend's grid (a VALU-bound kernel) instead of the
// memory-bound preprocess's.
int views_forward_batched(const FwdModel& m, std::vector<FwdCam>& cams, gsr_view* views,
                          hipStream_t call_stream, int ng) {
  const int V = (int)cams.size();
  const int debug = m.debug;
  if (V == 0) return GSR_OK;
  std::vector<hipStream_t> distinct;
  for (const FwdCam& c : cams)
    if (std::find(distinct.begin(), distinct.end(), c.stream) == distinct.end())
      distinct.push_back(c.stream);
  if (ng < 1) ng = 1;
  int per = (V + ng - 1) / ng;
  if (per > kMaxBatchViews) per = kMaxBatchViews;
  ng = (V + per - 1) / per;
  struct Group {
    int v0 = 0, n = 0;
    hipStream_t st = nullptr;
    hipEvent_t ready = nullptr;
    std::vector<int> live;  // views with P > 0
    bool depth_in_b = false;
    RenderArgs ras[kMaxBatchViews];  // the binned views' blend arguments (phase 2a -> 2b)
  };
  std::vector<Group> grp((size_t)ng);
  const int P = m.P;
  const size_t pre_blocks = ((size_t)P + 255) / 256;
  // every view's geometry and image buffer in ONE allocation callback (carved per view; the
  // first view's allocation holds them all, so the caller keeps every view's scratch alive as
  // before): a callback into the caller's allocator costs ~10-20 us of host time
  if (P > 0 && cams[0].alloc) {
    const size_t gb = carve_geom(nullptr, (size_t)P).bytes;
    const size_t ib = carve_img(nullptr, (size_t)cams[0].W, (size_t)cams[0].H).bytes;
    char* base = (char*)cams[0].alloc(cams[0].alloc_ctx, (size_t)V * (gb + ib), GSR_BUF_GEOM);
    if (!base) return fail(GSR_ERR_ALLOC, "scratch allocation of %zu bytes failed", (size_t)V * (gb + ib));
    for (int v = 0; v < V; v++) {
      cams[(size_t)v].given_g = base + (size_t)v * (gb + ib);
      cams[(size_t)v].given_i = cams[(size_t)v].given_g + gb;
    }
  }
  // phase 1 of a group: the views' preprocesses in one launch, then one launch per stage
  auto phase1 = [&](int gi) -> int {
    Group& G = grp[(size_t)gi];
    G.v0 = (int)((long long)gi * per);
    G.n = std::min(per, V - G.v0);
    G.st = gi == 0 ? call_stream : distinct[(size_t)(gi - 1) % distinct.size()];
    G.ready = readback_event(gi);
    if (!G.ready) return fail(GSR_ERR_HIP, "event creation failed");
    hipStream_t stream = G.st;
    SumSpec sums[kMaxBatchViews];
    SortSpec ds[kMaxBatchViews];
    PreArgs pas[kMaxBatchViews];
    for (int k = 0; k < G.n; k++) {
      const int v = G.v0 + k;
      FwdCam& c = cams[(size_t)v];
      c.stream = G.st;
      c.host = batch_slot(v, &c.host_dev);
      if (!c.host) return fail(GSR_ERR_HIP, "pinned read-back slot unavailable");
      c.ready = G.ready;
      c.defer_pre = true;
      if (int rc = fwd_prep(m, c)) return rc;
      if (c.done) continue;
      const GeomState& g = c.g;
      const int l = (int)G.live.size();
      pas[l] = c.pa;
      if (pas[l].acc_zero) {
        pas[l].acc_zero = 0;  // the view's forward blend zeroes the accumulator rows instead
        c.acc_clear = SideClear{g.acc, (size_t)P * kAccFloats * sizeof(float)};
      }
      sums[l] = SumSpec{g.pre_parts, g.pre_parts + pre_blocks, pre_blocks, g.flags + 1, c.host_dev,
                        m.prefiltered ? g.flags : nullptr};
      ds[l] = SortSpec{g.dkey_a, g.dval_a, g.dkey_b, g.dval_b, (size_t)P, g.sort, g.tiles_touched,
                       g.dkey_c, g.dval_c};
      // The tile counts ride in the depth sort's values when id and count fit 32 bits (20 + 12 at
      // 1008x756 and P <= 2^20): the last pass splits them instead of gathering tiles_touched by
      // id -- one random 4-B read per Gaussian, ~2x that pass's time.  Same sorted pairs.
      const uint32_t cbits = 32u - (uint32_t)__builtin_clz(c.gx * c.gy | 1u);  // counts <= tiles
      if (cbits < 32u && (uint64_t)P <= (1ull << (32u - cbits))) {
        pas[l].vpack = 32u - cbits;
        ds[l].key_payload = nullptr;
        ds[l].vsplit = (int)(32u - cbits);
      }
      G.live.push_back(v);
    }
    const int nl = (int)G.live.size();
    if (nl == 0) return GSR_OK;
    PROF_BEGIN(PREPROCESS);
    GSR_CHECK(launch_preprocess_views(pas, nl, stream));
    PROF_END(PREPROCESS);
    // the read-back sums ride in the depth sort's digit-totals launch (one launch fewer in the
    // chain); the read-back event follows that launch
    PROF_BEGIN(DEPTH_SORT);
    GSR_CHECK(radix_sort_pairs_views(ds, nl, 32, &G.depth_in_b, stream, /*sentinel_anywhere=*/true,
                                     /*precleared=*/true, sums, G.ready));
    PROF_END(DEPTH_SORT);
    ScanSpec sc[kMaxBatchViews];
    for (int l = 0; l < nl; l++) {
      FwdCam& c = cams[(size_t)G.live[(size_t)l]];
      c.depth_in_b = G.depth_in_b;
      const uint32_t* counts = G.depth_in_b ? c.g.dkey_b : c.g.dkey_a;
      sc[l] = ScanSpec{counts, c.g.offsets, (size_t)P, c.g.scan_parts};
    }
    PROF_BEGIN(SCAN);
    GSR_CHECK(scan_u32_views(sc, nl, true, stream));
    PROF_END(SCAN);
    return GSR_OK;
  };
  // phase 2a of a group: its read-back, then its binning (the blend's arguments left in G.ras)
  auto phase2a = [&](int gi) -> int {
    Group& G = grp[(size_t)gi];
    RenderArgs* ras = G.ras;
    hipStream_t stream = G.st;
    const int nl = (int)G.live.size();
    if (nl == 0) return GSR_OK;
    {
      const auto t0 = std::chrono::steady_clock::now();
      GSR_CHECK(hipEventSynchronize(G.ready));
      g_wait_ns.fetch_add((long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count(),
                          std::memory_order_relaxed);
    }
    DupSpec dup[kMaxBatchViews];
    SortSpec ts[kMaxBatchViews];
    const uint32_t ntiles = cams[(size_t)G.live[0]].gx * cams[(size_t)G.live[0]].gy;
    const int tbits = tile_bits(ntiles);
    // Keys-only tile sort when tile id and Gaussian id fit one 32-bit key (tile << pack | gid:
    // 12 + 20 bits at 1008x756 and P <= 2^20): the duplication writes 4 B per instance instead of
    // 8, every pass but the last moves 4 B instead of 8 each way, and the last pass writes the
    // same (tile, gid) pairs the pair sort does -- a stable sort on the tile bits keeps each
    // tile's depth order, so the result is bit-identical.  The deterministic rows path sorts
    // instance indices (egid) and keeps the pair sort.
    // (one tile, tbits = 0: no tile sort at all, plain pairs)
    const uint32_t pack = (!m.rows && tbits > 0 && tbits <= 16 &&
                           (uint64_t)P <= (1ull << (32 - tbits)))
                              ? (uint32_t)(32 - tbits)
                              : 0u;
    {  // the group's binning buffers in one allocation callback (sizes from the read-back)
      size_t off[kMaxBatchViews + 1] = {0};
      for (int l = 0; l < nl; l++) {
        const uint32_t R_ref = cams[(size_t)G.live[(size_t)l]].host[2];
        const size_t bb = R_ref <= 0x7fffffffu ? carve_bin(nullptr, R_ref, m.rows).bytes : 0;
        off[l + 1] = off[l] + bb;  // (an invalid count is reported by fwd_bin_alloc)
      }
      FwdCam& c0 = cams[(size_t)G.live[0]];
      char* base = (char*)c0.alloc(c0.alloc_ctx, off[nl] ? off[nl] : 256, GSR_BUF_BINNING);
      if (!base) return fail(GSR_ERR_ALLOC, "binning buffer allocation of %zu bytes failed", off[nl]);
      for (int l = 0; l < nl; l++) cams[(size_t)G.live[(size_t)l]].given_b = base + off[l];
    }
    for (int l = 0; l < nl; l++) {
      FwdCam& c = cams[(size_t)G.live[(size_t)l]];
      if (int rc = fwd_bin_alloc(m, c, /*tag_by_dup=*/true)) return rc;  // (debug: checks the depth sort)
      const GeomState& g = c.g;
      const BinState& b = c.b;
      const uint32_t R = (uint32_t)c.num_instances;
      dup[l] = DupSpec{P, G.depth_in_b ? g.dval_b : g.dval_a, g.offsets, g.rec, c.gx, c.gy,
                       b.tkey_a, b.tval_a, R,
                       SideClear{b.sort.aux, sort_clear_bytes(b.sort, R, tbits)},
                       SideClear{c.im.ranges, sizeof(uint2) * ntiles},
                       m.rows ? b.egid : nullptr, m.rows ? g.ebeg : nullptr, b.tag,
                       bin_layout_tag(m.det, m.rows), pack, g.bword};
      ts[l] = SortSpec{b.tkey_a, b.tval_a, b.tkey_b, b.tval_b, (size_t)R, b.sort, nullptr};
      ts[l].lo = (int)pack;
      if (tbits > 0 && tbits <= 16) {  // the tile sort's digit totals counted by the duplication (no totals launch)
        dup[l].ttot = g.ttot;
        dup[l].tbits = tbits;
        ts[l].totals = g.ttot;
      }
    }
    PROF_BEGIN(DUPLICATE);
    GSR_CHECK(launch_duplicate_views(dup, nl, stream));
    PROF_END(DUPLICATE);
    bool t_in_b = false;
    PROF_BEGIN(TILE_SORT);
    GSR_CHECK(radix_sort_pairs_views(ts, nl, tbits, &t_in_b, stream, false, /*precleared=*/true));
    PROF_END(TILE_SORT);
    RangesSpec rs[kMaxBatchViews];
    for (int l = 0; l < nl; l++) {
      FwdCam& c = cams[(size_t)G.live[(size_t)l]];
      const BinState& b = c.b;
      const uint32_t R = (uint32_t)c.num_instances;
      if (debug)
        if (int rc = check_sort_err(b.sort.aux + kSortAuxErr, stream, "tile sort")) return rc;
      const uint32_t* tiles_sorted = t_in_b ? b.tkey_b : b.tkey_a;
      const uint32_t* point_list = t_in_b ? b.tval_b : b.tval_a;
      if (m.rows) {
        uint32_t* pl = t_in_b ? b.tval_a : b.tval_b;
        GSR_CHECK(launch_det_gather(R, point_list, b.egid, pl, stream));
        point_list = pl;
      }
      int mail_slot = -1;
      uint32_t* host_status = mail_post(c.ibase, &mail_slot);
      rs[l] = RangesSpec{R, tiles_sorted, c.im.ranges, ntiles, c.g.sort.aux + kSortAuxErr,
                         b.sort.aux + kSortAuxErr, c.im.status, host_status,
                         forward_faults_word()};
      fwd_render_args(m, c, point_list, host_status);
      c.ra.clear = c.acc_clear;
      c.mail_slot = mail_slot;
      ras[l] = c.ra;
    }
    PROF_BEGIN(RANGES);
    GSR_CHECK(launch_tile_ranges_views(rs, nl, stream));
    GSR_CHECK(launch_render_schedule_views(ras, nl, stream));
    PROF_END(RANGES);
    return GSR_OK;
  };
  // phase 2b of a group: its blend on the group's stream, which then joins the call's stream.
  // The join comes right after the blend and before the views' mailbox events: those carry a
  // system-scope release (the host reads the status words), each a drain and L2 write-back that
  // would otherwise sit between the blend and the backward waiting on it.  Round 5
  // (profiles/r05_stream_gaps.txt): blending every group on the call's stream instead measured
  // slower (the groups' blends no longer overlap, and the mailbox events then sit in-stream).
  auto phase2b = [&](int gi) -> int {
    Group& G = grp[(size_t)gi];
    const int nl = (int)G.live.size();
    hipStream_t stream = G.st;
    if (nl > 0) {
      PROF_BEGIN(RENDER_FWD);
      GSR_CHECK(launch_render_forward_views(G.ras, nl, stream));
      PROF_END(RENDER_FWD);
    }
    if (G.st != call_stream) {
      hipEvent_t e = join_event(gi);
      if (!e || hipEventRecord(e, G.st) != hipSuccess ||
          hipStreamWaitEvent(call_stream, e, 0) != hipSuccess)
        return fail(GSR_ERR_HIP, "joining group %d's stream failed", gi);
    }
    for (int k = 0; k < G.n; k++) {
      const int v = G.v0 + k;
      FwdCam& c = cams[(size_t)v];
      if (c.done) c.num_rendered = c.num_instances = 0;
      if (int rc = fwd_blended(m, c, stream)) return rc;
      gsr_view& out = views[v];
      out.geom_buffer = c.gbase; out.binning_buffer = c.bbase; out.image_buffer = c.ibase;
      out.num_rendered = c.num_rendered; out.num_instances = c.num_instances;
    }
    return GSR_OK;
  };
  // Round 4 (profiles/r04_pipeline_ab.txt): every group's binning before the blends measured
  // slower than binning + blend per group -- the later group's binning then overlaps the earlier
  // group's blend (a full-chip launch) instead of running beside the other latency-bound binning
  for (int gi = 0; gi < ng; gi++)
    if (int rc = phase1(gi)) return rc;
  for (int gi = 0; gi < ng; gi++) {
    if (int rc = phase2a(gi)) return rc;
    if (int rc = phase2b(gi)) return rc;
  }
  g_last_instances = cams[(size_t)V - 1].num_instances;
  return GSR_OK;
}
}  // namespace

int gsr_rasterize_views_fused(int V, gsr_view* views, int image_height, int image_width, int P,
                              int M, const float* background, const float* means3D,
                              const float* features_dc, const float* features_rest,
                              const float* opacity_raw, const float* scaling_raw,
                              const float* rotation_raw, float scale_modifier, int degree,
                              int prefiltered, const float* language_feature,
                              const float* confidence, int include_feature, gsr_alloc_fn alloc,
                              int inflight, void* stream_ptr, int debug) {
  g_err.clear();
  if (V < 0 || V > kFwdSlots) return fail(GSR_ERR_ARGUMENT, "V = %d views: 0 .. %d supported", V, kFwdSlots);
  if (V > 0 && !views) return fail(GSR_ERR_ARGUMENT, "views missing");
  if (image_width <= 0 || image_height <= 0)
    return fail(GSR_ERR_ARGUMENT, "image size must be positive (got %dx%d)", image_width, image_height);
  FwdModel m;
  m.det = (debug & GSR_DEBUG_DETERMINISTIC) != 0;
  m.rows = m.det;
  m.debug = debug & 1;
  m.P = P; m.M = M; m.background = background; m.means3D = means3D;
  m.opacities = opacity_raw; m.scales = scaling_raw; m.rotations = rotation_raw;
  m.scale_modifier = scale_modifier; m.degree = degree; m.prefiltered = prefiltered;
  m.sh_language = language_feature; m.confidence = confidence;
  m.include_feature = include_feature; m.fused = 1; m.sh_dc = features_dc; m.sh_rest = features_rest;
  if (int rc = fwd_check_model(m)) return rc;
  hipStream_t call_stream = (hipStream_t)stream_ptr;
  std::vector<FwdCam> cams((size_t)V);
  for (int v = 0; v < V; v++) {
    const gsr_view& in = views[v];
    FwdCam& c = cams[(size_t)v];
    c.view = in.viewmatrix; c.proj = in.projmatrix; c.campos = in.campos;
    c.tanx = in.tan_fovx; c.tany = in.tan_fovy; c.W = image_width; c.H = image_height;
    c.pre_color = in.pre_color; c.pre_clamp = in.pre_clamp;
    c.out_color = in.out_color; c.out_depth = in.out_depth; c.out_alpha = in.out_alpha;
    c.out_feature = in.out_feature; c.radii = in.radii;
    c.alloc = alloc; c.alloc_ctx = in.alloc_ctx;
    c.stream = in.stream ? (hipStream_t)in.stream : call_stream;
  }
  // the views' streams start after the call's stream (inputs prepared there)
  hipEvent_t start = join_event(kFwdSlots);
  if (!start || hipEventRecord(start, call_stream) != hipSuccess)
    return fail(GSR_ERR_HIP, "event record on the call's stream failed");
  for (int v = 0; v < V; v++) {  // once per distinct stream
    hipStream_t s = cams[(size_t)v].stream;
    bool seen = s == call_stream;
    for (int u = 0; u < v && !seen; u++) seen = cams[(size_t)u].stream == s;
    if (!seen && hipStreamWaitEvent(s, start, 0) != hipSuccess)
      return fail(GSR_ERR_HIP, "stream wait failed");
  }
  (void)inflight;  // one group in flight per distinct view stream
  // two groups: group 1's binning overlaps group 0's blend
  return views_forward_batched(m, cams, views, call_stream, 2);
}

int gsr_rasterize_views_fused_backward(
    int V, const gsr_view* views, int image_height, int image_width, int P, int M,
    const float* background, const float* means3D, const float* features_dc,
    const float* features_rest, const float* opacity_raw, const float* scaling_raw,
    const float* rotation_raw, float scale_modifier, int degree, const float* language_feature,
    const float* confidence, int include_feature, float* dL_dmeans3D, float* dL_dfeatures_dc,
    float* dL_dfeatures_rest, float* dL_dopacity_raw, float* dL_dscaling_raw,
    float* dL_drotation_raw, float* dL_dlanguage_feature, int accumulate, void* stream_ptr,
    int debug) {
  return gsr_rasterize_views_fused_backward_sliced(
      V, views, image_height, image_width, P, M, background, means3D, features_dc, features_rest,
      opacity_raw, scaling_raw, rotation_raw, scale_modifier, degree, language_feature,
      confidence, include_feature, dL_dmeans3D, dL_dfeatures_dc, dL_dfeatures_rest,
      dL_dopacity_raw, dL_dscaling_raw, dL_drotation_raw, dL_dlanguage_feature, accumulate,
      stream_ptr, debug, 0, nullptr, nullptr);
}

int gsr_rasterize_views_fused_backward_sliced(
    int V, const gsr_view* views, int image_height, int image_width, int P, int M,
    const float* background, const float* means3D, const float* features_dc,
    const float* features_rest, const float* opacity_raw, const float* scaling_raw,
    const float* rotation_raw, float scale_modifier, int degree, const float* language_feature,
    const float* confidence, int include_feature, float* dL_dmeans3D, float* dL_dfeatures_dc,
    float* dL_dfeatures_rest, float* dL_dopacity_raw, float* dL_dscaling_raw,
    float* dL_drotation_raw, float* dL_dlanguage_feature, int accumulate, void* stream_ptr,
    int debug, int slice_rows, gsr_rows_fn on_rows, void* rows_ctx) {
  g_err.clear();
  if (slice_rows < 0 || (slice_rows % 256) != 0)
    return fail(GSR_ERR_ARGUMENT, "slice_rows = %d: a multiple of 256 (0 = one slice)", slice_rows);
  if (V < 0 || V > kFwdSlots) return fail(GSR_ERR_ARGUMENT, "V = %d views: 0 .. %d supported", V, kFwdSlots);
  if (V > 0 && !views) return fail(GSR_ERR_ARGUMENT, "views missing");
  hipStream_t call_stream = (hipStream_t)stream_ptr;
  std::vector<BwdCall> calls((size_t)V);
  for (int v = 0; v < V; v++) {
    const gsr_view& w = views[v];
    if (int rc = bwd_setup(calls[(size_t)v], P, M, w.num_rendered, background, means3D, w.radii,
                           nullptr, scaling_raw, rotation_raw, scale_modifier, nullptr,
                           w.viewmatrix, w.projmatrix, w.tan_fovx, w.tan_fovy, image_height,
                           image_width, w.dL_dout_color, w.dL_dout_depth, w.dL_dout_alpha,
                           w.dL_dout_feature, nullptr, degree, w.campos, language_feature,
                           nullptr, confidence, include_feature, w.geom_buffer,
                           w.binning_buffer, w.image_buffer, w.dL_dmeans2D, nullptr,
                           dL_dopacity_raw, dL_dmeans3D, nullptr, dL_dfeatures_dc,
                           dL_dscaling_raw, dL_drotation_raw, dL_dlanguage_feature, nullptr,
                           debug, 1, features_dc, features_rest, opacity_raw, dL_dfeatures_rest,
                           (v > 0 || accumulate) ? 1 : 0, w.dL_dcolor_sh, w.pre_jac,
                           /*sh_in_views=*/true))
      return rc;
  }
  // SH gradients formed by the per-Gaussian launch itself (every view with pre_jac and without
  // dL_dcolor_sh): all views in one launch, no per-view fallback
  int sh_in = 0;
  for (int v = 0; v < V; v++) sh_in += (views[v].pre_jac && !views[v].dL_dcolor_sh) ? 1 : 0;
  if (sh_in != 0 && (sh_in != V || V > kMaxBwdViews || (debug & GSR_DEBUG_TEST_PER_VIEW_PRE)))
    return fail(GSR_ERR_ARGUMENT, "SH gradients formed in the multi-view backward (pre_jac without "
                                  "dL_dcolor_sh) need it in every view and at most %d views",
                kMaxBwdViews);
  if (V == 0) {
    if (on_rows && P > 0) on_rows(rows_ctx, 0, P);
    return GSR_OK;
  }
  // The backward blends of all views run merged into launches of up to kMaxBwdViews views (one
  // launch's tiles are its views' tiles, so no per-view tail of idle CUs); the per-Gaussian parts
  // read-modify-write the leaves' gradients and run in view order on the call's stream, each
  // after the launch holding its view.  One launch: the blend runs on the call's stream too
  // (nothing to overlap it with); several: on views[0].stream, beside the previous launch's
  // per-Gaussian backward.
  const int per = V < kMaxBwdViews ? V : kMaxBwdViews;
  hipStream_t bs = (views[0].stream && per < V) ? (hipStream_t)views[0].stream : call_stream;
  hipEvent_t start = join_event(kFwdSlots);  // the upstream gradients were produced on the call's stream
  if (bs != call_stream) {
    if (!start || hipEventRecord(start, call_stream) != hipSuccess)
      return fail(GSR_ERR_HIP, "event record on the call's stream failed");
    if (hipStreamWaitEvent(bs, start, 0) != hipSuccess) return fail(GSR_ERR_HIP, "stream wait failed");
  }
  const int debug_sync = debug & 1;
  const bool no_blend = (debug & GSR_DEBUG_TEST_NO_BLEND) != 0;
  const bool per_view_pre = (debug & GSR_DEBUG_TEST_PER_VIEW_PRE) != 0;
  for (int v0 = 0; v0 < V; v0 += per) {
    const int n = V - v0 < per ? V - v0 : per;
    RenderBwdArgs rbs[kMaxBwdViews];
    int nb = 0;
    for (int k = 0; k < n; k++) {
      BwdCall& c = calls[(size_t)(v0 + k)];
      if (c.done || no_blend) continue;
      if (c.acc_zero) {
        BwdCall z = c;
        z.blend = false;  // the accumulator memset only
        if (int rc = bwd_blend(z, bs)) return rc;
      }
      if (c.blend) rbs[nb++] = c.rb;
    }
    if (nb > 0) {
      const int debug = debug_sync;
      hipStream_t stream = bs;
      PROF_BEGIN(RENDER_BWD);
      GSR_CHECK(launch_render_backward_views(rbs, nb, bs));
      PROF_END(RENDER_BWD);
    }
    hipEvent_t e = join_event(v0);
    if (bs != call_stream) {
      if (!e || hipEventRecord(e, bs) != hipSuccess ||
          hipStreamWaitEvent(call_stream, e, 0) != hipSuccess)
        return fail(GSR_ERR_HIP, "joining the blend stream failed");
    }
    // the chunk's per-Gaussian backwards: one launch for all of them where the configuration
    // allows (launch_preprocess_backward_views), else one per view
    BwdPreArgs bas[kMaxBwdViews];
    int np = 0;
    for (int k = 0; k < n; k++)
      if (!calls[(size_t)(v0 + k)].done) bas[np++] = calls[(size_t)(v0 + k)].ba;
    hipError_t ve = hipErrorNotSupported;
    // the last chunk's per-Gaussian backward finishes the leaves' gradients: in row slices, each
    // handed to on_rows as soon as it is enqueued (gsr.h: a multi-GPU caller all-reduces the
    // slice while the next one computes)
    const bool last = v0 + per >= V;
    const uint32_t step = (last && on_rows && slice_rows > 0) ? (uint32_t)slice_rows : (uint32_t)P;
    // one view takes the multi-view launch too when it forms the SH gradients (no per-view
    // kernel does); np == 0 (P == 0, every call done) falls through to the no-op per-view path
    if ((np > 1 || (np == 1 && sh_in)) && !per_view_pre) {
      const int debug = debug_sync;
      hipStream_t stream = call_stream;
      PROF_BEGIN(PREPROCESS_BWD);
      for (uint32_t r0 = 0; r0 < (uint32_t)P; r0 += step) {
        ve = launch_preprocess_backward_views(bas, np, call_stream, r0, r0 + step);
        if (ve != hipSuccess) break;
        if (last && on_rows && step < (uint32_t)P) on_rows(rows_ctx, (int)r0, (int)std::min(r0 + step, (uint32_t)P));
      }
      if (ve != hipSuccess && ve != hipErrorNotSupported)
        return fail(GSR_ERR_HIP, "launch_preprocess_backward_views: %s", hipGetErrorString(ve));
      if (ve == hipSuccess) {
        PROF_END(PREPROCESS_BWD);
        if (debug) GSR_CHECK(hipStreamSynchronize(stream));
        if (last && on_rows && step >= (uint32_t)P) on_rows(rows_ctx, 0, P);
      }
    }
    if (ve == hipErrorNotSupported && sh_in && np > 0)
      return fail(GSR_ERR_ARGUMENT, "SH gradients formed in the multi-view backward: this "
                                    "configuration has no multi-view per-Gaussian launch");
    if (ve == hipErrorNotSupported) {
      (void)hipGetLastError();
      for (int k = 0; k < n; k++)
        if (int rc = bwd_pre(calls[(size_t)(v0 + k)], call_stream)) return rc;
      if (last && on_rows) on_rows(rows_ctx, 0, P);
    }
  }
  return GSR_OK;
}

int gsr_sh_precolor(int P, int M, int degree, const float* means3D, const float* features_dc,
                    const float* features_rest, int nviews, const float* const* campos,
                    float* const* color, uint8_t* const* clamped, float* const* jac,
                    void* stream_ptr) {
  return gsr_sh_precolor_rows(P, 0, P, M, degree, means3D, features_dc, features_rest, nviews,
                              campos, color, clamped, jac, stream_ptr);
}

int gsr_sh_precolor_rows(int P, int row0, int row1, int M, int degree, const float* means3D,
                         const float* features_dc, const float* features_rest, int nviews,
                         const float* const* campos, float* const* color,
                         uint8_t* const* clamped, float* const* jac, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (P < 0 || nviews < 0) return fail(GSR_ERR_ARGUMENT, "invalid sizes");
  if (row0 < 0 || row1 < row0 || row1 > P)
    return fail(GSR_ERR_ARGUMENT, "rows [%d, %d) outside [0, %d)", row0, row1, P);
  if (P == 0 || nviews == 0 || row1 == row0) return GSR_OK;
  if (M < 1 || M > 16 || degree < 0 || degree > 3 || (degree + 1) * (degree + 1) > M)
    return fail(GSR_ERR_ARGUMENT, "invalid sh degree %d for M = %d", degree, M);
  if (!means3D || !features_dc || (M > 1 && !features_rest) || !campos)
    return fail(GSR_ERR_ARGUMENT, "null pointer");
  // either part may be left out: color + clamped both NULL (the Jacobian only) or jac NULL (the
  // colour only), e.g. the colour ahead of the forward and the Jacobian on another stream
  const bool want_col = color || clamped, want_jac = jac != nullptr;
  if ((color == nullptr) != (clamped == nullptr) || !(want_col || want_jac))
    return fail(GSR_ERR_ARGUMENT, "color and clamped go together, and one part is needed");
  for (int v0 = 0; v0 < nviews; v0 += kShFlushMaxViewsFwd) {
    PrecolorArgs a{};
    a.P = P; a.M = M; a.D = degree; a.means3D = means3D; a.sh_dc = features_dc;
    a.row0 = (uint32_t)row0; a.row1 = (uint32_t)row1;
    a.sh_rest = features_rest;
    a.nviews = nviews - v0 < kShFlushMaxViewsFwd ? nviews - v0 : kShFlushMaxViewsFwd;
    for (int v = 0; v < a.nviews; v++) {
      if (!campos[v0 + v] || (want_col && (!color[v0 + v] || !clamped[v0 + v])) ||
          (want_jac && !jac[v0 + v]))
        return fail(GSR_ERR_ARGUMENT, "null view pointer");
      a.campos[v] = campos[v0 + v];
      a.color[v] = want_col ? color[v0 + v] : nullptr;
      a.clamp[v] = want_col ? clamped[v0 + v] : nullptr;
      a.jac[v] = want_jac ? jac[v0 + v] : nullptr;
    }
    PROF_BEGIN(SH_PRECOLOR);
    GSR_CHECK(launch_sh_precolor(a, stream));
    PROF_END(SH_PRECOLOR);
  }
  return GSR_OK;
}

int gsr_sh_grad_flush(int P, int M, int degree, const float* means3D, int nviews,
                      const float* const* campos, const float* const* dL_dcolor_sh,
                      int64_t rgb_plane_stride, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
                      int accumulate, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (P < 0 || nviews < 0) return fail(GSR_ERR_ARGUMENT, "invalid sizes");
  if (P == 0 || nviews == 0) return GSR_OK;
  if (M < 1 || M > 16 || degree < 0 || degree > 3 || (degree + 1) * (degree + 1) > M)
    return fail(GSR_ERR_ARGUMENT, "invalid sh degree %d for M = %d", degree, M);
  if (!means3D || !campos || !dL_dcolor_sh || !dL_dfeatures_dc || (M > 1 && !dL_dfeatures_rest))
    return fail(GSR_ERR_ARGUMENT, "null pointer");
  if (rgb_plane_stride < P) return fail(GSR_ERR_ARGUMENT, "rgb_plane_stride < P");
  for (int v0 = 0; v0 < nviews; v0 += kShFlushMaxViews) {
    ShFlushArgs a{};
    a.P = P; a.M = M; a.D = degree; a.means3D = means3D;
    a.nviews = nviews - v0 < kShFlushMaxViews ? nviews - v0 : kShFlushMaxViews;
    a.accumulate = (v0 > 0 || accumulate) ? 1 : 0;
    a.rgb_stride = (size_t)rgb_plane_stride;
    for (int v = 0; v < a.nviews; v++) {
      if (!campos[v0 + v] || !dL_dcolor_sh[v0 + v]) return fail(GSR_ERR_ARGUMENT, "null view pointer");
      a.campos[v] = campos[v0 + v];
      a.dRGB[v] = dL_dcolor_sh[v0 + v];
    }
    a.dL_dsh_dc = dL_dfeatures_dc; a.dL_dsh_rest = dL_dfeatures_rest;
    PROF_BEGIN(SH_FLUSH);
    GSR_CHECK(launch_sh_grad_flush(a, stream));
    PROF_END(SH_FLUSH);
  }
  return GSR_OK;
}

// ---- test hooks (include/gsr_testing.h) -----------------------------------------------------------
static size_t sort_scratch_layout(char* base, size_t n, uint32_t** kb, uint32_t** vb,
                                  SortScratch* sc, uint32_t** kc = nullptr,
                                  uint32_t** vc = nullptr) {
  Carver c(base);
  uint32_t* a = c.take<uint32_t>(n);
  uint32_t* b = c.take<uint32_t>(n);
  uint32_t* a2 = c.take<uint32_t>(n);  // the planned sort's third pair
  uint32_t* b2 = c.take<uint32_t>(n);
  SortScratch s = take_sort_scratch(c, n);
  if (kb) *kb = a;
  if (vb) *vb = b;
  if (kc) *kc = a2;
  if (vc) *vc = b2;
  if (sc) *sc = s;
  return c.size();
}

size_t gsr_test_sort_scratch_bytes(size_t n) {
  return sort_scratch_layout(nullptr, n, nullptr, nullptr, nullptr);
}

static int test_radix_sort(uint32_t* keys, uint32_t* vals, size_t n, int bits, void* scratch,
                           void* stream_ptr, bool sentinel_anywhere, bool planned = false);

int gsr_test_radix_sort_pairs(uint32_t* keys, uint32_t* vals, size_t n, int bits, void* scratch,
                              void* stream_ptr) {
  return test_radix_sort(keys, vals, n, bits, scratch, stream_ptr, false);
}

int gsr_test_radix_sort_pairs_sentinel(uint32_t* keys, uint32_t* vals, size_t n, int bits,
                                       void* scratch, void* stream_ptr) {
  return test_radix_sort(keys, vals, n, bits, scratch, stream_ptr, true);
}

int gsr_test_radix_sort_pairs_planned(uint32_t* keys, uint32_t* vals, size_t n, int bits,
                                      int sentinel_anywhere, void* scratch, void* stream_ptr) {
  return test_radix_sort(keys, vals, n, bits, scratch, stream_ptr, sentinel_anywhere != 0, true);
}

static int test_radix_sort(uint32_t* keys, uint32_t* vals, size_t n, int bits, void* scratch,
                           void* stream_ptr, bool sentinel_anywhere, bool planned) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (n == 0) return GSR_OK;
  if (!keys || !vals || !scratch || bits < 0 || bits > 32) return fail(GSR_ERR_ARGUMENT, "bad args");
  if (n > 0xffffffffull) return fail(GSR_ERR_TOO_LARGE, "n too large");
  uint32_t *kb, *vb, *kc, *vc;
  SortScratch sc;
  sort_scratch_layout((char*)scratch, n, &kb, &vb, &sc, &kc, &vc);
  bool in_b = false;
  GSR_CHECK(radix_sort_pairs(keys, vals, kb, vb, n, bits, sc, &in_b, stream, sentinel_anywhere,
                             false, nullptr, planned ? kc : nullptr, planned ? vc : nullptr));
  uint32_t* host = pinned_slot(0);
  if (!host) return fail(GSR_ERR_HIP, "pinned host allocation failed");
  GSR_CHECK(hipMemcpyAsync(host + 2, sc.aux + kSortAuxErr, 4, hipMemcpyDeviceToHost, stream));
  GSR_CHECK(hipStreamSynchronize(stream));
  if (host[2]) return fail(GSR_ERR_HIP, "radix sort look-back timed out");
  if (in_b) {
    GSR_CHECK(hipMemcpyAsync(keys, kb, n * 4, hipMemcpyDeviceToDevice, stream));
    GSR_CHECK(hipMemcpyAsync(vals, vb, n * 4, hipMemcpyDeviceToDevice, stream));
  }
  return GSR_OK;
}

size_t gsr_test_scan_scratch_bytes(size_t n) { return align_up((scan_parts(n) + 1) * 4); }

int gsr_test_scan(const uint32_t* in, uint32_t* out, size_t n, int inclusive, void* scratch,
                  void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (n == 0) return GSR_OK;
  if (scan_parts(n) > (size_t)kScanMaxParts) return fail(GSR_ERR_TOO_LARGE, "n too large");
  GSR_CHECK(scan_u32(in, nullptr, out, n, inclusive != 0, (uint32_t*)scratch, stream));
  return GSR_OK;
}

// look-back scan of `views` independent arrays in one launch (in/out: views x n u32, back to
// back); scratch: views x gsr_test_scan_lookback_words(n) u64 words, zeroed here
size_t gsr_test_scan_lookback_words(size_t n) { return scan_lb_words(n); }

int gsr_test_scan_lookback(const uint32_t* in, uint32_t* out, size_t n, int views, void* scratch,
                           void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (n == 0 || views <= 0) return GSR_OK;
  if (views > kMaxBatchViews || n > 0xffffffffull) return fail(GSR_ERR_ARGUMENT, "bad sizes");
  uint32_t* err = pinned_slot(0);
  if (!err) return fail(GSR_ERR_HIP, "pinned host allocation failed");
  uint64_t* st = (uint64_t*)scratch;
  const size_t words = scan_lb_words(n);
  // error word after the status words of every view
  uint32_t* derr = (uint32_t*)(st + (size_t)views * words);
  GSR_CHECK(hipMemsetAsync(scratch, 0, (size_t)views * words * 8 + 16, stream));
  ScanLbSpec sp[kMaxBatchViews];
  for (int k = 0; k < views; k++)
    sp[k] = ScanLbSpec{in + (size_t)k * n, out + (size_t)k * n, n, st + (size_t)k * words, derr};
  GSR_CHECK(scan_u32_lookback_views(sp, views, stream));
  GSR_CHECK(hipMemcpyAsync(err, derr, 4, hipMemcpyDeviceToHost, stream));
  GSR_CHECK(hipStreamSynchronize(stream));
  if (*err) return fail(GSR_ERR_HIP, "scan look-back timed out");
  return GSR_OK;
}

int gsr_test_expf_pair(const float* x, float* ref, float* fast, size_t n, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (n && (!x || !ref || !fast)) return fail(GSR_ERR_ARGUMENT, "null pointer");
  GSR_CHECK(launch_expf_pair(x, ref, fast, n, stream));
  return GSR_OK;
}

int gsr_test_activations(const float* opacity_raw, const float* scaling_raw,
                         const float* rotation_raw, size_t P, float* opacity, float* scaling,
                         float* rotation, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (P && (!opacity_raw || !scaling_raw || !rotation_raw || !opacity || !scaling || !rotation))
    return fail(GSR_ERR_ARGUMENT, "null pointer");
  if (!aligned16(rotation_raw) || !aligned16(rotation))
    return fail(GSR_ERR_ARGUMENT, "rotations must be 16-byte aligned");
  GSR_CHECK(launch_activations(opacity_raw, scaling_raw, rotation_raw, P, opacity, scaling,
                               rotation, stream));
  return GSR_OK;
}

int gsr_test_binning_lists(const void* binning_buffer, const void* image_buffer, int num_rendered,
                           int image_height, int image_width, int flags, int n_instances,
                           uint32_t* point_list_out, uint32_t* ranges_out, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (num_rendered < 0 || n_instances < 0 || n_instances > num_rendered || image_height <= 0 ||
      image_width <= 0 || !image_buffer || !ranges_out ||
      (n_instances && (!binning_buffer || !point_list_out)))
    return fail(GSR_ERR_ARGUMENT, "invalid arguments");
  const bool rows = (flags & GSR_DEBUG_DETERMINISTIC) != 0;
  const uint32_t gx = (uint32_t)((image_width + kTile - 1) / kTile);
  const uint32_t gy = (uint32_t)((image_height + kTile - 1) / kTile);
  const ImgState im = carve_img((char*)image_buffer, (size_t)image_width, (size_t)image_height);
  GSR_CHECK(hipMemcpyAsync(ranges_out, im.ranges, sizeof(uint2) * gx * gy, hipMemcpyDeviceToHost,
                           stream));
  if (n_instances) {
    // the backward's own carve (backward_impl): same layout, same ping-pong parity
    const BinState b = carve_bin((char*)binning_buffer, (size_t)num_rendered, rows);
    const int passes = sort_passes(tile_bits(gx * gy));
    const uint32_t* pl = (passes & 1) ? b.tval_b : b.tval_a;
    if (rows) pl = (passes & 1) ? b.tval_a : b.tval_b;
    GSR_CHECK(hipMemcpyAsync(point_list_out, pl, sizeof(uint32_t) * (size_t)n_instances,
                             hipMemcpyDeviceToHost, stream));
  }
  GSR_CHECK(hipStreamSynchronize(stream));
  return GSR_OK;
}

int gsr_test_splat_records(const void* geom_buffer, int P, float* rec_out, void* stream_ptr) {
  g_err.clear();
  hipStream_t stream = (hipStream_t)stream_ptr;
  const int debug = 0;
  if (P < 0 || (P > 0 && (!geom_buffer || !rec_out))) return fail(GSR_ERR_ARGUMENT, "invalid arguments");
  if (P == 0) return GSR_OK;
  const GeomState g = carve_geom((char*)geom_buffer, (size_t)P);
  GSR_CHECK(hipMemcpyAsync(rec_out, g.rec, sizeof(float) * kRecFloats * (size_t)P,
                           hipMemcpyDeviceToHost, stream));
  GSR_CHECK(hipStreamSynchronize(stream));
  return GSR_OK;
}

void gsr_profile_enable(int stage_mask) { prof().mask.store((uint32_t)stage_mask); }

int gsr_profile_collect(double* ms, long long* calls) {
  Profiler& p = prof();
  std::vector<Profiler::Rec> recs;
  {
    std::lock_guard<std::mutex> g(p.mu);
    recs.swap(p.pending);
  }
  int rc = GSR_OK;
  for (auto& r : recs) {
    float t = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
      p.ms[r.stage] += t;
      p.calls[r.stage] += 1;
    } else {
      rc = fail(GSR_ERR_HIP, "event timing failed");
    }
  }
  std::lock_guard<std::mutex> g(p.mu);
  for (auto& r : recs) { p.pool.push_back(r.a); p.pool.push_back(r.b); }
  for (int i = 0; i < GSR_NUM_STAGES; i++) {
    if (ms) ms[i] = p.ms[i];
    if (calls) calls[i] = p.calls[i];
  }
  return rc;
}

void gsr_profile_reset(void) {
  Profiler& p = prof();
  gsr_profile_collect(nullptr, nullptr);
  std::lock_guard<std::mutex> g(p.mu);
  for (int i = 0; i < GSR_NUM_STAGES; i++) { p.ms[i] = 0; p.calls[i] = 0; }
}

const char* gsr_profile_stage_name(int stage) {
  return (stage >= 0 && stage < GSR_NUM_STAGES) ? kStageNames[stage] : "";
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream_ptr) {
  g_err.clear();
  (void)projmatrix;  // in_frustum projects but only tests view-space z (auxiliary.h:149-154)
  if (P < 0) return fail(GSR_ERR_ARGUMENT, "means3D must have dimensions (num_points, 3)");
  if (P == 0) return GSR_OK;
  if (!means3D || !viewmatrix || !present) return fail(GSR_ERR_ARGUMENT, "null pointer");
  hipError_t e = launch_mark_visible(P, means3D, viewmatrix, present, (hipStream_t)stream_ptr);
  if (e != hipSuccess) return fail(GSR_ERR_HIP, "mark_visible launch failed: %s", hipGetErrorString(e));
  return GSR_OK;
}

}  // extern "C"

extern "C" double gsr_test_host_wait_ms(int reset) {
  const long long ns = reset ? g_wait_ns.exchange(0) : g_wait_ns.load();
  return (double)ns * 1e-6;
}

// gsr_internal.h -- private buffer layouts and kernel launchers of libgsr (not part of the C-ABI).
//
// The three scratch byte buffers play the role of the reference's GeometryState / BinningState /
// ImageState (cuda_rasterizer/rasterizer_impl.h:21-73, rasterizer_impl.cu:155-194): the forward
// carves them, Python keeps them alive in the autograd context, and the backward re-carves the
// same offsets from the same bytes.  The layout itself is ours (a per-splat 64-byte record packed
// for the tile gather, a depth-first two-stage sort, per-splat gradient accumulators).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gsr {

constexpr int kTile = 16;                 // config.h:16-17 (BLOCK_X = BLOCK_Y = 16)
constexpr int kTilePix = kTile * kTile;   // 256 pixels = 4 waves of 64 lanes
constexpr size_t kAlign = 256;
constexpr int kRecFloats = 16;        // 4 x float4 splat record (see gsr_preprocess.hip)
constexpr int kAccFloats = 16;        // per-splat gradient accumulator row (64 B)
// Accumulator slots (one 64-byte row per Gaussian, filled by the backward blend)
enum AccSlot : int {
  kAccMx = 0, kAccMy = 1,                 // dL/dmean2D (NDC-scaled, backward.cu:545-546)
  kAccCa = 2, kAccCb = 3, kAccCc = 4,     // dL/dconic (x, y, w of the reference's float4)
  kAccOp = 5,                             // dL/dopacity (effective opacity)
  kAccR = 6, kAccG = 7, kAccB = 8,        // dL/dcolor
  kAccDepth = 9,                          // dL/ddepth (view-space z)
  kAccF0 = 10, kAccF1 = 11, kAccF2 = 12,  // dL/dfeature
  kAccUsed = 13                           // reserved (always 0); slots 14, 15 unused
};

inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(char* b) : base(b) {}
  template <class T>
  T* take(size_t n) {
    off = align_up(off);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
  size_t size() const { return align_up(off); }
};

// ---- device-wide primitives (gsr_sort.hip) -----------------------------------------------------
constexpr int kScanTile = 2048;       // elements per scan workgroup (256 threads x 8)
constexpr int kScanMaxParts = 8192;   // partials scanned by the single-workgroup middle pass
#ifndef GSR_SORT_KPT
#define GSR_SORT_KPT 16
#endif
#ifndef GSR_SORT_TICKET
#define GSR_SORT_TICKET 1  // one-sweep partitions by atomic ticket (1) or by blockIdx (0)
#endif
constexpr int kSortTile = 256 * GSR_SORT_KPT;  // keys per radix-sort workgroup (256 threads x KPT)

inline size_t scan_parts(size_t n) { return (n + kScanTile - 1) / kScanTile; }
inline size_t sort_blocks(size_t n) { return (n + kSortTile - 1) / kSortTile; }
constexpr int sort_passes(int bits) { return (bits + 7) / 8; }
// Digit width of a sort over `bits` key bits: the passes split the bits evenly (12-bit tile ids:
// 6 + 6 instead of 8 + 4) -- fewer, longer runs per bucket in the scatter of the first pass.  Any
// split gives the same stable order.  (constexpr: host and device)
constexpr int sort_digit_bits(int bits) {
  return (bits + sort_passes(bits) - 1) / sort_passes(bits);
}
constexpr int kSortMaxPasses = 4;
// Partitions per look-back super-partition: besides its own status word, every partition adds its
// digit counts into its super-partition's word, so a look-back crosses 16 partitions per word.
constexpr int kSortSuper = 16;
inline size_t sort_supers(size_t n) { return (sort_blocks(n) + kSortSuper - 1) / kSortSuper; }
// u64 look-back words of one pass: [partition][256] status words, then [super-partition][256]
// super words (count | contributors << 32)
inline size_t sort_pass_words(size_t n) { return (sort_blocks(n) + sort_supers(n)) * 256; }
inline size_t sort_status_len(size_t n) { return (size_t)kSortMaxPasses * sort_pass_words(n); }
// u32 aux words: digit totals as kSortTotShards partial copies [shard][kSortMaxPasses][256] (the
// totals kernel's workgroups add into shard blockIdx % kSortTotShards: same-line device-scope
// atomics serialise at the memory side, so one shared copy made ~250-720 workgroups queue on the
// same 8 lines), sentinel-key counts [shard], partition tickets [kSortMaxPasses][8], error flag
constexpr int kSortTotShards = 16;
constexpr size_t kSortTotTileWords = (size_t)kSortTotShards * kSortMaxPasses * 256;
constexpr size_t kSortAuxTotals = 0,
                 kSortAuxSent = kSortAuxTotals + (size_t)kSortTotShards * kSortMaxPasses * 256,
                 kSortAuxTickets = kSortAuxSent + kSortTotShards,
                 kSortAuxErr = kSortAuxTickets + 8 * kSortMaxPasses,
                 // planned sorts (a third buffer pair): the plan -- bit p set for each pass
                 // that runs (gsr_sort.hip sort_plan_kernel)
                 kSortAuxPlan = kSortAuxErr + 4, kSortAuxLen = kSortAuxPlan + 4;
// Key whose position in the sorted output does not matter (culled Gaussians: no tiles): it is
// left out of the count of digits present, so a pass whose digit is constant over every other key
// is a plain copy (see radix_onesweep_kernel).
constexpr uint32_t kSortSentinel = 0xffffffffu;

struct SortScratch {
  uint64_t* status;  // [sort_status_len(n)]
  uint32_t* aux;     // [kSortAuxLen]; aux[kSortAuxErr] != 0 after a sort = look-back timeout
};
// Bytes from scratch.aux that must be zero before a sort of n keys over `bits` bits (aux words
// and the status words of the passes used); a multiple of 16 (status is 256-B aligned).
inline size_t sort_clear_bytes(const SortScratch& sc, size_t n, int bits) {
  return (size_t)((char*)(sc.status + (size_t)sort_passes(bits) * sort_pass_words(n)) -
                  (char*)sc.aux);
}
// A zero-fill piggy-backed on a kernel that runs anyway (no separate memset launch): every
// thread of the grid clears its grid-stride share.  bytes: multiple of 4, p 16-B aligned.
struct SideClear {
  void* p;
  size_t bytes;
};
inline SortScratch take_sort_scratch(Carver& c, size_t n) {
  SortScratch s;
  s.aux = c.take<uint32_t>(kSortAuxLen);
  s.status = c.take<uint64_t>(sort_status_len(n));  // follows aux: one memset clears both
  return s;
}

// Exclusive (inclusive=false) or inclusive prefix sum of n u32 values; if gather != nullptr the
// input element i is in[gather[i]].  parts: scratch of scan_parts(n) u32.
hipError_t scan_u32(const uint32_t* in, const uint32_t* gather, uint32_t* out, size_t n,
                    bool inclusive, uint32_t* parts, hipStream_t s);
// out[0] = sum of n u32 partial sums (one launch); with parts2, out[1] = the sum of parts2[0..n).
hipError_t sum_u32_parts(const uint32_t* parts, size_t n, uint32_t* out, hipStream_t s,
                         const uint32_t* parts2 = nullptr);
// *out = sum of n u32 values (two launches); parts: scratch of scan_parts(n) u32.
hipError_t reduce_u32(const uint32_t* in, size_t n, uint32_t* parts, uint32_t* out,
                      hipStream_t s);
// Stable LSD radix sort of (key, value) u32 pairs over key bits [0, bits).  Ping-pongs between
// (ka, va) and (kb, vb); returns through *result_in_b whether the sorted data ended in (kb, vb).
// One-sweep passes: 1 memset + 1 digit-totals launch + 1 launch per 8-bit digit; a pass whose
// digit is the same for every key is a plain copy.  sentinel_anywhere: keys equal to
// kSortSentinel may end up at any position (the depth sort's culled Gaussians), so they do not
// count when deciding whether a digit is constant.
// precleared: sort_clear_bytes(scratch, n, bits) from scratch.aux are already zero (cleared by
// an earlier kernel on the stream through a SideClear): the memset launch is skipped.
// key_payload: when set, the LAST pass writes key_payload[value] instead of the sorted key (the
// keys themselves are not needed afterwards): the depth sort hands the scan its tile counts
// already in depth order, one gather inside the sort instead of two in the scan.
// kc, vc (optional, a third buffer pair): a PLANNED sort -- the digit-totals launch marks every
// pass whose digit is the same for every (non-sentinel) key, those passes do not run at all (not
// even as a copy), and the passes that do run ping-pong between (kc, vc) and (kb, vb) so that the
// last one writes (kb, vb): the result is always in (kb, vb), (ka, va) is only read.  Same
// result as the unplanned sort, bit for bit (a constant digit's stable pass is the identity).
hipError_t radix_sort_pairs(uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb, size_t n,
                            int bits, SortScratch scratch, bool* result_in_b, hipStream_t s,
                            bool sentinel_anywhere = false, bool precleared = false,
                            const uint32_t* key_payload = nullptr, uint32_t* kc = nullptr,
                            uint32_t* vc = nullptr);
// Several independent sorts / scans / sums, one launch per stage for all of them (the multi-view
// forward's batched binning, gsr_api.cpp): a view's workgroups are a contiguous block range of
// the launch, and inside it everything is the one-view kernel's (own totals, tickets, look-back
// words), so each result is bit-identical to its own radix_sort_pairs / scan_u32 / sum_u32_parts.
// The sorts ping-pong alike: *result_in_b holds for every view.
constexpr int kMaxBatchViews = 8;
struct SortSpec {
  uint32_t *ka, *va, *kb, *vb;
  size_t n;
  SortScratch scratch;
  const uint32_t* key_payload;
  uint32_t *kc = nullptr, *vc = nullptr;  // planned sort (radix_sort_pairs): all views or none
  // keys-only packed sort (lo > 0; all views or none, va / vb only receive the last pass's
  // values): the keys carry the sort key in bits [lo, lo + bits) and the value in bits [0, lo);
  // the result pair is (key >> lo, key & (2^lo - 1)) in the buffers the pair sort would use
  int lo = 0;
  // > 0: the values carry a payload in bits [vsplit, 32); the last pass writes (value >> vsplit)
  // in place of the key and value & (2^vsplit - 1) as the value (no key_payload gather)
  int vsplit = 0;
  // digit totals formed by an earlier kernel on the stream, laid out as the totals launch's
  // ([kSortTotShards][kSortMaxPasses][256], the multi-view duplication's GeomState::ttot): the
  // totals launch is skipped.  All views or none; not with a planned sort, sums or sentinels.
  const uint32_t* totals = nullptr;
};
// sums (one per view, optional): the views' read-back sums formed inside the digit-totals launch
// (sum_u32_parts_views folded in); after_totals (optional): recorded right after that launch
struct SumSpec;
hipError_t radix_sort_pairs_views(const SortSpec* v, int V, int bits, bool* result_in_b,
                                  hipStream_t s, bool sentinel_anywhere, bool precleared,
                                  const SumSpec* sums = nullptr, hipEvent_t after_totals = nullptr);
struct ScanSpec {
  const uint32_t* in;
  uint32_t* out;
  size_t n;
  uint32_t* parts;
};
hipError_t scan_u32_views(const ScanSpec* v, int V, bool inclusive, hipStream_t s);
// Inclusive scans in ONE launch (decoupled look-back): status = scan_lb_words(n) zeroed u64 words
// (a ticket counter, then one status word per kScanTile partition); err raised on a timed-out
// look-back.
inline size_t scan_lb_words(size_t n) { return scan_parts(n) + 1; }
struct ScanLbSpec {
  const uint32_t* in;
  uint32_t* out;
  size_t n;
  uint64_t* status;
  uint32_t* err;
};
hipError_t scan_u32_lookback_views(const ScanLbSpec* v, int V, hipStream_t s);
// out[0..1] = sums of parts / parts2 (n partials each); host (device pointer of pinned words, or
// null) receives {*flag0 (0 if null), out[0], out[1]}.
struct SumSpec {
  const uint32_t* parts;
  const uint32_t* parts2;
  size_t n;
  uint32_t* out;
  uint32_t* host;
  const uint32_t* flag0;
};
hipError_t sum_u32_parts_views(const SumSpec* v, int V, hipStream_t s);
// Device word counting look-back timeouts of any sort on the current device (sticky until the
// host resets it); every forward reads it back with its instance count.
uint32_t* sort_timeouts_word();
// Device address of the sticky per-device forward fault word (kStatus* bits; gsr.h
// gsr_forward_faults / gsr_reset_forward_faults): or-ed by the tile-ranges kernel and the forward
// blend of a failed call, read by the fused Adam step (which then skips the update).
uint32_t* forward_faults_word();

// ---- layouts -------------------------------------------------------------------------------------
struct GeomState {
  uint32_t* dkey_a;         // [P] depth-sort keys (float bits of z; 0xffffffff if culled)
  uint32_t* dval_a;         // [P] Gaussian ids, depth-sorted after the sort (see depth_sorted())
  uint32_t* dkey_b;          // the planned depth sort's result (radix_sort_pairs kb, vb)
  uint32_t* dval_b;
  uint32_t* dkey_c;          // its third buffer pair
  uint32_t* dval_c;
  uint8_t* clamped;         // [P] bit c set <=> SH colour channel c clamped (forward.cu:67-69)
  int32_t* radii;           // [P] internal radii (used when the caller passes none)
  float4* rec;              // [P*4] splat record for the blend
  // [P] the duplication's 8-B binning word of a Gaussian with tiles (gsr_preprocess.hip
  // bin_word): .x = x0 | y0 << 14 | rows << 28 of its tile rectangle, .y = its packed per-row kept
  // ranges (rec[3].w); .y = kNoRowPack: not packed, the duplication reads the record instead
  uint2* bword;
  uint32_t* tiles_touched;  // [P]
  uint32_t* offsets;        // [P] inclusive scan of tiles_touched in depth order
  float* acc;               // [P*16] backward accumulators (atomic mode; not the deterministic backward)
  uint32_t* ebeg;           // [P] per Gaussian id: its first emission index (rows mode, DET)
  uint32_t* flags;          // [4]  [0]: prefiltered violation
  SortScratch sort;         // depth-sort scratch
  uint32_t* scan_parts;
  // [scan_lb_words(P)] look-back scan status (the batched forward's scan); follows the sort
  // scratch so that the preprocess's side clear zeroes both (scan_clear_end)
  uint64_t* scan_status;
  // [kSortTotTileWords] the tile sort's digit totals, added up by the multi-view duplication
  // (DupSpec::ttot) for its sort (SortSpec::totals); zeroed by the same side clear
  uint32_t* ttot;
  // [2 * ceil(P/256)] per preprocess workgroup: the sum of its exact tile counts, then (second
  // half) the sum of its full 3-sigma tile rectangles -- the reference's tiles_touched
  // (forward.cu:255), whose total is the num_rendered the boundary returns
  uint32_t* pre_parts;
  size_t bytes;
};
GeomState carve_geom(char* base, size_t P);

struct BinState {
  uint32_t* tag;     // [4] the forward's layout: bin_layout_tag(det, rows) (first 256-B granule)
  uint32_t* tkey_a;  // [R] tile ids of the duplicated instances
  uint32_t* tval_a;  // [R] Gaussian ids
  uint32_t* tkey_b;
  uint32_t* tval_b;
  SortScratch sort;  // tile-sort scratch
  // rows layout (the deterministic backward, gsr.h debug bit 1): the tile sort carries each
  // instance's emission index e (depth order, Gaussian-major) instead of its Gaussian id, and the
  // backward blend stores one gradient row per instance instead of float atomics
  uint32_t* egid;    // [R] Gaussian id of emission index e
  float* partial;    // [R][kAccFloats] the blend backward's gradient row of each instance, by e
  size_t bytes;
};
BinState carve_bin(char* base, size_t R, bool rows = false);
// rec[3].w of a splat record whose per-row tile ranges did not fit the packing (gsr_preprocess.hip)
constexpr uint32_t kNoRowPack = 0xffffffffu;
constexpr uint32_t kBinLayoutMagic = 0x47535200u;  // "GSR\0"
inline uint32_t bin_layout_tag(bool det, bool rows) {
  return kBinLayoutMagic | (det ? 2u : 0u) | (rows ? 1u : 0u);
}

struct ImgState {
  float* final_T;       // [H*W]
  uint32_t* n_contrib;  // [H*W]
  uint2* ranges;        // [tiles]
  uint32_t* tile_last;  // [tiles] max n_contrib over the tile's pixels
  uint32_t* order;      // [tiles] workgroup -> tile schedule (heaviest first)
  // [4] per-call status of this forward (kStatus* bits): written by the tile-ranges kernel from
  // the two sorts' error words, or-ed by the forward blend when it clamps an out-of-range id; a
  // non-zero word poisons this call's outputs and gradients and fails its backward / status check
  uint32_t* status;
  size_t bytes;
};
ImgState carve_img(char* base, size_t W, size_t H);
constexpr uint32_t kStatusDepthSort = 1u, kStatusTileSort = 2u, kStatusClamp = 4u;

// workgroup -> tile schedule of the blend kernels (env GSR_TILE_ORDER: natural | xcd | lpt)
int tile_schedule_mode();

// ---- per-Gaussian kernels (gsr_preprocess.hip, gsr_backward.hip) ----------------------------------
constexpr int kShFlushMaxViewsFwd = 8;
struct PreArgs {
  int P, D, M, W, H;
  uint32_t gx, gy;
  const float *means3D, *scales, *rotations, *opacities, *shs, *cov3D_precomp, *colors_precomp;
  const float *sh_language, *lang_precomp, *confidence;
  const float *view, *proj, *campos;
  float scale_modifier, tanx, tany, fx, fy;
  int prefiltered, include_feature;
  int32_t* radii;
  GeomState g;
  // fused-activation inputs (gsr_rasterize_gaussians_fused): when fused != 0, scales / rotations /
  // opacities hold GaussianModel's raw _scaling (log), _rotation (unnormalised), _opacity (logit)
  // and the SH coefficients come split as sh_dc [P,1,3] + sh_rest [P,M-1,3]
  int fused;
  const float *sh_dc, *sh_rest;
  // zero-fills done by the preprocess grid: the depth sort's scratch, and (acc_zero != 0) the
  // backward's per-Gaussian gradient accumulator rows g.acc
  SideClear clear;
  int acc_zero;
  uint32_t* parts;  // [2 * gridDim.x] sums of the workgroup's exact / full-rectangle tile counts
  // multi-view colour pre-pass (fused only): when non-null, the SH colour of this view and its
  // clamp bits come precomputed (gsr_sh_precolor) instead of being evaluated from the SH rows
  const float* pre_color;
  const uint8_t* pre_clamp;
  // > 0: the depth sort's value is id | (exact tile count << vpack) (the sort's last pass splits it,
  // SortSpec::vsplit, instead of gathering the counts by id)
  uint32_t vpack = 0;
};
hipError_t launch_preprocess(const PreArgs& a, hipStream_t s);
// Several views of one model in one launch (every view's PreArgs share the model fields): per
// view the outputs of launch_preprocess, bit for bit.
struct PreViews {
  PreArgs v[kMaxBatchViews];
  int V;
};
static_assert(sizeof(PreViews) <= 4096, "kernel argument size");
hipError_t launch_preprocess_views(const PreArgs* views, int V, hipStream_t s);
struct PrecolorArgs {
  int P, M, D, nviews;
  uint32_t row0, row1;  // the Gaussian rows [row0, row1) of this launch (outputs: planes of P)
  const float *means3D, *sh_dc, *sh_rest;
  const float* campos[kShFlushMaxViewsFwd];
  float* color[kShFlushMaxViewsFwd];     // [3][P] (planar)
  uint8_t* clamp[kShFlushMaxViewsFwd];   // [P]
  float* jac[kShFlushMaxViewsFwd];       // [9][P] (planar): dRGB/ddir_x, _y, _z (vec3 over the channels)
};
hipError_t launch_sh_precolor(const PrecolorArgs& a, hipStream_t s);
// test hook: ref = OCML expf(x), fast = splat_exp(x) (gsr_device.h), the blends' exp
hipError_t launch_expf_pair(const float* x, float* ref, float* fast, size_t n, hipStream_t s);
// test hook: the fused path's in-kernel activations (sigmoid / exp / normalize of gsr_device.h)
hipError_t launch_activations(const float* op_raw, const float* sc_raw, const float* rot_raw,
                              size_t P, float* op, float* sc, float* rot, hipStream_t s);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present,
                               hipStream_t s);

struct BwdPreArgs {
  int P, D, M;
  const float *means3D, *scales, *rotations, *shs, *cov3D, *colors_precomp;
  const float *sh_language, *lang_precomp, *confidence;
  const float *view, *proj, *campos;
  float scale_modifier, tanx, tany, fx, fy;
  int include_feature;
  const int32_t* radii;
  const uint8_t* clamped;
  const float* acc;
  // outputs (every element written; with accumulate != 0 the grads of visible Gaussians are
  // added into the buffers and culled Gaussians are left untouched)
  float *dL_dmeans2D, *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales,
      *dL_drotations, *dL_dsh_language, *dL_dlanguage_feature;
  // fused mode: inputs are raw parameters (see PreArgs) and the outputs are the raw-parameter
  // grads: dL_dopacity -> d _opacity, dL_dscales -> d _scaling, dL_drotations -> d _rotation,
  // dL_dsh -> d features_dc, dL_dsh_rest -> d features_rest
  int fused, accumulate;
  const float *sh_dc, *sh_rest, *opacities_raw;
  float* dL_dsh_rest;
  // deferred SH gradients (fused only): when non-null, the SH grads are not written; instead the
  // clamp-masked colour gradient dL/dRGB, planar [3][P] (zeros when culled), is stored here for
  // launch_sh_grad_flush, which forms dL/dsh = basis(dir) x dL/dRGB for all views of a step
  float* dRGB_out;
  // with dRGB_out: the SH colour's direction Jacobian of this view from the pre-pass ([P,9]); the
  // SH rows are then not read at all
  const float* pre_jac;
  // the forward's status word (ImgState::status): non-zero -> NaN gradients (same-call poison)
  const uint32_t* status;
  // rows layout: Gaussian i's gradient row is the sum of rows[ebeg[i] .. ebeg[i] + count[i])
  // (its instances' rows in emission order) instead of acc[i]
  int use_rows;
  const float4* rows;
  const uint32_t* ebeg;
  const uint32_t* count;
};
hipError_t launch_preprocess_backward(const BwdPreArgs& a, hipStream_t s);
// the per-Gaussian backwards of several views in one launch (fused, deferred SH with the pre-pass
// Jacobian, shared gradient buffers, views after the first accumulating); hipErrorNotSupported
// for any other configuration (the caller then launches per view)
struct BwdPreViews {
  BwdPreArgs v[8];
  int V;
  uint32_t row0, row1;  // the Gaussian rows [row0, row1) of this launch
};
// rows [row0, row1) of the per-Gaussian backward (row1 > P: up to P)
hipError_t launch_preprocess_backward_views(const BwdPreArgs* views, int V, hipStream_t s,
                                            uint32_t row0 = 0, uint32_t row1 = 0xffffffffu);
constexpr int kShFlushMaxViews = 8;
struct ShFlushArgs {
  int P, M, D, nviews, accumulate;
  const float* means3D;
  const float* campos[kShFlushMaxViews];  // device [3] each
  const float* dRGB[kShFlushMaxViews];    // device planar [3][rgb_stride] each
  size_t rgb_stride;
  float *dL_dsh_dc, *dL_dsh_rest;         // features_dc [P,1,3] / features_rest [P,M-1,3] grads
};
hipError_t launch_sh_grad_flush(const ShFlushArgs& a, hipStream_t s);

// ---- binning (gsr_binning.hip) -------------------------------------------------------------------
// The duplicate grid also zero-fills clear0 / clear1 (the tile sort's scratch, the ranges).
// R bounds the writes (offsets of a complete depth order never exceed it).
// egid != nullptr (rows layout): tval gets emission indices, egid[e] the Gaussian id and
// ebeg[gid] the Gaussian's first emission index.
hipError_t launch_duplicate(int P, const uint32_t* order, const uint32_t* offsets,
                            const int32_t* radii, const float4* rec, uint32_t gx, uint32_t gy,
                            uint32_t* tkey, uint32_t* tval, uint32_t R, SideClear clear0,
                            SideClear clear1, hipStream_t s, uint32_t* egid = nullptr,
                            uint32_t* ebeg = nullptr, const uint2* bword = nullptr);
// ranges_cleared: the ranges are already zero (duplicate's side clear): no memset launch.
// Also writes the call's status word from the depth / tile sorts' error words (either may be null).
// A failed call also or-s its status into `fault` (forward_faults_word(), may be null).
hipError_t launch_tile_ranges(size_t R, const uint32_t* sorted_tiles, uint2* ranges,
                              uint32_t ntiles, const uint32_t* depth_err, const uint32_t* tile_err,
                              uint32_t* status, uint32_t* host_status, uint32_t* fault,
                              hipStream_t s, bool ranges_cleared = false);
// The same two stages for several views in one launch each (the batched binning; ranges must be
// cleared already, by the duplicate's side clear).
struct DupSpec {
  int P;
  const uint32_t* order;
  const uint32_t* offsets;
  const float4* rec;
  uint32_t gx, gy;
  uint32_t* tkey;
  uint32_t* tval;
  uint32_t R;
  SideClear clear0, clear1;
  uint32_t* egid;
  uint32_t* ebeg;
  uint32_t* tag = nullptr;  // written with tag_val by the launch (the binning buffer's layout tag)
  uint32_t tag_val = 0;
  // > 0: packed keys tile << pack | gid into tkey for the keys-only tile sort (tval not written;
  // needs gid < 2^pack, no egid)
  uint32_t pack = 0;
  const uint2* bword = nullptr;  // GeomState::bword (null: every Gaussian's record is read)
  // non-null: the duplication also adds the digit counts of the tile sort over `tbits` bits
  // (tbits <= 16) into these zeroed totals (layout of SortSpec::totals)
  uint32_t* ttot = nullptr;
  int tbits = 0;
};
hipError_t launch_duplicate_views(const DupSpec* v, int V, hipStream_t s);
struct RangesSpec {
  size_t R;
  const uint32_t* tiles;
  uint2* ranges;
  uint32_t ntiles;
  const uint32_t* depth_err;
  const uint32_t* tile_err;
  uint32_t* status;
  uint32_t* host_status;
  uint32_t* fault;
};
hipError_t launch_tile_ranges_views(const RangesSpec* v, int V, hipStream_t s);

// ---- blend (gsr_render.hip) ----------------------------------------------------------------------
struct RenderArgs {
  int W, H;
  uint32_t gx, gy;
  const uint2* ranges;
  const uint32_t* point_list;
  const float4* rec;
  uint32_t P;  // rows of rec: point_list entries are clamped to it (a failed sort cannot fault)
  const float* bg;
  float* final_T;
  uint32_t* n_contrib;
  uint32_t* tile_last;
  float *out_color, *out_depth, *out_alpha, *out_feature;
  int include_feature;
  uint32_t* order;
  int sched;
  uint32_t* status;  // ImgState::status: non-zero -> NaN outputs; kStatusClamp or-ed on a clamp
  uint32_t* host_status;  // pinned, device-mapped mirror of the clamp bit (may be null)
  uint32_t* fault;        // forward_faults_word() (may be null): kStatusClamp or-ed on a clamp
  // zero-fill done by the blend's grid (the multi-view call: the view's backward accumulator
  // rows, moved off the memory-bound preprocess onto this VALU-bound kernel); p = null: none
  SideClear clear;
};
hipError_t launch_render_forward(const RenderArgs& a, hipStream_t s);
// the two halves of launch_render_forward for multi-view calls: the heaviest-first tile schedule
// of one view, and the blends of several views in one launch
constexpr int kMaxFwdViews = 8;
struct RenderFwdViews {
  RenderArgs v[kMaxFwdViews];
  uint32_t first[kMaxFwdViews + 1];  // first workgroup of view k; first[V] = total
  int V;
};
hipError_t launch_render_schedule(const RenderArgs& a, hipStream_t s);
// the schedules of several views' tiles, one workgroup per view (views with sched != 2 skipped)
hipError_t launch_render_schedule_views(const RenderArgs* views, int V, hipStream_t s);
hipError_t launch_render_forward_views(const RenderArgs* views, int V, hipStream_t s);

struct RenderBwdArgs {
  int W, H;
  uint32_t gx, gy;
  const uint2* ranges;
  const uint32_t* point_list;
  const float4* rec;
  uint32_t P;  // rows of rec: point_list entries are clamped to it (a failed sort cannot fault)
  const float* bg;
  const float* final_T;
  const uint32_t* n_contrib;
  const uint32_t* tile_last;
  const float *dL_dcolor, *dL_ddepth, *dL_dalpha, *dL_dfeature;
  float* acc;
  int include_feature;
  uint32_t* order;
  int sched;
  // rows layout: per-instance rows partial[einst[q]] instead of atomics into acc; det selects
  // the deterministic summation order of the four waves' contributions (gsr.h debug bit 1)
  const uint32_t* einst;  // [R] emission index of tile-sorted instance q
  float* partial;         // [R][kAccFloats]
  int det;
  // rows of partial (the binning capacity): emission indices are clamped to it, so the output of
  // a sort that gave up cannot send a store out of bounds
  uint32_t nrows;
  const uint32_t* status;  // ImgState::status: a failed forward's backward blend writes nothing
};
hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t s);
// several views' backward blends in one launch (all views must share the template switches:
// upstream depth/alpha present, feature, rows layout, deterministic)
constexpr int kMaxBwdViews = 8;
struct RenderBwdViews {
  RenderBwdArgs v[kMaxBwdViews];
  uint32_t first[kMaxBwdViews + 1];  // first workgroup of view k; first[V] = total
  int V;
};
hipError_t launch_render_backward_views(const RenderBwdArgs* views, int V, hipStream_t s);
// rows layout forward: point_list[q] = egid[einst[q]]
hipError_t launch_det_gather(size_t R, const uint32_t* einst, const uint32_t* egid,
                             uint32_t* point_list, hipStream_t s);

}  // namespace gsr

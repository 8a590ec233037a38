/*
 * gsr_testing.h -- test hooks of libgsr (NOT part of the drop-in boundary in gsr.h).
 *
 * They expose the device-wide primitives that replace the reference's CUB calls
 * (cub::DeviceScan::InclusiveSum, rasterizer_impl.cu:277; cub::DeviceRadixSort::SortPairs,
 * :303-308) so that tests/ can check sortedness, stability and prefix sums at full size.
 */
#ifndef GSR_TESTING_H
#define GSR_TESTING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scratch bytes needed by gsr_test_radix_sort_pairs for n pairs. */
size_t gsr_test_sort_scratch_bytes(size_t n);
/* Stable LSD radix sort of (keys, vals) over key bits [0, bits), in place (device pointers). */
int gsr_test_radix_sort_pairs(uint32_t* keys, uint32_t* vals, size_t n, int bits, void* scratch,
                              void* stream);
/* Same, as the depth sort runs it: keys equal to 0xffffffff (culled Gaussians) may end up at any
 * position; every other key is in stable sorted order. */
/* Test hook: on != 0 makes every one-sweep look-back take its bounded-spin give-up path (the
 * sort's error word is raised and its output is garbage), to test the same-call backstop. */
int gsr_test_force_sort_timeout(int on);

int gsr_test_radix_sort_pairs_sentinel(uint32_t* keys, uint32_t* vals, size_t n, int bits,
                                       void* scratch, void* stream);
/* The planned sort (the depth sort's): passes whose digit is constant over the (non-sentinel)
 * keys do not run; same result as gsr_test_radix_sort_pairs[_sentinel]. */
int gsr_test_radix_sort_pairs_planned(uint32_t* keys, uint32_t* vals, size_t n, int bits,
                                      int sentinel_anywhere, void* scratch, void* stream);
/* Scratch bytes needed by gsr_test_scan for n elements. */
size_t gsr_test_scan_scratch_bytes(size_t n);
/* out = inclusive (or exclusive) prefix sum of in (device pointers). */
int gsr_test_scan(const uint32_t* in, uint32_t* out, size_t n, int inclusive, void* scratch,
                  void* stream);

/* ref[i] = expf(x[i]) (OCML), fast[i] = splat_exp(x[i]), the blends' deterministic exp
 * (gsr_device.h; the oracle evaluates the same sequence) (device pointers). */
int gsr_test_expf_pair(const float* x, float* ref, float* fast, size_t n, void* stream);

/* The tile-sorted instance list a forward left in its buffers (device pointers; sizes as the
 * forward was called): point_list_out[0 .. n_instances) -- the first gsr_last_forward_instances()
 * entries the blends read -- and ranges_out[tiles * 2] (uint2 [start, end) per tile, (0, 0) when
 * empty).  num_rendered is the forward's return value (it sizes the binning layout), debug its
 * debug word (bit 1: deterministic layout).  Lets tests/ pin the binning (duplicateWithKeys +
 * SortPairs + identifyTileRanges, rasterizer_impl.cu:70-138) to the oracle's lists. */
int gsr_test_binning_lists(const void* binning_buffer, const void* image_buffer, int num_rendered,
                           int image_height, int image_width, int debug, int n_instances,
                           uint32_t* point_list_out, uint32_t* ranges_out, void* stream);

/* The splat records a forward's preprocess left in its geometry buffer (geom_buffer: device; P as
 * the forward was called; rec_out: host, [P][16] floats): per Gaussian {x_px, y_px, conic.a,
 * conic.b}, {conic.c, opacity * confidence, depth, red}, {green, blue, f0, f1}, {f2, radius,
 * q_cut, packed rows} (gsr_preprocess.hip).  Lets tests/ compare the preprocess outputs
 * (preprocessCUDA, forward.cu:155-256: means2D, conic_opacity, depths, rgb) entry by entry with
 * the float64 oracle. */
int gsr_test_splat_records(const void* geom_buffer, int P, float* rec_out, void* stream);

/* The fused path's GaussianModel activations as its kernels evaluate them (device pointers):
 * opacity = sigmoid(opacity_raw) [P], scaling = exp(scaling_raw) [P,3],
 * rotation = normalize(rotation_raw) [P,4] (16-byte aligned).  Lets the tests feed the CPU oracle
 * the exact activated values the kernels used and compare them with torch's getters
 * (scene/gaussian_model.py:33-41). */
int gsr_test_activations(const float* opacity_raw, const float* scaling_raw,
                         const float* rotation_raw, size_t P, float* opacity, float* scaling,
                         float* rotation, void* stream);

/* Stage timing with hipEvents recorded on the caller's stream around the kernels of the forward
 * and backward (used by bench.py for the per-kernel roofline).  Off by default; each enabled
 * stage launch is bracketed by two events (a few microseconds per stage and view, so bench.py
 * instruments only the dominant stage inside its timed region). */
enum {
  GSR_STAGE_PREPROCESS = 0, GSR_STAGE_DEPTH_SORT, GSR_STAGE_SCAN, GSR_STAGE_DUPLICATE,
  GSR_STAGE_TILE_SORT, GSR_STAGE_RANGES, GSR_STAGE_RENDER_FWD, GSR_STAGE_ACC_ZERO,
  GSR_STAGE_RENDER_BWD, GSR_STAGE_PREPROCESS_BWD, GSR_STAGE_SH_PRECOLOR, GSR_STAGE_SH_FLUSH,
  GSR_NUM_STAGES
};
/* stage_mask: bit GSR_STAGE_x enables that stage; 0 disables; -1 (all bits) enables all. */
// Host wall time (ms) the forward calls of this process spent waiting for their instance-count
// read-back (hipEventSynchronize); reset != 0 zeroes the counter after reading it.
double gsr_test_host_wait_ms(int reset);
/* The batched forward's single-pass look-back scan (inclusive) of `views` arrays of n u32 each,
 * back to back in `in` / `out`; scratch: views * gsr_test_scan_lookback_words(n) * 8 + 16 bytes. */
size_t gsr_test_scan_lookback_words(size_t n);
int gsr_test_scan_lookback(const uint32_t* in, uint32_t* out, size_t n, int views, void* scratch,
                           void* stream);

void gsr_profile_enable(int stage_mask);
/* Waits for the recorded events, adds their durations into ms[GSR_NUM_STAGES] and
 * calls[GSR_NUM_STAGES] (accumulating since the last reset) and recycles the events. */
int gsr_profile_collect(double* ms, long long* calls);
void gsr_profile_reset(void);
const char* gsr_profile_stage_name(int stage);

#ifdef __cplusplus
}
#endif
/* Test-only bits of the multi-view backward's `debug` argument (gsr_rasterize_views_fused_backward):
 * NO_BLEND skips the accumulator clear and the backward blend, so the per-Gaussian backward runs
 * again on the gradient rows an earlier backward of the same forward left in the geometry
 * buffers; PER_VIEW_PRE runs it as one launch per view instead of the merged multi-view launch.
 * Together they compare the two per-Gaussian paths on identical inputs. */
#define GSR_DEBUG_TEST_NO_BLEND 256
#define GSR_DEBUG_TEST_PER_VIEW_PRE 512

#endif /* GSR_TESTING_H */

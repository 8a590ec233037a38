/*
 * gsr_densify.h -- C ABI of libgsr's adaptive density control.
 *
 * Replaces the boolean-mask / torch.cat bookkeeping of GaussianModel's densification
 * (scene/gaussian_model.py:400-612) and of the per-step statistics update in train.py:218-220:
 *   gsr_densify_stats     <- train.py:219 (max_radii2D) + add_densification_stats (:606-609)
 *   gsr_densify_classify  <- the per-Gaussian tests of densify_and_clone (:566-570),
 *                            densify_and_split (:537-542) and densify_and_prune (:583-597)
 *   gsr_select_rows       <- the nonzero() behind every boolean-mask index of those functions
 *   gsr_compact_rows      <- _prune_optimizer (:417-432), prune_points (:434-452),
 *                            cat_tensors_to_optimizer (:454-476) and densification_postfix
 *                            (:478-511): all parameter, Adam-moment, confidence and statistics
 *                            arrays rebuilt in ONE launch
 * All pointers are device pointers; the stream is a hipStream_t.  Return 0 on success, 1 on
 * invalid arguments, 2 on a launch error.
 */
#ifndef GSR_DENSIFY_H
#define GSR_DENSIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-step statistics, in place, for every i with update_filter[i] != 0 (or radii[i] > 0 when
 * update_filter is NULL -- render()'s visibility_filter):
 *   max_radii2D[i] = max(max_radii2D[i], (float)radii[i])          (skipped if max_radii2D NULL)
 *   grad_accum[i] += sqrt(g[i*grad_stride]^2 + g[i*grad_stride+1]^2),  denom[i] += 1
 *                                                (skipped if grad_accum and denom are NULL)
 * g is viewspace_point_tensor.grad ([P, grad_stride] floats, grad_stride >= 2). */
int gsr_densify_stats(int64_t P, const float* viewspace_grad, int64_t grad_stride,
                      const int32_t* radii, const uint8_t* update_filter, float* max_radii2D,
                      float* grad_accum, float* denom, void* stream);
/* The same for the V views of a multi-view step in one launch (filter radii > 0): view v's
 * gradient rows start at viewspace_grad + v * grad_view_stride, its radii at radii + v * P; per
 * Gaussian the views are applied in order, so the result equals V calls of gsr_densify_stats. */
int gsr_densify_stats_views(int V, int64_t P, const float* viewspace_grad, int64_t grad_stride,
                            int64_t grad_view_stride, const int32_t* radii, float* max_radii2D,
                            float* grad_accum, float* denom, void* stream);

/* flag bits written by gsr_densify_classify */
#define GSR_DENSIFY_CLONE 1u       /* |accum/denom| >= grad_threshold && max scale <= scale_limit */
#define GSR_DENSIFY_SPLIT 2u       /*  accum/denom  >= grad_threshold && max scale >  scale_limit */
#define GSR_DENSIFY_LOW_OPACITY 4u /* sigmoid(_opacity) < min_opacity */
#define GSR_DENSIFY_BIG_WS 8u      /* big_enable && max scale > big_limit */

/* One flag byte per Gaussian from the raw parameters (_scaling [P,3] log scales, _opacity [P]
 * logits) and the statistics (grad_accum, denom: [P]); NaN ratios count as 0 (:585-586).  With
 * denom NULL, grad_accum holds the caller's grads as they are (densify_and_clone / _split called
 * directly).  max scale = max_k exp(_scaling[i,k]).  counts (device, 2 x u32, may be NULL):
 * [#clone, #split]. */
int gsr_densify_classify(int64_t P, const float* grad_accum, const float* denom,
                         const float* scaling, const float* opacity, float grad_threshold,
                         float scale_limit, float min_opacity, int big_enable, float big_limit,
                         uint8_t* flags, uint32_t* counts, void* stream);

/* Stable selection: index[0..count) = ascending i < n with (flags[i] & mask) == want; *count
 * (device u32, may be NULL) receives the number selected.  index must hold n entries.
 * scratch: gsr_select_scratch_bytes(n) bytes of device memory. */
size_t gsr_select_scratch_bytes(int64_t n);
int gsr_select_rows(int64_t n, const uint8_t* flags, uint32_t mask, uint32_t want,
                    uint32_t* index, uint32_t* count, void* scratch, void* stream);

#define GSR_COMPACT_MAX_ARRAYS 32

/* Row gather over n_arrays row-major arrays in one launch.  Array t has row_bytes[t] bytes per row
 * (a multiple of 4, <= 4096).  Output row j (j < n_out) of dst[t] is row v = index[j] (index NULL:
 * v = j) of the virtual concatenation [src[t] (n_old rows) | extra[t]]: src[t][v] if v < n_old,
 * else extra[t][v - n_old]; where that part's pointer is NULL (or src / extra itself is NULL) the
 * row is filled with the 32-bit word fill[t] (fill NULL: 0).  Used with NULL src and extra it
 * writes constant arrays (zeroed statistics, ones). */
int gsr_compact_rows(int n_arrays, const void* const* src, const void* const* extra,
                     void* const* dst, const int64_t* row_bytes, const uint32_t* fill,
                     int64_t n_old, const uint32_t* index, int64_t n_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_DENSIFY_H */

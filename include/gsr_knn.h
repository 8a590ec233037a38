/*
 * gsr_knn.h -- C ABI of libgsr's exact 3-nearest-neighbour search.
 *
 * Replaces simple_knn._C.distCUDA2, the un-vendored native KNN the reference imports at
 * scene/gaussian_model.py:20 and calls as `dist, nearest_indices = distCUDA2(points)` in
 * create_from_pcd (:198, initial scales) and proximity (:514, proximity densification).
 */
#ifndef GSR_KNN_H
#define GSR_KNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Device scratch needed by gsr_dist_knn3 for P points. */
size_t gsr_knn_scratch_bytes(int64_t P);

/* points: [P,3] float32 (device, row-major).  For every i:
 *   indices[3i..3i+2] = the 3 nearest j != i, ascending by (squared distance, j)
 *   mean_dist[i]      = (d0 + d1 + d2) / 3 of their squared distances
 * with squared distance fma(dz, dz, fma(dy, dy, dx * dx)), d = p_j - p_i.  Fewer than 3 other
 * points: the missing entries count as FLT_MAX with index -1.  indices may be NULL.
 * Returns 0 on success, 1 on invalid arguments, 2 on a launch error. */
int gsr_dist_knn3(int64_t P, const float* points, float* mean_dist, int32_t* indices,
                  void* scratch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_KNN_H */

/*
 * gsr_oracle_knn.c -- CPU restatement of distCUDA2 (simple_knn), the 3-NN helper the reference
 * imports at scene/gaussian_model.py:20 and calls at :198 (create_from_pcd) and :514 (proximity).
 *
 * TEST INFRASTRUCTURE ONLY (see gsr_oracle.h).  Never linked into the product.
 *
 * simple_knn is an un-vendored dependency (environment.yml:17; absent from /root/reference), so
 * this restates its published algorithm's RESULT -- for every point the 3 nearest other points
 * by squared distance and the mean of those squared distances, (b0 + b1 + b2) / 3 -- by brute
 * force, which is what its Morton-box search computes exactly.  Parity unpinned: no fixtures of
 * simple_knn exist in the reference tree.  Conventions shared with include/gsr_knn.h:
 *   squared distance  fmaf(dz, dz, fmaf(dy, dy, dx * dx)), d = p_j - p_i  (nvcc's contraction of
 *                     simple_knn's d.x*d.x + d.y*d.y + d.z*d.z)
 *   order             (distance, index) ascending; missing neighbours FLT_MAX / -1
 */
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "gsr_oracle.h"

static int before(float d, int32_t i, float bd, int32_t bi) {
  return d < bd || (d == bd && (uint32_t)i < (uint32_t)bi);
}

void oracle_dist_knn3(int64_t P, const float* pts, float* mean, int32_t* idx) {
  for (int64_t i = 0; i < P; i++) {
    float bd[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    int32_t bi[3] = {-1, -1, -1};
    const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
    for (int64_t j = 0; j < P; j++) {
      if (j == i) continue;
      const float dx = pts[3 * j] - px, dy = pts[3 * j + 1] - py, dz = pts[3 * j + 2] - pz;
      const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
      int32_t id = (int32_t)j;
      if (!before(d, id, bd[2], bi[2])) continue;
      /* insertion into the sorted triple */
      int k = 2;
      while (k > 0 && before(d, id, bd[k - 1], bi[k - 1])) {
        bd[k] = bd[k - 1];
        bi[k] = bi[k - 1];
        k--;
      }
      bd[k] = d;
      bi[k] = id;
    }
    mean[i] = (bd[0] + bd[1] + bd[2]) / 3.0f;
    if (idx) {
      idx[3 * i] = bi[0];
      idx[3 * i + 1] = bi[1];
      idx[3 * i + 2] = bi[2];
    }
  }
}

/*
 * gsr_loss.h -- C ABI of libgsr's training losses.
 *
 * Replaces the loss code either side of the rasterizer in train.py:
 *   gsr_photometric_loss[_backward]  <- Ll1 = l1_loss(image, gt) (utils/loss_utils.py:106-107) and
 *                                       loss = (1 - lambda) Ll1 + lambda (1 - ssim(image, gt))
 *                                       (train.py:99-100; ssim / _ssim :129-162: 11x11 Gaussian
 *                                       window, sigma 1.5, zero padding, C1 = 1e-4, C2 = 9e-4)
 *   gsr_pearson_loss[_backward]      <- 1 - pearson_corrcoef(x, y) (torchmetrics, train.py:126-129,
 *                                       :149), optionally min over x and 1 / (offset - x)
 * All pointers are device pointers, the stream a hipStream_t.  Returns 0 / 1 (invalid arguments)
 * / 2 (launch error).
 */
#ifndef GSR_LOSS_H
#define GSR_LOSS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Device scratch for one (image, gt) pair of shape [C,H,W]; the forward leaves the backward
 * coefficients in it (12 B per pixel-channel), so forward and backward share one scratch. */
size_t gsr_photometric_scratch_bytes(int C, int H, int W);

/* image, gt: [C,H,W] float32 contiguous.  out (device, 3 floats): loss, L1 mean, SSIM mean.
 * need_grad = 0 skips the backward coefficients. */
int gsr_photometric_loss(int C, int H, int W, const float* image, const float* gt,
                         float lambda_dssim, int need_grad, float* out, void* scratch,
                         void* stream);

/* grad_image = d(out . g)/d image for upstream device scalars g = (grad_loss, grad_l1,
 * grad_ssim), each may be NULL (= 0).  Needs the scratch of a need_grad forward on the same
 * inputs. */
int gsr_photometric_loss_backward(int C, int H, int W, const float* image, const float* gt,
                                  float lambda_dssim, const float* grad_loss,
                                  const float* grad_l1, const float* grad_ssim, float* grad_image,
                                  void* scratch, void* stream);

/* Pearson correlation per column of x, y: [N, K] float32 (K <= 256).  variants = 1: r(x, y);
 * variants = 2: also r(1 / (offset - x), y) (train.py:127-128 with offset 200).  out_r
 * [variants*K] (may be NULL): the clamped r; out_loss [K] (may be NULL): min over variants of
 * 1 - r (the first variant on ties, as Python's min).  Scratch: gsr_pearson_scratch_bytes; the
 * backward reuses it. */
size_t gsr_pearson_scratch_bytes(int K, int variants);
int gsr_pearson_loss(int64_t N, int K, const float* x, const float* y, int variants, float offset,
                     float* out_r, float* out_loss, void* scratch, void* stream);
/* grad_y (and, variants = 1 only, grad_x) of sum_k grad_loss[k] * out_loss[k]; grad_loss device
 * [K] (NULL = ones); grad_y / grad_x may be NULL. */
int gsr_pearson_loss_backward(int64_t N, int K, const float* x, const float* y, int variants,
                              float offset, const float* grad_loss, float* grad_y, float* grad_x,
                              void* scratch, void* stream);

/* One training view's loss (train.py:99-131 with the depth branch), forward in two launches and
 * backward in one: total = (1 - lambda) L1 + lambda (1 - SSIM) of image vs gt, plus depth_weight *
 * min over {mono, 1 / (offset - mono)} of 1 - pearson(., depth) (the depth term of
 * gsr_pearson_loss with K = 1, variants = 2; single-pass shifted sums in double, same r to double
 * rounding).  image, gt [C,H,W]; depth, depth_mono [N].  out (device, 5 floats): photometric
 * loss, L1, SSIM, depth term, total; total (device, 1 float): the total again, a separate
 * tensor for autograd.  Scratch: gsr_view_loss_scratch_bytes, shared by forward and backward. */
size_t gsr_view_loss_scratch_bytes(int C, int H, int W);
int gsr_view_loss(int C, int H, int W, const float* image, const float* gt, float lambda_dssim,
                  int64_t N, const float* depth, const float* depth_mono, float offset,
                  float depth_weight, int need_grad, float* out, float* total, void* scratch,
                  void* stream);
/* grad_image, grad_depth of grad_total * total (grad_total: device scalar); needs the scratch of a
 * need_grad forward on the same inputs. */
int gsr_view_loss_backward(int C, int H, int W, const float* image, const float* gt,
                           float lambda_dssim, int64_t N, const float* depth,
                           const float* depth_mono, float offset, float depth_weight,
                           const float* grad_total, float* grad_image, float* grad_depth,
                           void* scratch, void* stream);
/* Up to 8 views of one training step in one launch per stage (the multi-view training step):
 * images [V][C][H][W] and depths [V][N] back to back (the multi-view call's stacked outputs), one
 * gt / depth_mono pointer per view, out [V][5], total [V], scratch V x
 * gsr_view_loss_scratch_bytes(C, H, W); per view the outputs and gradients of gsr_view_loss /
 * gsr_view_loss_backward, bit for bit (grad_total [V]: one scalar per view). */
int gsr_view_loss_views(int V, int C, int H, int W, const float* images, const float* const* gts,
                        float lambda_dssim, int64_t N, const float* depths,
                        const float* const* depth_monos, float offset, float depth_weight,
                        int need_grad, float* out, float* total, void* scratch, void* stream);
int gsr_view_loss_views_backward(int V, int C, int H, int W, const float* images,
                                 const float* const* gts, float lambda_dssim, int64_t N,
                                 const float* depths, const float* const* depth_monos,
                                 float offset, float depth_weight, const float* grad_total,
                                 float* grad_images, float* grad_depths, void* scratch,
                                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_LOSS_H */

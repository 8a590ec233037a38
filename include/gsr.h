/*
 * gsr.h -- C ABI of libgsr, the MI355X (gfx950) differentiable Gaussian rasterizer.
 *
 * This is the drop-in boundary that replaces the reference's pybind11 module `_C`
 * (submodules/diff-gaussian-rasterization/ext.cpp:15-19) and its libtorch glue
 * (rasterize_points.cu:27-217).  Plain pointers and sizes only: no torch types cross it.
 *
 * Conventions (identical to the reference binding):
 *  - every tensor is float32 (radii int32), C-contiguous, on the current HIP device;
 *  - a NULL pointer means "empty tensor" (the reference passes data_ptr() of torch.Tensor([]),
 *    i.e. nullptr: rasterize_points.cu:84-110, rasterizer_impl.cu:229-232,321,389,411);
 *  - images are planar [C,H,W];  the 4x4 matrices are the reference's row-major tensors
 *    world_view_transform / full_proj_transform (scene/cameras.py:76-81);
 *  - all work is enqueued on `stream` (a hipStream_t, NULL = legacy default stream); the forward
 *    performs one 12-byte device->host read of the instance counts (as rasterizer_impl.cu:281 does);
 *  - scratch memory is owned by the caller: the library requests it through `alloc`, mirroring
 *    resizeFunctional (rasterize_points.cu:27-33); `which` is GSR_BUF_GEOM / _BINNING / _IMAGE.
 *    The three buffers must be handed back unchanged to the backward;
 *  - errors are reported as a non-zero gsr_status; gsr_last_error() gives a message
 *    (thread-local).  No C++ exception crosses the ABI.
 *
 * Extended outputs (depth / alpha / language feature / confidence) follow DESIGN.md section 3.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 1

typedef enum gsr_status {
  GSR_OK = 0,
  GSR_ERR_ARGUMENT = 1,     /* shape / pointer / alignment validation (rasterize_points.cu:57-59) */
  GSR_ERR_HIP = 2,          /* a HIP runtime call or kernel launch failed */
  GSR_ERR_ALLOC = 3,        /* the allocator callback returned NULL */
  GSR_ERR_PREFILTERED = 4,  /* a Gaussian was culled although prefiltered was set (auxiliary.h:156-160) */
  GSR_ERR_TOO_LARGE = 5,    /* problem exceeds the scan/sort capacity */
  GSR_ERR_SORT = 6          /* a sort of this call gave up (bounded look-back) or an id was out of
                             * range: the call's outputs / gradients are NaN-poisoned (the
                             * reference traps instead, auxiliary.h:156-160) */
} gsr_status;

enum { GSR_BUF_GEOM = 0, GSR_BUF_BINNING = 1, GSR_BUF_IMAGE = 2 };

/* `debug` argument of every rasterize entry point: bit 0 = the reference's debug flag (synchronous
 * checks, rasterize_points.cu `debug`); bit 1 = deterministic backward -- the blend backward
 * writes per-instance gradient rows and sums every Gaussian's rows in a fixed order instead of
 * float atomics (the reference's backward.cu:523-554 atomics are run-to-run nondeterministic), so
 * gradients are bitwise reproducible; slower, and its binning buffer holds two more arrays.  A
 * backward must get the same bit 1 as its forward. */
#define GSR_DEBUG_DETERMINISTIC 2
/* Backward only, bit 2: take the layout (deterministic or not, per-instance rows or atomics) from
 * the tag word the forward wrote into its binning buffer instead of from bit 1 -- for callers
 * that keep only the buffers (the reference's `_C.rasterize_gaussians_backward` signature carries
 * just `debug`).  Costs one synchronous 4-byte read. */
#define GSR_DEBUG_LAYOUT_FROM_BUFFER 4

/* Returns a device pointer to at least `bytes` bytes (16-byte aligned) or NULL. */
typedef void* (*gsr_alloc_fn)(void* ctx, size_t bytes, int which);

int gsr_abi_version(void);
const char* gsr_last_error(void);

/* Status of the forward that used `image_buffer` (GSR_OK or GSR_ERR_SORT with gsr_last_error()).
 * The reference __trap()s on an invalid state inside the call (auxiliary.h:156-160); here the
 * one-sweep sorts bound their look-back spin, and a call whose sort gave up -- or whose blend had
 * to clamp an out-of-range id -- is failed: its outputs and gradients are NaN on the device, its
 * backward returns GSR_ERR_SORT once the status is published (checked on entry without a wait),
 * and these checks report it.  wait != 0 blocks until that forward has finished. */
int gsr_forward_status(const void* image_buffer, int wait);
/* The same over every forward not yet checked (on any stream of this process), plus failures of
 * forwards whose mailbox was recycled unchecked.  wait != 0 blocks until they have finished. */
int gsr_check_forwards(int wait);

/* Forward.  Replaces _C.rasterize_gaussians -> RasterizeGaussiansCUDA (rasterize_points.cu:35-115)
 * -> CudaRasterizer::Rasterizer::forward (rasterizer_impl.cu:198-336); argument order follows the
 * reference, the extended-API inputs/outputs are appended.  M = sh.size(1) (0 without SH).
 * Outputs: out_color[3,H,W] (= blend + T*bg), out_depth[1,H,W], out_alpha[1,H,W],
 * out_feature[3,H,W] (zeros unless include_feature), radii[P] (NULL -> internal),
 * *num_rendered (the reference's first return value, with its meaning: the sum over the Gaussians
 * of the tiles in their full 3-sigma rectangles, forward.cu:255 + rasterizer_impl.cu:281; the
 * binning buffer is sized for that many instances).  The library bins only the tiles of those
 * rectangles where the splat can reach alpha >= 1/255 ("exact tile culling"; no
 * output or gradient changes) -- gsr_last_forward_instances() gives that count.  With P == 0 nothing is written except
 * *num_rendered = 0 and out_* are zero-filled (the reference returns its zero-initialised tensors). */
int gsr_rasterize_gaussians(
    int P, int M,
    const float* background, const float* means3D, const float* colors_precomp,
    const float* opacities, const float* scales, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
    float tan_fovx, float tan_fovy, int image_height, int image_width,
    const float* sh, int degree, const float* campos, int prefiltered,
    const float* sh_language, const float* language_feature_precomp, const float* confidence,
    int include_feature,
    float* out_color, float* out_depth, float* out_alpha, float* out_feature, int* radii,
    int* num_rendered,
    gsr_alloc_fn alloc, void* alloc_ctx,
    void* stream, int debug);

/* Tile instances binned by the last forward on this host thread (<= its num_rendered: the
 * instances of the reference's list that can contribute).  0 before any forward. */
int gsr_last_forward_instances(void);

/* Sticky per-device fault word: the kStatus bits (1 depth sort, 2 tile sort, 4 clamped id) of
 * every forward on the current device that failed since the last reset.  While it is non-zero,
 * gsr_adam_step (gsr_optim.h) leaves parameters and moments unchanged, so the NaN gradients of a
 * failed call cannot reach them (the reference __trap()s instead).  gsr_forward_faults() reads it
 * (synchronously; -1 on a HIP error), gsr_reset_forward_faults() clears it (0 = ok). */
int gsr_forward_faults(void);
int gsr_reset_forward_faults(void);

/* Backward.  Replaces _C.rasterize_gaussians_backward -> RasterizeGaussiansBackwardCUDA
 * (rasterize_points.cu:117-196) -> CudaRasterizer::Rasterizer::backward (rasterizer_impl.cu:340-434).
 * R is the forward's num_rendered; geom/binning/image are the buffers the forward allocated.
 * Upstream grads dL_dout_depth / _alpha / _feature may be NULL (== zeros).
 * Every element of every non-NULL grad output is written (culled Gaussians get zeros):
 *   dL_dmeans2D[P,3] (NDC-scaled x,y; z = 0), dL_dcolors[P,3] (may be NULL), dL_dopacity[P],
 *   dL_dmeans3D[P,3], dL_dcov3D[P,6] (may be NULL), dL_dsh[P,M,3] (required iff sh),
 *   dL_dscales[P,3] / dL_drotations[P,4] (required iff scales), dL_dsh_language[P,3],
 *   dL_dlanguage_feature[P,3]. */
int gsr_rasterize_gaussians_backward(
    int P, int M, int R,
    const float* background, const float* means3D, const int* radii, const float* colors_precomp,
    const float* scales, const float* rotations, float scale_modifier, const float* cov3D_precomp,
    const float* viewmatrix, const float* projmatrix, float tan_fovx, float tan_fovy,
    int image_height, int image_width,
    const float* dL_dout_color, const float* dL_dout_depth, const float* dL_dout_alpha,
    const float* dL_dout_feature,
    const float* sh, int degree, const float* campos,
    const float* sh_language, const float* language_feature_precomp, const float* confidence,
    int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer,
    float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
    float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations,
    float* dL_dsh_language, float* dL_dlanguage_feature,
    void* stream, int debug);

/* Fused-activation forward.  Same rasterization as gsr_rasterize_gaussians for the
 * render() configuration that the reference runs by default (pipe.convert_SHs_python = False,
 * pipe.compute_cov3D_python = False, override_color/override_language = None;
 * gaussian_renderer/__init__.py:209-290), but reading GaussianModel's raw leaves directly:
 *   features_dc[P,1,3], features_rest[P,M-1,3]   (instead of get_features = cat(...),
 *                                                  scene/gaussian_model.py:159-162)
 *   opacity_raw[P]      sigmoid in-kernel          (get_opacity, gaussian_model.py:38,172-173)
 *   scaling_raw[P,3]    exp in-kernel              (get_scaling, gaussian_model.py:33,147-148)
 *   rotation_raw[P,4]   normalize in-kernel        (get_rotation, gaussian_model.py:41,151-152;
 *                                                  r / max(|r|, 1e-12) as F.normalize)
 *   language_feature[P,3]  = shs_language           (get_language_feature, :175)
 * Removes the cat/activation kernels PyTorch would launch around every view.  Outputs as above. */
int gsr_rasterize_gaussians_fused(
    int P, int M,
    const float* background, const float* means3D,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    const float* viewmatrix, const float* projmatrix,
    float tan_fovx, float tan_fovy, int image_height, int image_width,
    int degree, const float* campos, int prefiltered,
    const float* language_feature, const float* confidence, int include_feature,
    float* out_color, float* out_depth, float* out_alpha, float* out_feature, int* radii,
    int* num_rendered,
    gsr_alloc_fn alloc, void* alloc_ctx,
    void* stream, int debug);

/* Backward of gsr_rasterize_gaussians_fused: writes the gradients of the raw leaves
 * (the chain through sigmoid / exp / normalize / cat is applied in-kernel).
 * accumulate = 0: every element written (zeros for culled Gaussians), as the plain backward.
 * accumulate = 1: visible Gaussians' grads are ADDED into the buffers and culled ones are left
 *   untouched, so the buffers may be the leaves' .grad tensors across views of one step.
 * dL_dmeans2D[P,3] is the screen-space gradient (the reference's means2D.grad): a per-call
 * output, always stored (zeros for culled Gaussians), also when accumulate = 1. */
int gsr_rasterize_gaussians_fused_backward(
    int P, int M, int R,
    const float* background, const float* means3D, const int* radii,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    const float* viewmatrix, const float* projmatrix, float tan_fovx, float tan_fovy,
    int image_height, int image_width,
    const float* dL_dout_color, const float* dL_dout_depth, const float* dL_dout_alpha,
    const float* dL_dout_feature,
    int degree, const float* campos,
    const float* language_feature, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer,
    float* dL_dmeans2D, float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
    float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
    float* dL_dlanguage_feature, int accumulate,
    void* stream, int debug);

/* Deferred SH gradients for multi-view steps (gsr_amd/pipeline.py; no reference counterpart: the
 * reference steps after every view).  Same as gsr_rasterize_gaussians_fused_backward, but when
 * dL_dcolor_sh != NULL the SH gradients are NOT written (dL_dfeatures_dc / _rest may be NULL);
 * instead the clamp-masked colour gradient dL/dRGB of every Gaussian (planar [3][P], zeros when
 * culled) is stored there.  The SH gradient is basis(dir) x dL/dRGB (backward.cu:20-139), so
 * gsr_sh_grad_flush forms it for all deferred views of a step in one pass over the SH rows.
 * pre_jac (optional, needs dL_dcolor_sh): this view's colour Jacobian from gsr_sh_precolor; the
 * SH rows are then not read. */
int gsr_rasterize_gaussians_fused_backward_deferred(
    int P, int M, int R,
    const float* background, const float* means3D, const int* radii,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    const float* viewmatrix, const float* projmatrix, float tan_fovx, float tan_fovy,
    int image_height, int image_width,
    const float* dL_dout_color, const float* dL_dout_depth, const float* dL_dout_alpha,
    const float* dL_dout_feature,
    int degree, const float* campos,
    const float* language_feature, const float* confidence, int include_feature,
    void* geom_buffer, void* binning_buffer, void* image_buffer,
    float* dL_dmeans2D, float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
    float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
    float* dL_dlanguage_feature, float* dL_dcolor_sh, const float* pre_jac, int accumulate,
    void* stream, int debug);

/* Multi-view colour pre-pass (gsr_amd/pipeline.py): for nviews cameras, one pass over the SH
 * rows writes per view the fused forward's colour clamp(SH(dir) + 0.5) (forward.cu:20-71), its
 * clamp bits [P] (u8) and the colour's direction Jacobian dRGB/d(dir_x, dir_y, dir_z)
 * (backward.cu:56-131), colour and Jacobian PLANAR: color[c * P + i] ([3][P]) and
 * jac[(3 * r + c) * P + i] = d colour_c / d dir_r ([9][P]).  campos / color / clamped / jac: HOST arrays of nviews DEVICE pointers.
 * Either part may be skipped: color and clamped both NULL (the Jacobian only), or jac NULL (the
 * colour only) -- the forward needs the colour before it starts, the Jacobian only its backward. */
int gsr_sh_precolor(int P, int M, int degree, const float* means3D, const float* features_dc,
                    const float* features_rest, int nviews, const float* const* campos,
                    float* const* color, uint8_t* const* clamped, float* const* jac, void* stream);
/* gsr_sh_precolor for the Gaussian rows [row0, row1) only (outputs stay planes of P): the next
 * step's pre-pass issued slice by slice behind the optimizer's row slices (a multi-GPU step,
 * gsr_amd.trainer.train_step_views).  Rows outside the range are not touched. */
int gsr_sh_precolor_rows(int P, int row0, int row1, int M, int degree, const float* means3D,
                         const float* features_dc, const float* features_rest, int nviews,
                         const float* const* campos, float* const* color,
                         uint8_t* const* clamped, float* const* jac, void* stream);

/* gsr_rasterize_gaussians_fused with the SH colour and clamp bits of this view taken from
 * gsr_sh_precolor (identical outputs; the SH rows are not read). */
int gsr_rasterize_gaussians_fused_precolor(
    int P, int M, const float* background, const float* means3D, const float* features_dc,
    const float* features_rest, const float* opacity_raw, const float* scaling_raw,
    const float* rotation_raw, float scale_modifier, const float* viewmatrix,
    const float* projmatrix, float tan_fovx, float tan_fovy, int image_height, int image_width,
    int degree, const float* campos, int prefiltered, const float* language_feature,
    const float* confidence, int include_feature, const float* pre_color,
    const uint8_t* pre_clamp, float* out_color, float* out_depth, float* out_alpha,
    float* out_feature, int* radii, int* num_rendered, gsr_alloc_fn alloc, void* alloc_ctx,
    void* stream, int debug);

/* dL/dfeatures_dc [P,1,3] and dL/dfeatures_rest [P,M-1,3] of nviews deferred views:
 * sum_v basis(normalize(means3D - campos[v])) x dL_dcolor_sh[v], coefficients above `degree`
 * zero; stored (accumulate = 0) or added (accumulate = 1).  campos / dL_dcolor_sh: HOST arrays
 * of nviews DEVICE pointers ([3] and planar dL/dRGB: channel c of Gaussian i at
 * dL_dcolor_sh[v][c * rgb_plane_stride + i], rgb_plane_stride >= P, so a row slice [a, b) of a
 * [3][P_total] plane is the pointer + a with the full stride).  Views are summed in order in
 * registers. */
int gsr_sh_grad_flush(int P, int M, int degree, const float* means3D, int nviews,
                      const float* const* campos, const float* const* dL_dcolor_sh,
                      int64_t rgb_plane_stride, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
                      int accumulate, void* stream);

/* ---- multi-view calls (no reference counterpart: a step of several views in one host call) ----
 * One camera of gsr_rasterize_views_fused / _backward.  The forward fills the scratch pointers
 * and counts; the backward reads them back unchanged.  The per-view fields mean what the
 * single-view entry points' arguments of the same names mean. */
typedef struct gsr_view {
  /* camera */
  const float* viewmatrix; const float* projmatrix; const float* campos;
  float tan_fovx, tan_fovy;
  /* optional colour pre-pass of this view (gsr_sh_precolor): both or neither */
  const float* pre_color; const uint8_t* pre_clamp;
  /* forward outputs: [3,H,W], [1,H,W], [1,H,W], [3,H,W] (may be NULL as in the single-view
   * call, except out_color), radii[P] (NULL -> internal) */
  float* out_color; float* out_depth; float* out_alpha; float* out_feature; int* radii;
  /* scratch of this view: requested by the forward through alloc(alloc_ctx, bytes, which) */
  void* alloc_ctx;
  void* geom_buffer; void* binning_buffer; void* image_buffer;   /* set by the forward */
  int num_rendered;    /* set by the forward: the reference's count (as *num_rendered) */
  int num_instances;   /* set by the forward: instances binned (gsr_last_forward_instances) */
  /* HIP stream of this view's work (NULL = the call's stream) */
  void* stream;
  /* backward: upstream gradients (depth / alpha / feature may be NULL), the screen-space
   * gradient dL_dmeans2D[P,3] (always stored), and -- deferred SH gradients -- the planar
   * dL/dRGB [3][P] this view stores (NULL: the SH gradients are added directly) with the
   * pre-pass Jacobian pre_jac (optional).  pre_jac without dL_dcolor_sh, in every view of a
   * call of at most 8 views: the call's single per-Gaussian launch forms the SH gradients itself
   * from the views' dL/dRGB (the deferred path's flush fused: same values, no [3][P] planes) */
  const float* dL_dout_color; const float* dL_dout_depth; const float* dL_dout_alpha;
  const float* dL_dout_feature;
  float* dL_dmeans2D; float* dL_dcolor_sh; const float* pre_jac;
} gsr_view;

/* Fused forward of V views of the same Gaussians (gsr_rasterize_gaussians_fused per view, same
 * outputs bit for bit) issued from one host call: the first phase of up to `inflight` views
 * (preprocess, depth sort, scan and the instance-count read-back) is queued ahead of the views'
 * binning, so the host's wait for a view's read-back finds it done and every view stream stays
 * fed.  View v's preprocess and binning run on views[v].stream (which first waits for `stream`,
 * the call's stream); the blends of consecutive groups of views (up to 8 per group) run merged
 * into one launch each on `stream`, which is ordered after every view's work on return. */
int gsr_rasterize_views_fused(
    int V, gsr_view* views, int image_height, int image_width,
    int P, int M, const float* background, const float* means3D,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    int degree, int prefiltered, const float* language_feature, const float* confidence,
    int include_feature, gsr_alloc_fn alloc, int inflight, void* stream, int debug);

/* Backward of gsr_rasterize_views_fused: the views' blend backwards merged into launches of up to
 * 8 views on views[0].stream (after the call's `stream`, where the upstream gradients were
 * produced), and the views' per-Gaussian backwards in view order on `stream`, adding into the
 * raw leaves' gradients exactly as
 * consecutive gsr_rasterize_gaussians_fused_backward[_deferred] calls with accumulate = 1 for
 * every view after the first (the first uses `accumulate`).  With views[v].dL_dcolor_sh set the
 * SH gradients are deferred (dL_dfeatures_dc / _rest may be NULL); with pre_jac and no
 * dL_dcolor_sh they are formed in the per-Gaussian launch (gsr_view). */
int gsr_rasterize_views_fused_backward(
    int V, const gsr_view* views, int image_height, int image_width,
    int P, int M, const float* background, const float* means3D,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    int degree, const float* language_feature, const float* confidence, int include_feature,
    float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
    float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
    float* dL_dlanguage_feature, int accumulate, void* stream, int debug);

/* Called by the sliced backward below after the per-Gaussian backward of rows [row_begin,
 * row_end) has been enqueued on the call's stream (every leaf gradient of those rows is final
 * once that work runs).  Runs on the calling thread, inside the call. */
typedef void (*gsr_rows_fn)(void* ctx, int row_begin, int row_end);

/* gsr_rasterize_views_fused_backward with the per-Gaussian backward issued in row slices of
 * slice_rows (a multiple of 256; 0 = one slice) and on_rows(ctx, a, b) called after each slice
 * (after the single launch when 0; for [0, P) when the merged launch is not available): a
 * multi-GPU caller starts the slice's gradient all-reduce there while the next slice computes
 * (gsr_amd.pipeline).  Results are identical to the unsliced call. */
int gsr_rasterize_views_fused_backward_sliced(
    int V, const gsr_view* views, int image_height, int image_width,
    int P, int M, const float* background, const float* means3D,
    const float* features_dc, const float* features_rest, const float* opacity_raw,
    const float* scaling_raw, const float* rotation_raw, float scale_modifier,
    int degree, const float* language_feature, const float* confidence, int include_feature,
    float* dL_dmeans3D, float* dL_dfeatures_dc, float* dL_dfeatures_rest,
    float* dL_dopacity_raw, float* dL_dscaling_raw, float* dL_drotation_raw,
    float* dL_dlanguage_feature, int accumulate, void* stream, int debug, int slice_rows,
    gsr_rows_fn on_rows, void* rows_ctx);

/* Replaces _C.mark_visible -> markVisible (rasterize_points.cu:198-217) -> checkFrustum
 * (rasterizer_impl.cu:54-66): present[i] = view-space z > 0.2 (bool as uint8). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/* Byte sizes of the three scratch buffers (for callers that pre-allocate).  R = num_rendered;
 * gsr_binning_buffer_bytes_det: the same with the deterministic backward (GSR_DEBUG_DETERMINISTIC),
 * whose binning buffer holds two more per-instance arrays. */
size_t gsr_geom_buffer_bytes(int P);
size_t gsr_binning_buffer_bytes(int R);
size_t gsr_binning_buffer_bytes_det(int R);
size_t gsr_image_buffer_bytes(int image_height, int image_width);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */

/*
 * gsr_oracle.h -- CPU restatement of the reference differentiable Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline.  The product path
 * (sdp-gs_amd/) never links, loads or calls it.
 *
 * What it restates (all citations relative to /root/reference/submodules/diff-gaussian-rasterization):
 *   forward : Rasterizer::forward            cuda_rasterizer/rasterizer_impl.cu:198-336
 *             preprocessCUDA (fwd)           cuda_rasterizer/forward.cu:155-256
 *             duplicateWithKeys + SortPairs  cuda_rasterizer/rasterizer_impl.cu:70-111, 300-318
 *             renderCUDA (fwd)               cuda_rasterizer/forward.cu:261-374
 *   backward: Rasterizer::backward           cuda_rasterizer/rasterizer_impl.cu:340-434
 *             renderCUDA (bwd)               cuda_rasterizer/backward.cu:399-557
 *             computeCov2DCUDA               cuda_rasterizer/backward.cu:144-274
 *             preprocessCUDA (bwd)           cuda_rasterizer/backward.cu:346-396
 *   visible : checkFrustum / in_frustum      rasterizer_impl.cu:54-66, auxiliary.h:139-164
 *
 * Extended outputs (depth / alpha / language feature / confidence) are not in the reference
 * tree; they are defined in DESIGN.md section 3 and restated
 * here as extra blend channels on the reference's blend arithmetic.
 *
 * Arithmetic: float32, reference expression order, glm column-major conventions, compiled
 * with -ffp-contract=off (no silent FMA contraction); ndc2Pix in double as auxiliary.h:41-44;
 * the blend's exp(power) is splat_exp, the deterministic float exp the HIP kernels also use.
 * Deterministic: single-threaded by default (the reference's sequential order);
 * oracle_set_threads(n) splits the loops into n fixed chunks (forward bit-identical; backward
 * sums per chunk, added in chunk order) for the full-size tests and the CPU baseline.
 */
#ifndef GSR_ORACLE_H
#define GSR_ORACLE_H

#include <stdint.h>

/* The restatement's arithmetic type: float (the checker) or double (-DORACLE_REAL=double, the
 * float64 build used to show that the float32 results differ only by rounding).  Output images
 * and gradients are written in this type; inputs are the reference's float32 tensors. */
#ifndef ORACLE_REAL
#define ORACLE_REAL float
#endif
typedef ORACLE_REAL oreal;

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_state oracle_state;

/* Host threads used by oracle_forward / oracle_backward (1 = sequential, the default). */
void oracle_set_threads(int n);
int oracle_get_threads(void);

/* Forward.  Argument order mirrors _C.rasterize_gaussians (rasterize_points.cu:35-55) plus the
 * extended-API inputs.  NULL means "empty tensor" exactly like the reference's nullptr
 * convention (rasterize_points.cu:84-110, rasterizer_impl.cu:229-232,321).  Output images are
 * planar [C,H,W].  Returns a state handle consumed by oracle_backward (NULL on error). */
oracle_state* oracle_forward(
    int P, int M,
    const float* background,                 /* [3] */
    const float* means3D,                    /* [P,3] */
    const float* colors_precomp,             /* [P,3] or NULL */
    const float* opacities,                  /* [P] */
    const float* scales,                     /* [P,3] or NULL */
    const float* rotations,                  /* [P,4] or NULL */
    float scale_modifier,
    const float* cov3D_precomp,              /* [P,6] or NULL */
    const float* viewmatrix,                 /* [16] */
    const float* projmatrix,                 /* [16] */
    float tan_fovx, float tan_fovy,
    int image_height, int image_width,
    const float* sh,                         /* [P,M,3] or NULL */
    int degree,
    const float* campos,                     /* [3] */
    int prefiltered,
    const float* sh_language,                /* [P,3] or NULL */
    const float* language_feature_precomp,   /* [P,3] or NULL */
    const float* confidence,                 /* [P] or NULL (== all ones) */
    int include_feature,
    oreal* out_color,                        /* [3,H,W] */
    oreal* out_depth,                        /* [1,H,W] */
    oreal* out_alpha,                        /* [1,H,W] */
    oreal* out_feature,                      /* [3,H,W] */
    int* radii,                              /* [P] */
    int* num_rendered);

/* Backward.  Consumes the forward state; upstream grads may be NULL (== zeros).
 * Every grad buffer that is non-NULL is fully written. */
int oracle_backward(
    oracle_state* st,
    const float* dL_dout_color,              /* [3,H,W] */
    const float* dL_dout_depth,              /* [1,H,W] or NULL */
    const float* dL_dout_alpha,              /* [1,H,W] or NULL */
    const float* dL_dout_feature,            /* [3,H,W] or NULL */
    oreal* dL_dmeans2D,                      /* [P,3] */
    oreal* dL_dcolors,                       /* [P,3] */
    oreal* dL_dopacity,                      /* [P] */
    oreal* dL_dmeans3D,                      /* [P,3] */
    oreal* dL_dcov3D,                        /* [P,6] */
    oreal* dL_dsh,                           /* [P,M,3] or NULL */
    oreal* dL_dscales,                       /* [P,3] or NULL */
    oreal* dL_drotations,                    /* [P,4] or NULL */
    oreal* dL_dsh_language,                  /* [P,3] or NULL */
    oreal* dL_dlanguage_feature);            /* [P,3] or NULL */

/* The backward in two parts, for the float64 rounding analysis (tests/test_f64_parity.py).
 * rows: [15*P] in the oracle's accumulator layout -- colours [P,3] | depth [P] | feature [P,3] |
 * means2D [P,3] | conic [P,4] (a, b, -, c) | opacity [P].
 * oracle_blend_rows: the blend backward's per-Gaussian sums (renderCUDA bwd); with mass != 0 each
 * entry is instead the sum of the ABSOLUTE values of its per-pixel terms (dL/dalpha replaced by
 * the sum of its channel terms' absolute values): the scale of the rounding error any float32
 * evaluation of the sum can make.
 * oracle_backward_rows: the per-Gaussian backward (preprocess bwd) from given rows; linear in the
 * rows, so unit rows give its Jacobian.  Outputs as oracle_backward. */
int oracle_blend_rows(oracle_state* st, const float* dL_dout_color, const float* dL_dout_depth,
                      const float* dL_dout_alpha, const float* dL_dout_feature, int mass,
                      oreal* rows);
int oracle_backward_rows(oracle_state* st, const oreal* rows, oreal* dL_dmeans2D,
                         oreal* dL_dcolors, oreal* dL_dopacity, oreal* dL_dmeans3D,
                         oreal* dL_dcov3D, oreal* dL_dsh, oreal* dL_dscales,
                         oreal* dL_drotations, oreal* dL_dsh_language,
                         oreal* dL_dlanguage_feature);

/* The next oracle_forward on the calling thread uses these instance lists (point_list [R],
 * ranges [tiles*2], as oracle_get_point_list / _ranges return them) instead of binning; NULL
 * point_list = bin normally again.  Test diagnostic: the float64 build on the float32 lists. */
void oracle_use_lists(const unsigned* point_list, int R, const unsigned* ranges);
/* The next oracle_forward on this thread blends with these per-pixel decisions (another
 * evaluation's oracle_accept_bits) instead of its own threshold tests (float64 parity). */
void oracle_use_decisions(const unsigned* n_contrib, const uint64_t* word_offsets,
                          const unsigned* words);
/* Per pixel: word offsets (H*W + 1) of the bitsets of the list positions the forward blended;
 * with words != NULL also the bitsets.  Returns the number of 32-bit words. */
long oracle_accept_bits(const oracle_state* st, uint64_t* offs, unsigned* words);
/* The next oracle_forward on this thread takes another evaluation's SH colour clamp bits [P*3]
 * (oracle_get_clamped) instead of its own result < 0 tests (float64 parity). */
void oracle_use_clamp(const unsigned char* clamped);
/* The next oracle_forward on this thread blends with another evaluation's screen means [P*2]
 * and conic + opacity [P*4] instead of its own preprocess's (float64 parity). */
void oracle_use_geometry(const float* means2D, const float* conic_opacity);
int oracle_get_clamped(const oracle_state* st, unsigned char* out);

void oracle_free(oracle_state* st);

int oracle_mark_visible(int P, const float* means3D, const float* viewmatrix,
                        const float* projmatrix, unsigned char* present);

/* Introspection for parity tests (copies internal state out). */
int oracle_get_point_list(const oracle_state* st, unsigned* out);   /* [num_rendered] */
int oracle_get_ranges(const oracle_state* st, unsigned* out);       /* [tiles*2] */
/* point_list / ranges with the HIP build's exact tile cull applied (gsr_oracle.c); returns the
 * instances kept.  point_list_out holds num_rendered entries, ranges_out tiles*2. */
int oracle_cut_lists(const oracle_state* st, unsigned* point_list_out, unsigned* ranges_out);
void oracle_splat_log(long n, const float* x, float* out);
int oracle_get_final_T(const oracle_state* st, float* out);         /* [H*W] */
int oracle_get_n_contrib(const oracle_state* st, unsigned* out);    /* [H*W] */
/* [H*W] min relative distance of the pixel's blend decisions from alpha = 1/255 and
 * T = 1e-4 (test diagnostic: where two correct float evaluations may decide differently) */
int oracle_get_margin(const oracle_state* st, float* out);
int oracle_get_means2D(const oracle_state* st, float* out);         /* [P*2] */
int oracle_get_conic_opacity(const oracle_state* st, float* out);   /* [P*4] */
int oracle_get_depths(const oracle_state* st, float* out);          /* [P] */
int oracle_get_rgb(const oracle_state* st, float* out);             /* [P*3] */
int oracle_get_tiles_touched(const oracle_state* st, unsigned* out);/* [P] */
int oracle_get_cov3D(const oracle_state* st, float* out);           /* [P*6] */
/* [P][13] doubles: x_px, y_px, conic a b c, opacity, depth, rgb, feature (the build's precision) */
int oracle_get_preprocess_f64(const oracle_state* st, double* out);

/* The blend's exp(power): the deterministic single-precision exp shared with the HIP kernels. */
void oracle_splat_exp(long n, const float* x, float* out);

/* distCUDA2 (simple_knn, un-vendored; scene/gaussian_model.py:20,198,514) by brute force:
 * gsr_oracle_knn.c.  pts [P,3]; mean [P]; idx [P,3] or NULL. */
void oracle_dist_knn3(int64_t P, const float* pts, float* mean, int32_t* idx);

#ifdef __cplusplus
}
#endif
#endif

/*
 * gsr_optim.h -- C ABI of libgsr's fused optimizer step.
 *
 * Replaces the torch.optim.Adam step that train.py runs after every backward
 * (train.py:229-231) over GaussianModel's parameter groups (scene/gaussian_model.py:217-271:
 * Adam(groups, lr=0.0, eps=1e-15), one tensor per group).  The optimizer state stays in the
 * caller's tensors (PyTorch's Adam state dict: exp_avg, exp_avg_sq, step), so the reference's
 * densification code that edits optimizer.state (gaussian_model.py:400-470) keeps working.
 */
#ifndef GSR_OPTIM_H
#define GSR_OPTIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ADAM_MAX_TENSORS 16

/* One Adam step over n_tensors float32 tensors in ONE launch (non-amsgrad, L2 weight decay).
 * params/grads/exp_avg/exp_avg_sq[t]: device pointers to numel[t] contiguous floats;
 * lr[t], weight_decay[t]: the tensor's group hyper-parameters; step[t]: the step count AFTER
 * increment (>= 1).  Arithmetic and host scalars follow torch.optim.adam._multi_tensor_adam.
 * Guard: a one-lane launch first snapshots the device's forward fault word (gsr.h
 * gsr_forward_faults: a rasterizer forward failed and its gradients are NaN) into a device slot,
 * and while that snapshot is set the Adam launch leaves every parameter and moment unchanged --
 * decided on the device, no host synchronisation, one decision for every tensor of the step.
 * Returns 0 on success, 1 on invalid arguments, 2 on a launch error. */
int gsr_adam_step(int n_tensors, float* const* params, const float* const* grads,
                  float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                  const double* lr, const double* weight_decay, const double* step,
                  double beta1, double beta2, double eps, void* stream);

/* slot[0] = 1.0f if the device's forward fault word is set, else 0.0f (one lane, on stream).
 * A float so that a multi-GPU caller can put the slot in its gradient all-reduce buffer: after a
 * SUM over the ranks, slot != 0 means some rank's forward failed, and every rank then skips the
 * step (the summed gradients carry that rank's NaNs).  0 ok, 1 NULL slot, 2 launch error. */
int gsr_step_guard(float* slot, void* stream);

/* gsr_adam_step with an explicit skip decision: the step is skipped when *skip != 0 (device
 * float written earlier on `stream`, e.g. gsr_step_guard's slot after the all-reduce); skip NULL
 * = snapshot the device's fault word as gsr_adam_step does.  host_skipped (pinned host memory or
 * NULL) receives 1 if the launch skipped the step, 0 if it applied it, so the caller can learn
 * about a skip without synchronising (and roll back its step counters, gsr_amd.optim). */
int gsr_adam_step_guarded(int n_tensors, float* const* params, const float* const* grads,
                          float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                          const double* lr, const double* weight_decay, const double* step,
                          double beta1, double beta2, double eps, const float* skip,
                          uint32_t* host_skipped, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_OPTIM_H */

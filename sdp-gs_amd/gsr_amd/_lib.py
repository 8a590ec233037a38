"""ctypes binding of libgsr.so (include/gsr.h), the hand-written gfx950 rasterizer.

There is no CPU fallback: if the shared library is missing or the tensors are not on a HIP device
the calls raise.  `import torch` happens first so that libgsr resolves libamdhip64.so.7 to the HIP
runtime torch already loaded (same soname), which makes torch's hipStream_t valid here.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# GSR_LIB_PATH selects an alternative in-tree build (A/B experiments of compile flags)
LIB_PATH = os.environ.get("GSR_LIB_PATH") or os.path.join(_HERE, "libgsr.so")

_f = ctypes.c_float
_i = ctypes.c_int
_p = ctypes.c_void_p
_sz = ctypes.c_size_t

ALLOC_FN = ctypes.CFUNCTYPE(_p, _p, _sz, _i)

_lib = None
_lock = threading.Lock()


# ---- device / stream plumbing without torch's per-call device-count queries -----------------------
# torch.cuda.stream(s) and device lookups with no explicit index go through torch.cuda.is_available()
# (a hipGetDeviceCount, ~4 us each); at ~10 per view they were a tenth of the host's cost per view.
def _index(dev) -> int:
    return dev.index if dev.index is not None else torch._C._cuda_getDevice()


def raw_stream(dev) -> int:
    """The current HIP stream of `dev` as the integer handle the C ABI takes."""
    return torch._C._cuda_getCurrentRawStream(_index(dev))


class on_device:
    """`with torch.cuda.device(dev)`, switching only when `dev` is not already current."""
    __slots__ = ("idx", "prev")

    def __init__(self, dev):
        self.idx = _index(dev)
        self.prev = -1

    def __enter__(self):
        self.prev = torch._C._cuda_getDevice()
        if self.prev != self.idx:
            torch._C._cuda_setDevice(self.idx)
        return self

    def __exit__(self, *exc):
        if self.prev != self.idx:
            torch._C._cuda_setDevice(self.prev)
        return False


class on_stream:
    """`with torch.cuda.stream(s)`: makes `s` the current stream of its device.  torch.cuda.
    set_stream also makes that device current, so the previous current device is restored on
    exit when it was another one (as torch.cuda.stream does)."""
    __slots__ = ("stream", "prev", "prev_dev")

    def __init__(self, stream):
        self.stream = stream
        self.prev = None
        self.prev_dev = -1

    def __enter__(self):
        self.prev_dev = torch._C._cuda_getDevice()
        self.prev = torch.cuda.current_stream(self.stream.device)
        torch.cuda.set_stream(self.stream)
        return self.stream

    def __exit__(self, *exc):
        torch.cuda.set_stream(self.prev)
        if torch._C._cuda_getDevice() != self.prev_dev:
            torch._C._cuda_setDevice(self.prev_dev)
        return False


class GsrView(ctypes.Structure):
    """include/gsr.h gsr_view: one camera of a multi-view call (field order and types as in C)."""
    _fields_ = [("viewmatrix", _p), ("projmatrix", _p), ("campos", _p),
                ("tan_fovx", _f), ("tan_fovy", _f),
                ("pre_color", _p), ("pre_clamp", _p),
                ("out_color", _p), ("out_depth", _p), ("out_alpha", _p), ("out_feature", _p),
                ("radii", _p),
                ("alloc_ctx", _p), ("geom_buffer", _p), ("binning_buffer", _p),
                ("image_buffer", _p),
                ("num_rendered", _i), ("num_instances", _i),
                ("stream", _p),
                ("dL_dout_color", _p), ("dL_dout_depth", _p), ("dL_dout_alpha", _p),
                ("dL_dout_feature", _p),
                ("dL_dmeans2D", _p), ("dL_dcolor_sh", _p), ("pre_jac", _p)]


class GsrError(RuntimeError):
    pass


def load():
    """Load libgsr.so (raises ImportError with the build hint if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libgsr.so not found at {LIB_PATH}: build it with "
                "`make -C sdp-gs_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        L.gsr_abi_version.restype = _i
        L.gsr_abi_version.argtypes = []
        L.gsr_last_error.restype = ctypes.c_char_p
        L.gsr_last_error.argtypes = []
        L.gsr_rasterize_gaussians.restype = _i
        L.gsr_rasterize_gaussians.argtypes = [
            _i, _i,                      # P, M
            _p, _p, _p, _p, _p, _p, _f,  # bg, means3D, colors, opacities, scales, rotations, scale_mod
            _p, _p, _p,                  # cov3D_precomp, view, proj
            _f, _f, _i, _i,              # tanfovx, tanfovy, H, W
            _p, _i, _p, _i,              # sh, degree, campos, prefiltered
            _p, _p, _p, _i,              # sh_language, lang_precomp, confidence, include_feature
            _p, _p, _p, _p, _p,          # out_color, out_depth, out_alpha, out_feature, radii
            ctypes.POINTER(_i),          # num_rendered
            ALLOC_FN, _p,                # alloc, alloc_ctx
            _p, _i]                      # stream, debug
        L.gsr_rasterize_gaussians_backward.restype = _i
        L.gsr_rasterize_gaussians_backward.argtypes = [
            _i, _i, _i,                  # P, M, R
            _p, _p, _p, _p,              # bg, means3D, radii, colors
            _p, _p, _f, _p,              # scales, rotations, scale_mod, cov3D_precomp
            _p, _p, _f, _f, _i, _i,      # view, proj, tanfovx, tanfovy, H, W
            _p, _p, _p, _p,              # dL_dcolor, dL_ddepth, dL_dalpha, dL_dfeature
            _p, _i, _p,                  # sh, degree, campos
            _p, _p, _p, _i,              # sh_language, lang_precomp, confidence, include_feature
            _p, _p, _p,                  # geom, binning, image buffers
            _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,  # grads
            _p, _i]                      # stream, debug
        L.gsr_rasterize_gaussians_fused.restype = _i
        L.gsr_rasterize_gaussians_fused.argtypes = [
            _i, _i,                      # P, M
            _p, _p,                      # bg, means3D
            _p, _p, _p,                  # features_dc, features_rest, opacity_raw
            _p, _p, _f,                  # scaling_raw, rotation_raw, scale_modifier
            _p, _p,                      # view, proj
            _f, _f, _i, _i,              # tanfovx, tanfovy, H, W
            _i, _p, _i,                  # degree, campos, prefiltered
            _p, _p, _i,                  # language_feature, confidence, include_feature
            _p, _p, _p, _p, _p,          # out_color, out_depth, out_alpha, out_feature, radii
            ctypes.POINTER(_i),          # num_rendered
            ALLOC_FN, _p,                # alloc, alloc_ctx
            _p, _i]                      # stream, debug
        L.gsr_rasterize_gaussians_fused_precolor.restype = _i
        fa = L.gsr_rasterize_gaussians_fused.argtypes
        L.gsr_rasterize_gaussians_fused_precolor.argtypes = fa[:22] + [_p, _p] + fa[22:]
        L.gsr_rasterize_gaussians_fused_backward.restype = _i
        L.gsr_rasterize_gaussians_fused_backward.argtypes = [
            _i, _i, _i,                  # P, M, R
            _p, _p, _p,                  # bg, means3D, radii
            _p, _p, _p,                  # features_dc, features_rest, opacity_raw
            _p, _p, _f,                  # scaling_raw, rotation_raw, scale_modifier
            _p, _p, _f, _f, _i, _i,      # view, proj, tanfovx, tanfovy, H, W
            _p, _p, _p, _p,              # dL_dcolor, dL_ddepth, dL_dalpha, dL_dfeature
            _i, _p,                      # degree, campos
            _p, _p, _i,                  # language_feature, confidence, include_feature
            _p, _p, _p,                  # geom, binning, image buffers
            _p, _p, _p, _p, _p, _p, _p, _p,  # grads: means2D, means3D, dc, rest, op, scale, rot, lang
            _i,                          # accumulate
            _p, _i]                      # stream, debug
        L.gsr_rasterize_gaussians_fused_backward_deferred.restype = _i
        L.gsr_rasterize_gaussians_fused_backward_deferred.argtypes = (
            L.gsr_rasterize_gaussians_fused_backward.argtypes[:-3] + [_p, _p, _i, _p, _i])
        _pv = ctypes.POINTER(GsrView)
        L.gsr_rasterize_views_fused.restype = _i
        L.gsr_rasterize_views_fused.argtypes = [
            _i, _pv, _i, _i,             # V, views, H, W
            _i, _i, _p, _p,              # P, M, bg, means3D
            _p, _p, _p,                  # features_dc, features_rest, opacity_raw
            _p, _p, _f,                  # scaling_raw, rotation_raw, scale_modifier
            _i, _i, _p, _p, _i,          # degree, prefiltered, language_feature, confidence, incl
            ALLOC_FN, _i, _p, _i]        # alloc, inflight, stream, debug
        L.gsr_rasterize_views_fused_backward.restype = _i
        L.gsr_rasterize_views_fused_backward.argtypes = [
            _i, _pv, _i, _i,             # V, views, H, W
            _i, _i, _p, _p,              # P, M, bg, means3D
            _p, _p, _p,                  # features_dc, features_rest, opacity_raw
            _p, _p, _f,                  # scaling_raw, rotation_raw, scale_modifier
            _i, _p, _p, _i,              # degree, language_feature, confidence, include_feature
            _p, _p, _p, _p, _p, _p, _p,  # grads: means3D, dc, rest, op, scale, rot, lang
            _i, _p, _i]                  # accumulate, stream, debug
        L.gsr_rasterize_views_fused_backward_sliced.restype = _i
        L.gsr_rasterize_views_fused_backward_sliced.argtypes = list(
            L.gsr_rasterize_views_fused_backward.argtypes) + [_i, ROWS_FN, _p]
        L.gsr_sh_precolor.restype = _i
        L.gsr_sh_precolor.argtypes = [_i, _i, _i, _p, _p, _p, _i, ctypes.POINTER(_p),
                                      ctypes.POINTER(_p), ctypes.POINTER(_p), ctypes.POINTER(_p), _p]
        L.gsr_sh_precolor_rows.restype = _i
        L.gsr_sh_precolor_rows.argtypes = [_i, _i, _i] + list(L.gsr_sh_precolor.argtypes[1:])
        L.gsr_sh_grad_flush.restype = _i
        L.gsr_sh_grad_flush.argtypes = [_i, _i, _i, _p, _i, ctypes.POINTER(_p),
                                        ctypes.POINTER(_p), ctypes.c_int64, _p, _p, _i, _p]
        # include/gsr_optim.h
        _pp = ctypes.POINTER(_p)
        L.gsr_adam_step.restype = _i
        L.gsr_adam_step.argtypes = [
            _i, _pp, _pp, _pp, _pp,                      # n, params, grads, exp_avg, exp_avg_sq
            ctypes.POINTER(ctypes.c_int64),              # numel
            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),  # lr, weight_decay
            ctypes.POINTER(ctypes.c_double),             # step
            ctypes.c_double, ctypes.c_double, ctypes.c_double,  # beta1, beta2, eps
            _p]                                          # stream
        L.gsr_adam_step_guarded.restype = _i
        L.gsr_adam_step_guarded.argtypes = list(L.gsr_adam_step.argtypes[:-1]) + [_p, _p, _p]
        L.gsr_step_guard.restype = _i
        L.gsr_step_guard.argtypes = [_p, _p]
        # include/gsr_densify.h
        _i64 = ctypes.c_int64
        _u32 = ctypes.c_uint32
        L.gsr_densify_stats.restype = _i
        L.gsr_densify_stats.argtypes = [_i64, _p, _i64, _p, _p, _p, _p, _p, _p]
        L.gsr_densify_stats_views.restype = _i
        L.gsr_densify_stats_views.argtypes = [_i, _i64, _p, _i64, _i64, _p, _p, _p, _p, _p]
        L.gsr_densify_classify.restype = _i
        L.gsr_densify_classify.argtypes = [_i64, _p, _p, _p, _p, _f, _f, _f, _i, _f, _p, _p, _p]
        L.gsr_select_scratch_bytes.restype = _sz
        L.gsr_select_scratch_bytes.argtypes = [_i64]
        L.gsr_select_rows.restype = _i
        L.gsr_select_rows.argtypes = [_i64, _p, _u32, _u32, _p, _p, _p, _p]
        L.gsr_compact_rows.restype = _i
        L.gsr_compact_rows.argtypes = [_i, _pp, _pp, _pp, ctypes.POINTER(_i64),
                                       ctypes.POINTER(_u32), _i64, _p, _i64, _p]
        # include/gsr_loss.h
        L.gsr_photometric_scratch_bytes.restype = _sz
        L.gsr_photometric_scratch_bytes.argtypes = [_i, _i, _i]
        L.gsr_photometric_loss.restype = _i
        L.gsr_photometric_loss.argtypes = [_i, _i, _i, _p, _p, _f, _i, _p, _p, _p]
        L.gsr_photometric_loss_backward.restype = _i
        L.gsr_photometric_loss_backward.argtypes = [_i, _i, _i, _p, _p, _f, _p, _p, _p, _p, _p,
                                                    _p]
        L.gsr_pearson_scratch_bytes.restype = _sz
        L.gsr_pearson_scratch_bytes.argtypes = [_i, _i]
        L.gsr_pearson_loss.restype = _i
        L.gsr_pearson_loss.argtypes = [_i64, _i, _p, _p, _i, _f, _p, _p, _p, _p]
        L.gsr_pearson_loss_backward.restype = _i
        L.gsr_pearson_loss_backward.argtypes = [_i64, _i, _p, _p, _i, _f, _p, _p, _p, _p, _p]
        L.gsr_view_loss_scratch_bytes.restype = _sz
        L.gsr_view_loss_scratch_bytes.argtypes = [_i, _i, _i]
        L.gsr_view_loss.restype = _i
        L.gsr_view_loss.argtypes = [_i, _i, _i, _p, _p, _f, _i64, _p, _p, _f, _f, _i, _p, _p, _p,
                                    _p]
        L.gsr_view_loss_backward.restype = _i
        L.gsr_view_loss_backward.argtypes = [_i, _i, _i, _p, _p, _f, _i64, _p, _p, _f, _f, _p, _p,
                                             _p, _p, _p]
        L.gsr_view_loss_views.restype = _i
        L.gsr_view_loss_views.argtypes = [_i, _i, _i, _i, _p, _p, _f, _i64, _p, _p, _f, _f, _i,
                                          _p, _p, _p, _p]
        L.gsr_view_loss_views_backward.restype = _i
        L.gsr_view_loss_views_backward.argtypes = [_i, _i, _i, _i, _p, _p, _f, _i64, _p, _p, _f,
                                                   _f, _p, _p, _p, _p, _p]
        # include/gsr_knn.h
        L.gsr_knn_scratch_bytes.restype = _sz
        L.gsr_knn_scratch_bytes.argtypes = [_i64]
        L.gsr_dist_knn3.restype = _i
        L.gsr_dist_knn3.argtypes = [_i64, _p, _p, _p, _p, _p]
        L.gsr_mark_visible.restype = _i
        L.gsr_mark_visible.argtypes = [_i, _p, _p, _p, _p, _p]
        L.gsr_forward_status.restype = _i
        L.gsr_forward_status.argtypes = [_p, _i]
        L.gsr_check_forwards.restype = _i
        L.gsr_check_forwards.argtypes = [_i]
        for n in ("gsr_last_forward_instances", "gsr_forward_faults", "gsr_reset_forward_faults"):
            getattr(L, n).restype = _i
            getattr(L, n).argtypes = []
        for n in ("gsr_geom_buffer_bytes", "gsr_binning_buffer_bytes",
                  "gsr_binning_buffer_bytes_det"):
            getattr(L, n).restype = _sz
            getattr(L, n).argtypes = [_i]
        L.gsr_image_buffer_bytes.restype = _sz
        L.gsr_image_buffer_bytes.argtypes = [_i, _i]
        # test hooks (include/gsr_testing.h); every pointer is typed so ctypes never truncates it
        L.gsr_test_sort_scratch_bytes.restype = _sz
        L.gsr_test_sort_scratch_bytes.argtypes = [_sz]
        L.gsr_test_radix_sort_pairs.restype = _i
        L.gsr_test_radix_sort_pairs.argtypes = [_p, _p, _sz, _i, _p, _p]
        L.gsr_test_radix_sort_pairs_sentinel.restype = _i
        L.gsr_test_radix_sort_pairs_sentinel.argtypes = [_p, _p, _sz, _i, _p, _p]
        L.gsr_test_radix_sort_pairs_planned.restype = _i
        L.gsr_test_radix_sort_pairs_planned.argtypes = [_p, _p, _sz, _i, _i, _p, _p]
        L.gsr_test_scan_scratch_bytes.restype = _sz
        L.gsr_test_scan_scratch_bytes.argtypes = [_sz]
        L.gsr_test_scan.restype = _i
        L.gsr_test_scan.argtypes = [_p, _p, _sz, _i, _p, _p]
        L.gsr_test_expf_pair.restype = _i
        L.gsr_test_expf_pair.argtypes = [_p, _p, _p, _sz, _p]
        L.gsr_test_force_sort_timeout.restype = _i
        L.gsr_test_force_sort_timeout.argtypes = [_i]
        L.gsr_test_binning_lists.restype = _i
        L.gsr_test_splat_records.restype = _i
        L.gsr_test_splat_records.argtypes = [_p, _i, _p, _p]
        L.gsr_test_binning_lists.argtypes = [_p, _p, _i, _i, _i, _i, _i, _p, _p, _p]
        L.gsr_test_activations.restype = _i
        L.gsr_test_activations.argtypes = [_p, _p, _p, _sz, _p, _p, _p, _p]
        L.gsr_profile_enable.restype = None
        L.gsr_profile_enable.argtypes = [_i]
        L.gsr_profile_collect.restype = _i
        L.gsr_profile_collect.argtypes = [ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_longlong)]
        L.gsr_profile_reset.restype = None
        L.gsr_profile_reset.argtypes = []
        L.gsr_profile_stage_name.restype = ctypes.c_char_p
        L.gsr_profile_stage_name.argtypes = [_i]
        L.gsr_test_scan_lookback_words.restype = _sz
        L.gsr_test_scan_lookback_words.argtypes = [_sz]
        L.gsr_test_scan_lookback.restype = _i
        L.gsr_test_scan_lookback.argtypes = [_p, _p, _sz, _i, _p, _p]
        L.gsr_test_host_wait_ms.restype = ctypes.c_double
        L.gsr_test_host_wait_ms.argtypes = [_i]
        _lib = L
    return _lib


# include/gsr.h gsr_rows_fn: (ctx, row_begin, row_end)
ROWS_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)


def check(rc: int):
    if rc != 0:
        msg = load().gsr_last_error().decode(errors="replace")
        raise GsrError(f"libgsr error {rc}: {msg}")


def forward_faults() -> int:
    """The device's sticky forward fault word (include/gsr.h gsr_forward_faults; synchronous)."""
    return int(load().gsr_forward_faults())


_FAULT_RESETS = [0]  # how many times reset_forward_faults() ran (gsr_amd.optim reads it)


def reset_forward_faults():
    """Clear the fault word (after a failure has been handled); FusedAdam steps again."""
    if load().gsr_reset_forward_faults() != 0:
        raise GsrError("gsr_reset_forward_faults failed")
    _FAULT_RESETS[0] += 1


def fault_resets() -> int:
    return _FAULT_RESETS[0]


def step_guard(slot: "torch.Tensor"):
    """Write the device's forward-fault snapshot (1.0 failed / 0.0 ok) into the one-float device
    tensor `slot` on the current stream (include/gsr_optim.h gsr_step_guard)."""
    import torch
    if slot.dtype != torch.float32 or slot.numel() < 1 or not slot.is_cuda:
        raise ValueError("step_guard: slot must be a float32 device tensor")
    with on_device(slot.device):
        check(load().gsr_step_guard(slot.data_ptr(), raw_stream(slot.device)))


def check_forwards(wait: bool = True):
    """Raise GsrError if any forward not yet checked failed (a sort gave up its bounded
    look-back or an id had to be clamped; that call's outputs and gradients are NaN).  wait
    blocks until those forwards have finished (include/gsr.h gsr_check_forwards)."""
    check(load().gsr_check_forwards(1 if wait else 0))


# --- allocator callback: the library asks for its three scratch buffers through it ---------------
_holders: dict[int, "BufferHolder"] = {}
_holder_lock = threading.Lock()
_holder_seq = [0]


class BufferHolder:
    """Owns the geometry / binning / image byte tensors of one forward (the reference keeps the
    same three tensors in the autograd context, diff_gaussian_rasterization/__init__.py:97)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.bufs = [None, None, None]
        with _holder_lock:
            _holder_seq[0] += 1
            self.key = _holder_seq[0]
            _holders[self.key] = self

    def release(self):
        with _holder_lock:
            _holders.pop(self.key, None)

    def ptr(self, which: int):
        b = self.bufs[which]
        return None if b is None else b.data_ptr()


def _alloc_cb(ctx, nbytes, which):
    h = _holders.get(int(ctx or 0))
    if h is None:
        return None
    try:
        t = torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device=h.device)
    except Exception:  # out of memory: the library reports GSR_ERR_ALLOC
        return None
    h.bufs[which] = t
    return t.data_ptr()


_ALLOC_CB = ALLOC_FN(_alloc_cb)


def alloc_callback():
    return _ALLOC_CB


NUM_STAGES = 12


class StageTimer:
    """Per-stage device time from the library's hipEvent instrumentation (gsr_testing.h)."""

    def __init__(self):
        self.L = load()

    def enable(self, on=True, stages=None):
        """on: instrument every stage (stages None) or only the named stages."""
        if not on:
            mask = 0
        elif stages is None:
            mask = -1
        else:
            names = [self.L.gsr_profile_stage_name(i).decode() for i in range(NUM_STAGES)]
            mask = 0
            for s in stages:
                mask |= 1 << names.index(s)
        self.L.gsr_profile_enable(mask)

    def reset(self):
        self.L.gsr_profile_reset()

    def collect(self):
        ms = (ctypes.c_double * NUM_STAGES)()
        calls = (ctypes.c_longlong * NUM_STAGES)()
        check(self.L.gsr_profile_collect(ms, calls))
        return {self.L.gsr_profile_stage_name(i).decode(): (ms[i], calls[i])
                for i in range(NUM_STAGES)}

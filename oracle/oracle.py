"""ctypes front-end of the CPU restatement (oracle/gsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / CPU baseline -- never by the product package (sdp-gs_amd/).

The arrays follow the reference rasterizer's tensor conventions
(submodules/diff-gaussian-rasterization/rasterize_points.cu:35-196): float32, C-contiguous,
images planar [C,H,W], `None` == empty tensor == nullptr.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# variants of the same source (oracle/Makefile): "f32" the checker, "f64" the float64 build,
# "expf" float32 with libm's expf as the blend exp (threshold census)
_LIB_FILES = {"f32": "libgsr_oracle.so", "f64": "libgsr_oracle_f64.so",
              "expf": "libgsr_oracle_expf.so"}
_LIB_PATH = os.path.join(_HERE, "_build", _LIB_FILES["f32"])
_libs = {}

_f = ctypes.c_float
_i = ctypes.c_int
_p = ctypes.c_void_p


def build() -> str:
    """Compile the oracle with gcc (seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(variant: str = "f32"):
    L = _libs.get(variant)
    if L is None:
        path = os.path.join(_HERE, "_build", _LIB_FILES[variant])
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_forward.restype = _p
        L.oracle_forward.argtypes = [
            _i, _i, _p, _p, _p, _p, _p, _p, _f, _p, _p, _p, _f, _f, _i, _i, _p, _i, _p, _i,
            _p, _p, _p, _i, _p, _p, _p, _p, _p, ctypes.POINTER(_i)]
        L.oracle_backward.restype = _i
        L.oracle_backward.argtypes = [_p] + [_p] * 14
        L.oracle_blend_rows.restype = _i
        L.oracle_blend_rows.argtypes = [_p, _p, _p, _p, _p, _i, _p]
        L.oracle_backward_rows.restype = _i
        L.oracle_backward_rows.argtypes = [_p] * 12
        L.oracle_free.restype = None
        L.oracle_free.argtypes = [_p]
        L.oracle_use_lists.restype = None
        L.oracle_use_lists.argtypes = [_p, _i, _p]
        L.oracle_use_decisions.restype = None
        L.oracle_use_decisions.argtypes = [_p, _p, _p]
        L.oracle_use_geometry.restype = None
        L.oracle_use_geometry.argtypes = [_p, _p]
        L.oracle_use_clamp.restype = None
        L.oracle_use_clamp.argtypes = [_p]
        L.oracle_get_clamped.restype = _i
        L.oracle_get_clamped.argtypes = [_p, _p]
        L.oracle_accept_bits.restype = ctypes.c_long
        L.oracle_accept_bits.argtypes = [_p, _p, _p]
        L.oracle_mark_visible.restype = _i
        L.oracle_mark_visible.argtypes = [_i, _p, _p, _p, _p]
        L.oracle_splat_exp.restype = None
        L.oracle_splat_exp.argtypes = [ctypes.c_long, _p, _p]
        L.oracle_splat_log.restype = None
        L.oracle_splat_log.argtypes = [ctypes.c_long, _p, _p]
        L.oracle_cut_lists.restype = _i
        L.oracle_cut_lists.argtypes = [_p, _p, _p]
        L.oracle_set_threads.restype = None
        L.oracle_set_threads.argtypes = [_i]
        L.oracle_get_threads.restype = _i
        L.oracle_get_threads.argtypes = []
        L.oracle_dist_knn3.restype = None
        L.oracle_dist_knn3.argtypes = [ctypes.c_int64, _p, _p, _p]
        for name in ("point_list", "ranges", "final_T", "n_contrib", "margin", "means2D", "conic_opacity",
                     "depths", "rgb", "tiles_touched", "cov3D", "preprocess_f64"):
            fn = getattr(L, "oracle_get_" + name)
            fn.restype = _i
            fn.argtypes = [_p, _p]
        _libs[variant] = L
    return L


def set_threads(n: int) -> int:
    """Host threads of the oracle's loops (1 = the sequential restatement); returns the value set
    (every variant)."""
    for v in _LIB_FILES:
        lib(v).oracle_set_threads(int(n))
    return int(lib().oracle_get_threads())


def _arr(x, dtype=np.float32):
    if x is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    return a


def _ptr(a):
    return None if a is None else a.ctypes.data


class OracleRaster:
    """One forward (+ optional backward) of the restated rasterizer on host arrays.  variant:
    "f32" (the checker), "f64" (the same restatement in float64: images and gradients come back
    as float64) or "expf" (float32 with libm's expf as the blend exp).  lists=(point_list, ranges)
    skips the binning and blends those instance lists (another raster's point_list() / ranges());
    decisions=(n_contrib, offsets, words) blends with another raster's per-pixel decisions
    (its accept_bits()) instead of this one's own threshold tests; clamp= [P,3] u8 takes another
    raster's SH colour clamp bits (its clamped()) instead of this one's result < 0 tests;
    geometry=(means2D [P,2], conic_opacity [P,4]) blends another raster's projected splats."""

    def __init__(self, *, variant="f32", means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy,
                 image_height, image_width, bg, scale_modifier=1.0, sh_degree=0, shs=None,
                 colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
                 shs_language=None, language_feature_precomp=None, confidence=None,
                 include_feature=True, prefiltered=False, lists=None, decisions=None,
                 clamp=None, geometry=None):
        L = lib(variant)
        self.variant = variant
        self._L = L
        od = np.float64 if variant == "f64" else np.float32
        self._od = od
        self._keep = {}
        k = self._keep
        k["means3D"] = _arr(means3D).reshape(-1, 3)
        P = k["means3D"].shape[0]
        k["opac"] = _arr(opacities).reshape(P)
        k["view"] = _arr(viewmatrix).reshape(16)
        k["proj"] = _arr(projmatrix).reshape(16)
        k["campos"] = _arr(campos).reshape(3)
        k["bg"] = _arr(bg).reshape(3)
        k["shs"] = None if shs is None else _arr(shs).reshape(P, -1, 3)
        M = 0 if k["shs"] is None else k["shs"].shape[1]
        k["colors"] = None if colors_precomp is None else _arr(colors_precomp).reshape(P, 3)
        k["scales"] = None if scales is None else _arr(scales).reshape(P, 3)
        k["rot"] = None if rotations is None else _arr(rotations).reshape(P, 4)
        k["cov"] = None if cov3D_precomp is None else _arr(cov3D_precomp).reshape(P, 6)
        k["shl"] = None if shs_language is None else _arr(shs_language).reshape(P, 3)
        k["lfp"] = None if language_feature_precomp is None else _arr(language_feature_precomp).reshape(P, 3)
        k["conf"] = None if confidence is None else _arr(confidence).reshape(P)
        H, W = int(image_height), int(image_width)
        self.P, self.M, self.H, self.W = P, M, H, W
        self.color = np.zeros((3, H, W), od)
        self.depth = np.zeros((1, H, W), od)
        self.alpha = np.zeros((1, H, W), od)
        self.feature = np.zeros((3, H, W), od)
        self.radii = np.zeros((P,), np.int32)
        nr = _i(0)
        if lists is not None:
            k["pl"] = np.ascontiguousarray(lists[0], np.uint32)
            k["rg"] = np.ascontiguousarray(lists[1], np.uint32)
            if k["rg"].size != 2 * ((W + 15) // 16) * ((H + 15) // 16):
                raise ValueError("lists: ranges must hold two entries per tile")
            L.oracle_use_lists(_ptr(k["pl"]), int(k["pl"].size), _ptr(k["rg"]))
        if decisions is not None:
            k["dnc"] = np.ascontiguousarray(decisions[0], np.uint32).reshape(-1)
            k["doffs"] = np.ascontiguousarray(decisions[1], np.uint64).reshape(-1)
            k["dwords"] = np.ascontiguousarray(decisions[2], np.uint32).reshape(-1)
            if k["dnc"].size != H * W or k["doffs"].size != H * W + 1 or \
                    k["dwords"].size < int(k["doffs"][-1]):
                raise ValueError("decisions: (n_contrib [H*W], offsets [H*W+1], words) expected")
            L.oracle_use_decisions(_ptr(k["dnc"]), _ptr(k["doffs"]), _ptr(k["dwords"]))
        if clamp is not None:
            k["clamp"] = np.ascontiguousarray(clamp, np.uint8).reshape(-1)
            if k["clamp"].size != 3 * P:
                raise ValueError("clamp: [P, 3] clamp bits expected")
            L.oracle_use_clamp(_ptr(k["clamp"]))
        if geometry is not None:
            k["gm"] = np.ascontiguousarray(geometry[0], np.float32).reshape(-1)
            k["gc"] = np.ascontiguousarray(geometry[1], np.float32).reshape(-1)
            if k["gm"].size != 2 * P or k["gc"].size != 4 * P:
                raise ValueError("geometry: (means2D [P,2], conic_opacity [P,4]) expected")
            L.oracle_use_geometry(_ptr(k["gm"]), _ptr(k["gc"]))
        try:
            self._st = L.oracle_forward(
            P, M, _ptr(k["bg"]), _ptr(k["means3D"]), _ptr(k["colors"]), _ptr(k["opac"]),
            _ptr(k["scales"]), _ptr(k["rot"]), float(scale_modifier), _ptr(k["cov"]),
            _ptr(k["view"]), _ptr(k["proj"]), float(tanfovx), float(tanfovy), H, W,
            _ptr(k["shs"]), int(sh_degree), _ptr(k["campos"]), int(bool(prefiltered)),
            _ptr(k["shl"]), _ptr(k["lfp"]), _ptr(k["conf"]), int(bool(include_feature)),
            _ptr(self.color), _ptr(self.depth), _ptr(self.alpha), _ptr(self.feature),
            _ptr(self.radii), ctypes.byref(nr))
        finally:
            if lists is not None:
                L.oracle_use_lists(None, 0, None)
            if decisions is not None:
                L.oracle_use_decisions(None, None, None)
            if clamp is not None:
                L.oracle_use_clamp(None)
            if geometry is not None:
                L.oracle_use_geometry(None, None)
        if not self._st:
            raise RuntimeError("oracle_forward rejected its arguments")
        self.num_rendered = int(nr.value)
        self.gx = (W + 15) // 16
        self.gy = (H + 15) // 16

    def __del__(self):
        st = getattr(self, "_st", None)
        if st:
            self._L.oracle_free(st)
            self._st = None

    # ---- state introspection -------------------------------------------------------------
    def _get(self, name, shape, dtype):
        out = np.zeros(shape, dtype)
        getattr(self._L, "oracle_get_" + name)(self._st, _ptr(out))
        return out

    def point_list(self):
        return self._get("point_list", (self.num_rendered,), np.uint32)

    def ranges(self):
        return self._get("ranges", (self.gx * self.gy, 2), np.uint32)

    def cut_lists(self):
        """(point_list, ranges) of the reference's binning with the HIP build's exact tile cull
        applied (oracle/gsr_oracle.c oracle_cut_lists): the instances that can contribute, in
        the reference's order."""
        pl = np.zeros((max(self.num_rendered, 1),), np.uint32)
        rg = np.zeros((self.gx * self.gy, 2), np.uint32)
        n = self._L.oracle_cut_lists(self._st, _ptr(pl), _ptr(rg))
        return pl[:n].copy(), rg

    def final_T(self):
        return self._get("final_T", (self.H, self.W), np.float32)

    def n_contrib(self):
        return self._get("n_contrib", (self.H, self.W), np.uint32)

    def accept_bits(self):
        """The forward's blend decisions: (n_contrib [H*W], word offsets [H*W + 1], bitset words)
        -- per pixel, bit q set iff list position q < n_contrib was blended (the `decisions=` of
        another raster)."""
        offs = np.zeros(self.H * self.W + 1, np.uint64)
        n = int(self._L.oracle_accept_bits(self._st, _ptr(offs), None))
        words = np.zeros(max(n, 1), np.uint32)
        self._L.oracle_accept_bits(self._st, _ptr(offs), _ptr(words))
        return self.n_contrib().reshape(-1), offs, words

    def clamped(self):
        """The SH colour clamp bits [P, 3] (forward.cu:67-69: channel clamped at 0, its dL/dRGB
        masked in the backward) -- the `clamp=` of another raster."""
        out = np.zeros((self.P, 3), np.uint8)
        self._L.oracle_get_clamped(self._st, _ptr(out))
        return out

    def margin(self):
        """Per pixel: the smallest relative distance of any blend decision from its threshold
        (|255 alpha - 1|, |1e4 test_T - 1|, 0 for |power| < 1e-6).  Test-side diagnostic: a
        pixel whose margin is a few ulps can legitimately flip between two correct float
        implementations (the reference's own expf is specified to 2 ulp)."""
        return self._get("margin", (self.H, self.W), np.float32)

    def means2D(self):
        return self._get("means2D", (self.P, 2), np.float32)

    def conic_opacity(self):
        return self._get("conic_opacity", (self.P, 4), np.float32)

    def depths(self):
        return self._get("depths", (self.P,), np.float32)

    def rgb(self):
        return self._get("rgb", (self.P, 3), np.float32)

    def tiles_touched(self):
        return self._get("tiles_touched", (self.P,), np.uint32)

    def cov3D(self):
        return self._get("cov3D", (self.P, 6), np.float32)

    def preprocess_f64(self):
        """[P, 13] float64 at the build's own precision, in the GPU splat record's order: x_px,
        y_px, conic a, b, c, opacity, depth, r, g, b, f0, f1, f2 (culled rows: zeros)."""
        return self._get("preprocess_f64", (self.P, 13), np.float64)

    # ---- backward --------------------------------------------------------------------------
    def backward(self, dL_dcolor, dL_ddepth=None, dL_dalpha=None, dL_dfeature=None):
        k = self._keep
        P, M = self.P, self.M
        od = self._od
        dc = _arr(dL_dcolor).reshape(3, self.H, self.W)
        dd = None if dL_ddepth is None else _arr(dL_ddepth).reshape(1, self.H, self.W)
        da = None if dL_dalpha is None else _arr(dL_dalpha).reshape(1, self.H, self.W)
        df = None if dL_dfeature is None else _arr(dL_dfeature).reshape(3, self.H, self.W)
        g = {
            "means2D": np.zeros((P, 3), od),
            "colors": np.zeros((P, 3), od),
            "opacity": np.zeros((P, 1), od),
            "means3D": np.zeros((P, 3), od),
            "cov3D": np.zeros((P, 6), od),
            "sh": np.zeros((P, M, 3), od) if k["shs"] is not None else None,
            "scales": np.zeros((P, 3), od) if k["scales"] is not None else None,
            "rotations": np.zeros((P, 4), od) if k["rot"] is not None else None,
            "sh_language": np.zeros((P, 3), od) if k["shl"] is not None else None,
            "language_feature": np.zeros((P, 3), od) if k["lfp"] is not None else None,
        }
        self._keep_bwd = (dc, dd, da, df)
        rc = self._L.oracle_backward(
            self._st, _ptr(dc), _ptr(dd), _ptr(da), _ptr(df), _ptr(g["means2D"]), _ptr(g["colors"]),
            _ptr(g["opacity"]), _ptr(g["means3D"]), _ptr(g["cov3D"]), _ptr(g["sh"]),
            _ptr(g["scales"]), _ptr(g["rotations"]), _ptr(g["sh_language"]),
            _ptr(g["language_feature"]))
        if rc != 0:
            raise RuntimeError("oracle_backward failed")
        return g


    # ---- the backward in two parts (float64 rounding analysis, tests/f64_ref.py) ---------------
    ROW_SLOTS = 15  # colours 3 | depth 1 | feature 3 | means2D 3 | conic 4 | opacity 1 (per P)

    def blend_rows(self, dL_dcolor, dL_ddepth=None, dL_dalpha=None, dL_dfeature=None, mass=False):
        """The blend backward's per-Gaussian sums as the oracle's [15 * P] accumulator block
        (gsr_oracle.h oracle_blend_rows); mass: sums of the terms' absolute values."""
        dc = _arr(dL_dcolor).reshape(3, self.H, self.W)
        dd = None if dL_ddepth is None else _arr(dL_ddepth).reshape(1, self.H, self.W)
        da = None if dL_dalpha is None else _arr(dL_dalpha).reshape(1, self.H, self.W)
        df = None if dL_dfeature is None else _arr(dL_dfeature).reshape(3, self.H, self.W)
        rows = np.zeros(self.ROW_SLOTS * self.P, self._od)
        if self._L.oracle_blend_rows(self._st, _ptr(dc), _ptr(dd), _ptr(da), _ptr(df),
                                     int(bool(mass)), _ptr(rows)) != 0:
            raise RuntimeError("oracle_blend_rows failed")
        return rows

    def backward_rows(self, rows):
        """The per-Gaussian backward from an accumulator block (linear in it); the gradient dict
        of backward()."""
        k = self._keep
        P, M, od = self.P, self.M, self._od
        rows = np.ascontiguousarray(rows, od).reshape(-1)
        assert rows.size == self.ROW_SLOTS * P
        g = {
            "means2D": np.zeros((P, 3), od), "colors": np.zeros((P, 3), od),
            "opacity": np.zeros((P, 1), od), "means3D": np.zeros((P, 3), od),
            "cov3D": np.zeros((P, 6), od),
            "sh": np.zeros((P, M, 3), od) if k["shs"] is not None else None,
            "scales": np.zeros((P, 3), od) if k["scales"] is not None else None,
            "rotations": np.zeros((P, 4), od) if k["rot"] is not None else None,
            "sh_language": np.zeros((P, 3), od) if k["shl"] is not None else None,
            "language_feature": np.zeros((P, 3), od) if k["lfp"] is not None else None,
        }
        if self._L.oracle_backward_rows(
                self._st, _ptr(rows), _ptr(g["means2D"]), _ptr(g["colors"]), _ptr(g["opacity"]),
                _ptr(g["means3D"]), _ptr(g["cov3D"]), _ptr(g["sh"]), _ptr(g["scales"]),
                _ptr(g["rotations"]), _ptr(g["sh_language"]), _ptr(g["language_feature"])) != 0:
            raise RuntimeError("oracle_backward_rows failed")
        return g


def splat_exp(x):
    """The blend's exp (oracle/gsr_oracle.c splat_exp) of a float32 array."""
    xs = _arr(x).reshape(-1)
    out = np.empty_like(xs)
    lib().oracle_splat_exp(xs.size, _ptr(xs), _ptr(out))
    return out


def splat_log(x):
    """The culling threshold's log (oracle/gsr_oracle.c splat_log) of a float32 array."""
    xs = _arr(x).reshape(-1)
    out = np.empty_like(xs)
    lib().oracle_splat_log(xs.size, _ptr(xs), _ptr(out))
    return out


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _arr(means3D).reshape(-1, 3)
    v = _arr(viewmatrix).reshape(16)
    p = _arr(projmatrix).reshape(16)
    out = np.zeros((m.shape[0],), np.uint8)
    lib().oracle_mark_visible(m.shape[0], _ptr(m), _ptr(v), _ptr(p), _ptr(out))
    return out.astype(bool)


def dist_knn3(points):
    """distCUDA2 restated (oracle/gsr_oracle_knn.c): (mean sq. dist [P] f32, indices [P,3] i32)."""
    pts = _arr(points).reshape(-1, 3)
    P = pts.shape[0]
    mean = np.zeros(P, np.float32)
    idx = np.zeros((P, 3), np.int32)
    lib().oracle_dist_knn3(P, _ptr(pts), _ptr(mean), _ptr(idx))
    return mean, idx

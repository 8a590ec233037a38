"""First-order float32 rounding bound of the forward preprocess outputs.

TEST INFRASTRUCTURE (tests/test_pre_f64_parity.py, tests/test_f64_oracle.py).  The preprocess
(preprocessCUDA, forward.cu:155-256, restated by oracle/gsr_oracle.c preprocess_one) maps float32
inputs to the splat record through a fixed sequence of float operations.  Evaluated in float32,
each operation rounds its result by at most u |result| (u = 2^-24, round to nearest) and passes on
its operands' errors scaled by the operation's partial derivatives.  `E` carries a value in float64
and that propagated bound e (in units of u) through the same expressions, in the same order, as
the oracle:

    a + b, a - b:  e = e_a + e_b + |a +- b|
    a * b:         e = |a| e_b + |b| e_a + |a b|
    a / b:         e = (e_a + |a / b| e_b) / |b| + |a / b|
    sqrt(a):       e = e_a / (2 sqrt a) + |sqrt a|
    min / max:     the chosen operand's e

so |fl32(f) - f| <= u e to first order for every output f (a worst case: all roundings aligned).
The inputs (means, activated scales / rotations, SH rows, matrices) and the float constants are
exact in both builds.  ndc2Pix runs in double in the reference (auxiliary.h:41-44): its error is
the float input's error times S / 2 plus the final rounding to float.
"""
from __future__ import annotations

import math

import numpy as np

COLUMNS = ("x", "y", "conic_a", "conic_b", "conic_c", "opacity", "depth", "r", "g", "b",
           "f0", "f1", "f2")

# auxiliary.h:22-39 (float constants, exact in both builds)
SH_C0 = float(np.float32(0.28209479177387814))
SH_C1 = float(np.float32(0.4886025119029199))
SH_C2 = [float(np.float32(c)) for c in (1.0925484305920792, -1.0925484305920792,
                                        0.31539156525252005, -1.0925484305920792,
                                        0.5462742152960396)]
SH_C3 = [float(np.float32(c)) for c in (-0.5900435899266435, 2.890611442640554,
                                        -0.4570457994644658, 0.3731763325901154,
                                        -0.4570457994644658, 1.445305721320277,
                                        -0.5900435899266435)]


def f32c(x):
    """A float literal of the C source (1.3f, 0.3f, 1e-7f, ...): exact, rounded to float."""
    return float(np.float32(x))


class E:
    """float64 value + first-order float32 rounding bound (units of u)."""
    __slots__ = ("v", "e")

    def __init__(self, v, e=None):
        self.v = np.asarray(v, np.float64)
        self.e = np.zeros(np.shape(self.v)) if e is None else e

    @staticmethod
    def _w(x):
        return x if isinstance(x, E) else E(x)

    def __add__(self, o):
        o = E._w(o)
        v = self.v + o.v
        return E(v, self.e + o.e + np.abs(v))

    __radd__ = __add__

    def __sub__(self, o):
        o = E._w(o)
        v = self.v - o.v
        return E(v, self.e + o.e + np.abs(v))

    def __rsub__(self, o):
        return E._w(o) - self

    def __mul__(self, o):
        o = E._w(o)
        v = self.v * o.v
        return E(v, np.abs(self.v) * o.e + np.abs(o.v) * self.e + np.abs(v))

    __rmul__ = __mul__

    def __truediv__(self, o):
        o = E._w(o)
        with np.errstate(divide="ignore", invalid="ignore"):
            v = self.v / o.v
            e = (self.e + np.abs(v) * o.e) / np.abs(o.v) + np.abs(v)
        return E(v, e)

    def __rtruediv__(self, o):
        return E._w(o) / self

    def __neg__(self):
        return E(-self.v, self.e)


def sqrt(a):
    v = np.sqrt(np.maximum(a.v, 0.0))
    with np.errstate(divide="ignore", invalid="ignore"):
        e = np.where(v > 0, a.e / (2.0 * np.maximum(v, 1e-300)), 0.0) + v
    return E(v, e)


def fmin(a, b):
    a, b = E._w(a), E._w(b)
    pick = a.v <= b.v
    return E(np.where(pick, a.v, b.v), np.where(pick, a.e, b.e))


def fmax(a, b):
    a, b = E._w(a), E._w(b)
    pick = a.v >= b.v
    return E(np.where(pick, a.v, b.v), np.where(pick, a.e, b.e))


# glm column-major 3x3 (m[col][row]) in the oracle's order (gsr_oracle.c m3_mul, m3_T)
def m3_cols(*a):
    return [[a[0], a[1], a[2]], [a[3], a[4], a[5]], [a[6], a[7], a[8]]]


def m3_mul(a, b):
    return [[(a[0][w] * b[c][0] + a[1][w] * b[c][1]) + a[2][w] * b[c][2] for w in range(3)]
            for c in range(3)]


def m3_T(a):
    return [[a[w][c] for w in range(3)] for c in range(3)]


def _xf43(p, m, row):
    """transformPoint4x3 / 4x4 component `row` (auxiliary.h:58-77): left-to-right sums."""
    return ((m[row] * p[0] + m[4 + row] * p[1]) + m[8 + row] * p[2]) + m[12 + row]


def preprocess_bound(means, scales, rotations, opacity, shs, sh_degree, lang, view, proj, campos,
                     tanfovx, tanfovy, W, H, scale_modifier=1.0):
    """(value [P, 13] float64, bound [P, 13] in units of u) of the preprocess outputs in COLUMNS
    order, for every Gaussian (culling is not applied: compare visible rows only).  Inputs as the
    oracle takes them: float32 arrays, activated scales / rotations / opacity, SH [P, M, 3],
    language feature [P, 3] (its degree-0 SH), view / proj [16] (the reference's row-major
    tensors read as column-major), campos [3]."""
    P = means.shape[0]
    tanfovx, tanfovy = f32c(tanfovx), f32c(tanfovy)  # float arguments of the ABI
    mx, my, mz = (E(means[:, k].astype(np.float64)) for k in range(3))
    vw = [float(x) for x in np.asarray(view, np.float32).reshape(-1)]
    pj = [float(x) for x in np.asarray(proj, np.float32).reshape(-1)]
    p = (mx, my, mz)
    # depth: p_view.z (auxiliary.h:58-64)
    depth = _xf43(p, vw, 2)
    # projection (forward.cu:176-178)
    ph = [_xf43(p, pj, k) for k in range(4)]
    pw = 1.0 / (ph[3] + f32c(1e-7))
    pxn, pyn = ph[0] * pw, ph[1] * pw

    def ndc2pix(v, S):
        val = ((v.v + 1.0) * S - 1.0) * 0.5
        return E(val, v.e * S * 0.5 + np.abs(val))

    px, py = ndc2pix(pxn, W), ndc2pix(pyn, H)
    # computeCov3D (forward.cu:118-152), no quaternion normalisation in the kernel
    s = [E(scales[:, k].astype(np.float64)) * f32c(scale_modifier) for k in range(3)]
    r, x, y, z = (E(rotations[:, k].astype(np.float64)) for k in range(4))
    zero, one = E(np.zeros(P)), E(np.ones(P))
    S = m3_cols(s[0], zero, zero, zero, s[1], zero, zero, zero, s[2])
    R = m3_cols(1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - r * z), 2.0 * (x * z + r * y),
                2.0 * (x * y + r * z), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - r * x),
                2.0 * (x * z - r * y), 2.0 * (y * z + r * x), 1.0 - 2.0 * (x * x + y * y))
    M = m3_mul(S, R)
    Sig = m3_mul(m3_T(M), M)
    c3 = [Sig[0][0], Sig[0][1], Sig[0][2], Sig[1][1], Sig[1][2], Sig[2][2]]
    # computeCov2D (forward.cu:74-113)
    fx = E(float(W)) / (2.0 * E(float(tanfovx)))
    fy = E(float(H)) / (2.0 * E(float(tanfovy)))
    t = [_xf43(p, vw, k) for k in range(3)]
    limx, limy = f32c(1.3) * E(float(tanfovx)), f32c(1.3) * E(float(tanfovy))
    txtz, tytz = t[0] / t[2], t[1] / t[2]
    tx = fmin(limx, fmax(-limx, txtz)) * t[2]
    ty = fmin(limy, fmax(-limy, tytz)) * t[2]
    J = m3_cols(fx / t[2], zero, -(fx * tx) / (t[2] * t[2]), zero, fy / t[2],
                -(fy * ty) / (t[2] * t[2]), zero, zero, zero)
    Wm = m3_cols(*(E(np.full(P, vw[k])) for k in (0, 4, 8, 1, 5, 9, 2, 6, 10)))
    T = m3_mul(Wm, J)
    Vrk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5])
    cov = m3_mul(m3_mul(m3_T(T), m3_T(Vrk)), T)
    ca, cb, cc = cov[0][0] + f32c(0.3), cov[0][1], cov[1][1] + f32c(0.3)
    det = ca * cc - cb * cb
    det_inv = 1.0 / det
    con = (cc * det_inv, (-cb) * det_inv, ca * det_inv)
    # computeColorFromSH (forward.cu:20-71)
    cp = [float(v) for v in np.asarray(campos, np.float32).reshape(-1)]
    d = [mx - cp[0], my - cp[1], mz - cp[2]]
    ln = sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
    dx, dy, dz = d[0] / ln, d[1] / ln, d[2] / ln

    def sh(k):
        return [E(shs[:, k, c].astype(np.float64)) for c in range(3)]

    res = [SH_C0 * v for v in sh(0)]
    if sh_degree > 0:
        for c in range(3):
            res[c] = ((res[c] - (SH_C1 * dy) * sh(1)[c]) + (SH_C1 * dz) * sh(2)[c]) - \
                (SH_C1 * dx) * sh(3)[c]
        if sh_degree > 1:
            xx, yy, zz = dx * dx, dy * dy, dz * dz
            xy, yz, xz = dx * dy, dy * dz, dx * dz
            basis = [SH_C2[0] * xy, SH_C2[1] * yz, SH_C2[2] * ((2.0 * zz - xx) - yy),
                     SH_C2[3] * xz, SH_C2[4] * (xx - yy)]
            if sh_degree > 2:
                basis += [(SH_C3[0] * dy) * ((3.0 * xx) - yy), (SH_C3[1] * xy) * dz,
                          (SH_C3[2] * dy) * ((4.0 * zz - xx) - yy),
                          (SH_C3[3] * dz) * ((2.0 * zz - 3.0 * xx) - 3.0 * yy),
                          (SH_C3[4] * dx) * ((4.0 * zz - xx) - yy), (SH_C3[5] * dz) * (xx - yy),
                          (SH_C3[6] * dx) * (xx - 3.0 * yy)]
            for j, bj in enumerate(basis):
                cf = sh(4 + j)
                for c in range(3):
                    res[c] = res[c] + bj * cf[c]
    rgb = [fmax(v + 0.5, 0.0) for v in res]
    # language feature: normalize(SH_C0 * l) (gaussian_renderer/__init__.py:280-287)
    u = [SH_C0 * E(lang[:, k].astype(np.float64)) for k in range(3)]
    n = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2])
    den = n + f32c(1e-9)
    feat = [uk / den for uk in u]
    op = E(np.asarray(opacity, np.float32).reshape(-1).astype(np.float64))
    cols = [px, py, con[0], con[1], con[2], op, depth] + rgb + feat
    return (np.stack([c.v for c in cols], 1), np.stack([c.e for c in cols], 1))


def bound_stats(got, f64, bound, rows, C, rel=1e-5):
    """Per column over `rows`: |got - f64| against max(rel |f64|, C u B) -- the worst ratio to
    u B, the worst relative error, the failures and the bitwise-equal fraction."""
    U = 2.0 ** -24
    out = {}
    for k, name in enumerate(COLUMNS):
        g, r, b = got[rows, k].astype(np.float64), f64[rows, k], bound[rows, k]
        if g.size == 0:
            out[name] = {"n": 0}
            continue
        d = np.abs(g - r)
        ub = U * np.maximum(b, 1e-300)
        ok = d <= np.maximum(rel * np.abs(r), C * ub)
        with np.errstate(divide="ignore", invalid="ignore"):
            relerr = np.where(np.abs(r) > 0, d / np.abs(r), d)
        out[name] = {"n": int(g.size), "ratio_max": float((d / ub).max()),
                     "ratio_p999": float(np.quantile(d / ub, 0.999)),
                     "rel_max": float(relerr.max()), "fail": int((~ok).sum())}
    return out


def camera_args(cam):
    return dict(view=cam.world_view_transform.cpu().numpy().reshape(-1),
                proj=cam.full_proj_transform.cpu().numpy().reshape(-1),
                campos=cam.camera_center.cpu().numpy(), tanfovx=math.tan(cam.FoVx * 0.5),
                tanfovy=math.tan(cam.FoVy * 0.5), W=cam.image_width, H=cam.image_height)

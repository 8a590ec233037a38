"""PLY on-disk format of the Gaussians, without plyfile.

Byte-compatible with what the reference writes through plyfile (`PlyData([PlyElement.describe(
elements, 'vertex')]).write(path)`): header `ply / format binary_little_endian 1.0 / element
vertex N / property float <name>... / end_header`, then N packed little-endian records.
  construct_list_of_attributes  <- scene/gaussian_model.py:286-301
  save_ply / load_ply           <- :303-325 / :357-398 (load_ply, like the reference, restores
                                   xyz, features, opacity, scales, rotations; the language
                                   feature only with load_language=True)
  fetch_ply / store_ply         <- scene/dataset_readers.py:485-511 (point clouds)
The reference builds each record with `list(map(tuple, attributes))` (a Python loop); here the
attribute matrix is written as one float32 block, which has the identical byte layout.
Host-side I/O; tensors come from / go to the model's device.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import nn

_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
          "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4",
          "uint32": "u4", "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}
_NAMES = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint",
          "f4": "float", "f8": "double"}


def write_ply(path, columns, element="vertex"):
    """columns: list of (name, 1-D array, numpy dtype code like 'f4' / 'u1'), all of length N."""
    n = len(columns[0][1]) if columns else 0
    dtype = np.dtype([(name, "<" + code) for name, _, code in columns])
    rec = np.empty(n, dtype=dtype)
    for name, arr, _ in columns:
        rec[name] = arr
    header = ["ply", "format binary_little_endian 1.0", f"element {element} {n}"]
    header += [f"property {_NAMES[code]} {name}" for name, _, code in columns]
    header.append("end_header")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(rec.tobytes())


def _write_f4_block(path, names, block):
    """Fast path for all-float32 records: the [N, len(names)] matrix IS the record array."""
    block = np.ascontiguousarray(block, dtype="<f4")
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {block.shape[0]}"]
    header += [f"property float {n}" for n in names]
    header.append("end_header")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(block.tobytes())


def read_ply(path, element="vertex"):
    """-> (structured numpy array of `element`, property names in file order).  Formats: ascii,
    binary_little_endian, binary_big_endian; list properties are supported only on elements after
    the requested one."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii").split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = [tok[1], int(tok[2]), []]
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    cur[2].append((tok[4], None))
                else:
                    cur[2].append((tok[2], _TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        order = {"binary_little_endian": "<", "binary_big_endian": ">", "ascii": "<"}[fmt]
        for name, count, props in elements:
            if any(code is None for _, code in props):
                if name == element:
                    raise ValueError("list properties in the requested element are not supported")
                raise ValueError(f"element '{name}' with list properties precedes '{element}'")
            dtype = np.dtype([(p, order + code) for p, code in props])
            if fmt == "ascii":
                rows = [f.readline().split() for _ in range(count)]
                data = np.array([tuple(r) for r in rows], dtype=dtype) if count else \
                    np.empty(0, dtype)
            else:
                data = np.frombuffer(f.read(dtype.itemsize * count), dtype=dtype, count=count)
            if name == element:
                return data, [p for p, _ in props]
    raise ValueError(f"{path}: no element '{element}'")


def construct_list_of_attributes(self):
    """scene/gaussian_model.py:286-301."""
    names = ["x", "y", "z", "nx", "ny", "nz"]
    names += [f"f_dc_{i}" for i in range(self._features_dc.shape[1] * self._features_dc.shape[2])]
    names += [f"f_rest_{i}"
              for i in range(self._features_rest.shape[1] * self._features_rest.shape[2])]
    names.append("opacity")
    names += [f"scale_{i}" for i in range(self._scaling.shape[1])]
    names += [f"rot_{i}" for i in range(self._rotation.shape[1])]
    if getattr(self, "_language_feature", None) is not None:
        names += [f"languagefeature_{i}" for i in range(self._language_feature.shape[1])]
    return names


def save_ply(self, path):
    """scene/gaussian_model.py:303-325: SH stored channel-major (transpose(1, 2) then flatten)."""
    with torch.no_grad():
        xyz = self._xyz.detach()
        parts = [xyz, torch.zeros_like(xyz),
                 self._features_dc.detach().transpose(1, 2).flatten(start_dim=1),
                 self._features_rest.detach().transpose(1, 2).flatten(start_dim=1),
                 self._opacity.detach(), self._scaling.detach(), self._rotation.detach()]
        if getattr(self, "_language_feature", None) is not None:
            parts.append(self._language_feature.detach())
        block = torch.cat([p.reshape(p.shape[0], -1).float() for p in parts], dim=1).cpu().numpy()
    _write_f4_block(path, construct_list_of_attributes(self), block)


def _sorted_cols(names, prefix):
    cols = [n for n in names if n.startswith(prefix)]
    return sorted(cols, key=lambda x: int(x.split("_")[-1]))


def load_ply(self, path, load_language=False, device=None):
    """scene/gaussian_model.py:357-398."""
    v, names = read_ply(path)
    dev = device if device is not None else getattr(self._xyz, "device", "cuda")
    n = v.shape[0]
    col = lambda c: np.asarray(v[c], dtype=np.float64)  # noqa: E731
    xyz = np.stack([col("x"), col("y"), col("z")], axis=1)
    opac = col("opacity")[:, None]
    dc = np.stack([col(f"f_dc_{i}") for i in range(3)], axis=1)[:, :, None]      # [P,3,1]
    extra = _sorted_cols(names, "f_rest_")
    if len(extra) != 3 * (self.max_sh_degree + 1) ** 2 - 3:
        raise ValueError(f"{path}: {len(extra)} f_rest columns for max_sh_degree "
                         f"{self.max_sh_degree}")
    rest = (np.stack([col(c) for c in extra], axis=1) if extra else np.zeros((n, 0)))
    rest = rest.reshape(n, 3, (self.max_sh_degree + 1) ** 2 - 1)
    scales = np.stack([col(c) for c in _sorted_cols(names, "scale_")], axis=1)
    rots = np.stack([col(c) for c in _sorted_cols(names, "rot")], axis=1)

    def param(a, transpose=False):
        t = torch.tensor(a, dtype=torch.float, device=dev)
        if transpose:
            t = t.transpose(1, 2).contiguous()
        return nn.Parameter(t.requires_grad_(True))

    self._xyz = param(xyz)
    self._features_dc = param(dc, True)
    self._features_rest = param(rest, True)
    self._opacity = param(opac)
    self._scaling = param(scales)
    self._rotation = param(rots)
    lang = _sorted_cols(names, "languagefeature_")
    if load_language and lang:
        self._language_feature = param(np.stack([col(c) for c in lang], axis=1))
    self.active_sh_degree = self.max_sh_degree


def fetch_ply(path):
    """scene/dataset_readers.py:485-494 -> (positions [N,3], colors [N,3] in [0,1], normals|None)."""
    v, names = read_ply(path)
    pos = np.vstack([v["x"], v["y"], v["z"]]).T
    colors = np.vstack([v["red"], v["green"], v["blue"]]).T / 255.0
    normals = np.vstack([v["nx"], v["ny"], v["nz"]]).T if "nx" in names else None
    return pos, colors, normals


def store_ply(path, xyz, rgb):
    """scene/dataset_readers.py:496-511 (float xyz, zero normals, uchar colours)."""
    xyz = np.asarray(xyz)
    rgb = np.asarray(rgb)
    cols = [(n, xyz[:, i], "f4") for i, n in enumerate("xyz")]
    cols += [(n, np.zeros(len(xyz)), "f4") for n in ("nx", "ny", "nz")]
    cols += [(n, rgb[:, i], "u1") for i, n in enumerate(("red", "green", "blue"))]
    write_ply(path, cols)


METHODS = ("construct_list_of_attributes", "save_ply", "load_ply")


def install(cls):
    g = globals()
    for name in METHODS:
        setattr(cls, name, g[name])
    return cls

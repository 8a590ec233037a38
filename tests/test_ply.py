"""PLY format (gsr_amd.ply) against the reference's layout (scene/gaussian_model.py:286-398,
scene/dataset_readers.py:485-511 via plyfile).  plyfile is not installed: its binary writer is
restated here byte by byte (header lines joined by newlines, records packed little-endian) as the
independent check.  Host-only tests (no GPU)."""
import numpy as np
import pytest
import torch

from gsr_amd import ply
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_gaussians


def _plyfile_bytes(names_codes, rows):
    """What PlyData([PlyElement.describe(structured, 'vertex')]).write() emits (binary LE)."""
    tname = {"f4": "float", "u1": "uchar"}
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {len(rows)}"]
    head += [f"property {tname[c]} {n}" for n, c in names_codes]
    head.append("end_header")
    rec = np.empty(len(rows), dtype=[(n, "<" + c) for n, c in names_codes])
    rec[:] = list(map(tuple, rows))            # the reference's record construction
    return ("\n".join(head) + "\n").encode() + rec.tobytes()


def _model(P=257, lang=True):
    m = SplatModel(make_gaussians(P, sh_degree=3, seed=2), device="cpu")
    if not lang:
        m._language_feature = None
    return m


@pytest.mark.parametrize("lang", [True, False])
def test_save_ply_bytes_match_reference_layout(tmp_path, lang):
    m = _model(lang=lang)
    path = str(tmp_path / "pc" / "point_cloud.ply")
    m.save_ply(path)
    names = m.construct_list_of_attributes()
    assert names[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert len(names) == 6 + 3 + 45 + 1 + 3 + 4 + (3 if lang else 0)
    # the reference's attribute matrix (gaussian_model.py:306-322)
    parts = [m._xyz.detach().numpy(), np.zeros((257, 3), np.float32),
             m._features_dc.detach().transpose(1, 2).flatten(start_dim=1).numpy(),
             m._features_rest.detach().transpose(1, 2).flatten(start_dim=1).numpy(),
             m._opacity.detach().numpy(), m._scaling.detach().numpy(),
             m._rotation.detach().numpy()]
    if lang:
        parts.append(m._language_feature.detach().numpy())
    attrs = np.concatenate(parts, axis=1)
    expect = _plyfile_bytes([(n, "f4") for n in names], attrs)
    assert open(path, "rb").read() == expect


def test_load_ply_round_trip(tmp_path):
    m = _model()
    path = str(tmp_path / "a.ply")
    m.save_ply(path)
    m2 = _model(P=5)
    m2.load_ply(path, device="cpu")
    for a in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
        assert torch.equal(getattr(m2, a).detach(), getattr(m, a).detach()), a
        assert isinstance(getattr(m2, a), torch.nn.Parameter)
    assert m2._language_feature.shape[0] == 5   # the reference's load_ply leaves it alone
    m2.load_ply(path, load_language=True, device="cpu")
    assert torch.equal(m2._language_feature.detach(), m._language_feature.detach())


def test_load_ply_checks_sh_degree(tmp_path):
    m = _model()
    path = str(tmp_path / "a.ply")
    m.save_ply(path)
    m2 = SplatModel(make_gaussians(4, sh_degree=2, seed=0), device="cpu")
    with pytest.raises(ValueError):
        m2.load_ply(path, device="cpu")


def test_point_cloud_store_fetch(tmp_path):
    rng = np.random.default_rng(0)
    xyz = rng.standard_normal((100, 3))
    rgb = rng.integers(0, 256, (100, 3))
    path = str(tmp_path / "points3D.ply")
    ply.store_ply(path, xyz, rgb)
    names = [("x", "f4"), ("y", "f4"), ("z", "f4"), ("nx", "f4"), ("ny", "f4"), ("nz", "f4"),
             ("red", "u1"), ("green", "u1"), ("blue", "u1")]
    rows = np.concatenate((xyz, np.zeros_like(xyz), rgb), axis=1)
    assert open(path, "rb").read() == _plyfile_bytes(names, rows)
    pos, col, nrm = ply.fetch_ply(path)
    assert np.array_equal(pos, xyz.astype(np.float32))
    assert np.allclose(col, rgb / 255.0) and np.all(nrm == 0)


def test_read_ascii_and_big_endian(tmp_path):
    p1 = tmp_path / "a.ply"
    p1.write_bytes(b"ply\nformat ascii 1.0\ncomment x\nelement vertex 2\nproperty float x\n"
                   b"property uchar red\nend_header\n1.5 7\n-2 255\n")
    v, names = ply.read_ply(str(p1))
    assert names == ["x", "red"] and v["x"].tolist() == [1.5, -2.0] and v["red"].tolist() == [7, 255]
    p2 = tmp_path / "b.ply"
    rec = np.array([(1.25, 3)], dtype=[("x", ">f4"), ("n", ">i4")])
    p2.write_bytes(b"ply\nformat binary_big_endian 1.0\nelement vertex 1\nproperty float x\n"
                   b"property int n\nend_header\n" + rec.tobytes())
    v, _ = ply.read_ply(str(p2))
    assert v["x"][0] == 1.25 and v["n"][0] == 3


@pytest.mark.gpu
def test_from_point_cloud_matches_create_from_pcd():
    """create_from_pcd (gaussian_model.py:189-214) restated in torch with the CPU KNN oracle."""
    from oracle.oracle import dist_knn3
    rng = np.random.default_rng(1)
    pts = rng.standard_normal((3000, 3))
    cols = rng.random((3000, 3))
    m = SplatModel.from_point_cloud(pts, cols)
    p32 = torch.tensor(pts).float()
    d, _ = dist_knn3(p32.numpy())
    dist2 = torch.clamp_min(torch.from_numpy(d), 0.0000001)
    scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
    assert torch.equal(m._xyz.detach().cpu(), p32)
    # device vs host log/sqrt differ by an ulp: absolute bound on the log-scale
    torch.testing.assert_close(m._scaling.detach().cpu(), scales, rtol=1e-6, atol=1e-6)
    C0 = 0.28209479177387814
    # RGB2SH: the device divides by the scalar as a multiply by its reciprocal (an ulp)
    torch.testing.assert_close(m._features_dc.detach().cpu()[:, 0],
                               (torch.tensor(cols).float() - 0.5) / C0, rtol=1e-6, atol=1e-7)
    assert torch.all(m._features_rest == 0) and torch.all(m._rotation[:, 0] == 1)
    x = torch.tensor(0.1)
    assert torch.allclose(torch.sigmoid(m._opacity), torch.full_like(m._opacity, 0.1))
    assert m.active_sh_degree == 0 and float(torch.log(x / (1 - x))) == float(m._opacity[0])

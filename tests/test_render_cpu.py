"""CPU checks of the camera-image row (§8(f) rank 4, pybullet.py:69-264): the
oracle's restatement of render()/deproject() against the goldens the
reference's own code produced (tests/golden/make_render_golden.py), and the
host-only camera arithmetic of libpandasim (ps_camera) against them."""
import ctypes as C

import numpy as np
import pytest
import render_oracle as RO


def _cams(g):
    for k in range(int(g["n_cameras"])):
        yield k, {n[len(f"c{k}_"):]: v for n, v in g.items() if n.startswith(f"c{k}_")}


def test_oracle_render_postprocessing_matches_reference_goldens(render_golden):
    for k, c in _cams(render_golden):
        pts, cols, pix2d, flat = RO.deproject_image(c["depth_in"], c["tran"], c["px_in"])
        # same numpy operations in the same order: bit for bit
        assert np.array_equal(pts, c["points"]), k
        assert np.array_equal(cols, c["colors"]), k
        assert np.array_equal(pix2d, c["pixels_2d"]), k
        assert np.array_equal(c["depth"], c["depth_in"].astype(np.float64)), k
        # rgb: the reference returns the channel-swapped (cv2 BGR2RGB) pixels
        assert np.array_equal(c["rgb"], c["px_in"][:, :, 2::-1]), k


def test_oracle_deproject_matches_reference_goldens(render_golden):
    for k, c in _cams(render_golden):
        w, h = int(c["camera"][0]), int(c["camera"][1])
        assert np.array_equal(RO.deproject(c["depth"], c["pixels"], c["tran"], w, h), c["deproject"]), k


def test_camera_tran_is_inverse_of_projection_times_view(render_golden):
    for k, c in _cams(render_golden):
        P = np.asarray(c["proj"], np.float64).reshape(4, 4, order="F")
        V = np.asarray(c["view"], np.float64).reshape(4, 4, order="F")
        assert np.allclose(c["tran"] @ (P @ V), np.eye(4), atol=1e-9), k


def test_ps_camera_host_arithmetic(render_golden):
    """libpandasim's ps_camera (host code, no GPU) against the matrices and
    inv(P V) of the goldens (the matrices themselves are the oracle's restated
    formula: unpinned against PyBullet, which is absent)."""
    from pandasim import _lib as L

    lib = L.lib()
    for k, c in _cams(render_golden):
        w, h, tx, ty, tz, dist, yaw, pitch, roll = c["camera"]
        view, proj, tran = (C.c_float * 16)(), (C.c_float * 16)(), (C.c_double * 16)()
        rc = lib.ps_camera((C.c_float * 3)(tx, ty, tz), dist, yaw, pitch, roll, int(w), int(h), view, proj, tran)
        assert rc == 0
        assert np.allclose(np.array(view[:]), c["view"], atol=2e-7), k
        assert np.array_equal(np.array(proj[:], np.float32), c["proj"]), k
        t = np.array(tran[:]).reshape(4, 4)
        assert np.allclose(t, c["tran"], rtol=1e-5, atol=1e-6 * np.abs(c["tran"]).max()), k


def test_mgrid_sizes_the_reference_cannot_render():
    from pandasim.sim import PandaSim

    PandaSim._check_image_size(480, 480)
    PandaSim._check_image_size(64, 48)
    with pytest.raises(ValueError):
        PandaSim._check_image_size(49, 64)  # np.mgrid[-1:1:2/49] has 50 entries

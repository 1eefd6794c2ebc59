"""The hand-written device model (mhpc_model.h) compiled for the host vs the reference's
CasADi kernels (committed known-answer vectors) -- the CPU-side check of the physics."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from _util import KAT_TOL, golden, rel_err

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "model_hostcheck.cpp")
SO = os.path.join(ROOT, "tests", "_build", "libmodel_hostcheck.so")


@pytest.fixture(scope="module")
def hc():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", SO, SRC], check=True)
    return ctypes.CDLL(SO)


def P(a):
    return np.ascontiguousarray(a).ctypes.data_as(ctypes.POINTER(ctypes.c_double))


@pytest.fixture(scope="module")
def kat():
    return golden("kat_model.npz")


@pytest.mark.parametrize("mode,name", [(1, "Dyn_BS"), (2, "Dyn_FL"), (3, "Dyn_FS")])
def test_dynamics_and_jacobians(hc, kat, mode, name):
    x, u = kat["x"], kat["u"]
    for i in range(len(x)):
        xd, y = np.zeros(14), np.zeros(4)
        hc.hc_wb_dynamics(P(x[i]), P(u[i]), mode, P(xd), P(y))
        assert rel_err(xd, kat[name + ".xdot"][i]) < KAT_TOL["value"]
        assert rel_err(y, kat[name + ".y"][i]) < KAT_TOL["value"]
        A, B, C, D = np.zeros(196), np.zeros(56), np.zeros(56), np.zeros(16)
        hc.hc_wb_partials(P(x[i]), P(u[i]), mode, P(A), P(B), P(C), P(D))
        assert rel_err(A.reshape(14, 14, order="F"), kat[name + "_par.Ac"][i]) < KAT_TOL["jac"]
        assert rel_err(B.reshape(14, 4, order="F"), kat[name + "_par.Bc"][i]) < KAT_TOL["jac"]
        assert rel_err(C.reshape(4, 14, order="F"), kat[name + "_par.C"][i]) < KAT_TOL["jac"]
        assert rel_err(D.reshape(4, 4, order="F"), kat[name + "_par.D"][i]) < KAT_TOL["jac"]


@pytest.mark.parametrize("mode,name", [(1, "Dyn_BS"), (2, "Dyn_FL"), (3, "Dyn_FS"), (4, "Dyn_FL")])
def test_jacobians_by_implicit_differentiation(hc, kat, mode, name):
    """The partials kernel's method (implicit differentiation of the KKT system at the
    knot's solution, wb_partial_column) vs the reference's CasADi Jacobians and vs
    forward-mode dual numbers through the whole forward dynamics (the same derivative)."""
    x, u = kat["x"], kat["u"]
    worst = 0.0
    for i in range(len(x)):
        A, B, C, D = np.zeros(196), np.zeros(56), np.zeros(56), np.zeros(16)
        hc.hc_wb_partials_ift(P(x[i]), P(u[i]), mode, P(A), P(B), P(C), P(D))
        A2, B2, C2, D2 = np.zeros(196), np.zeros(56), np.zeros(56), np.zeros(16)
        hc.hc_wb_partials(P(x[i]), P(u[i]), mode, P(A2), P(B2), P(C2), P(D2))
        for m, m2, key, shape in ((A, A2, "Ac", (14, 14)), (B, B2, "Bc", (14, 4)),
                                  (C, C2, "C", (4, 14)), (D, D2, "D", (4, 4))):
            assert rel_err(m.reshape(shape, order="F"), kat[f"{name}_par.{key}"][i]) < KAT_TOL["jac"]
            worst = max(worst, rel_err(m, m2))
    assert worst < 1e-10, worst


@pytest.mark.parametrize("foot,name", [(0, "Imp_F"), (1, "Imp_B")])
def test_impact(hc, kat, foot, name):
    for i, x in enumerate(kat["x"]):
        xp, lam, Px = np.zeros(14), np.zeros(2), np.zeros(196)
        hc.hc_wb_impact(P(x), foot, P(xp), P(lam))
        hc.hc_wb_impact_par(P(x), foot, P(Px))
        assert rel_err(xp, kat[name + ".xplus"][i]) < KAT_TOL["value"]
        assert rel_err(lam, kat[name + ".y"][i][2 * foot:2 * foot + 2]) < KAT_TOL["value"]
        assert rel_err(Px.reshape(14, 14, order="F"), kat[name + "_par.Px"][i]) < KAT_TOL["jac"]


@pytest.mark.parametrize("foot,name", [(0, "WB_FL1_terminal_constr"), (1, "WB_FL2_terminal_constr")])
def test_touchdown_constraint(hc, kat, foot, name):
    for i, x in enumerate(kat["x"]):
        h, hx, hxx = np.zeros(1), np.zeros(14), np.zeros(196)
        hc.hc_wb_touchdown(P(x), foot, P(h), P(hx), P(hxx))
        assert abs(h[0] - kat[name + ".h"][i]) < 1e-14
        assert rel_err(hx, kat[name + ".hx"][i]) < 1e-14
        assert rel_err(hxx.reshape(14, 14), kat[name + ".hxx"][i]) < 1e-14


@pytest.mark.parametrize("foot,name", [(0, "Jacob_F"), (1, "Jacob_B")])
def test_foot_jacobian(hc, kat, foot, name):
    for i, x in enumerate(kat["x"]):
        J, Jd = np.zeros(14), np.zeros(14)
        hc.hc_wb_foot_jacobian(P(x), foot, P(J), P(Jd))
        assert rel_err(J.reshape(2, 7), kat[name + ".J"][i]) < 1e-14
        assert rel_err(Jd.reshape(2, 7), kat[name + ".Jd"][i]) < 1e-13


def test_srb_bit_exact(hc, kat):
    for i in range(len(kat["srb.x"])):
        args = [kat[k][i] for k in ("srb.x", "srb.u", "srb.p", "srb.s")]
        xd, A, B = np.zeros(6), np.zeros(36), np.zeros(24)
        hc.hc_srb_dynamics(*[P(a) for a in args], P(xd))
        hc.hc_srb_jacobians(*[P(a) for a in args], P(A), P(B))
        np.testing.assert_array_equal(xd, kat["FBDynamics.xdot"][i])
        np.testing.assert_array_equal(A.reshape(6, 6), kat["FBDynamics_par.Ac"][i])
        np.testing.assert_array_equal(B.reshape(6, 4), kat["FBDynamics_par.Bc"][i])

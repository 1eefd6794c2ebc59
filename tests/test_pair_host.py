"""The lane-pair whole-body dynamics (mhpc_model_pair.h) vs the single-lane model
(mhpc_model.h) on the host: the pair emulated by two threads (tests/native/
pair_hostcheck.cpp), both without FMA contraction as on the device.  Bitwise equality =
the two models perform the same operations in the same order, which is what makes the line
search's result independent of the variant (pair / single lane) a batch size selects."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from _util import golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "pair_hostcheck.cpp")
SO = os.path.join(ROOT, "tests", "_build", "libpair_hostcheck.so")


@pytest.fixture(scope="module")
def hc():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-fPIC", "-shared",
                    "-pthread", "-o", SO, SRC], check=True)
    return ctypes.CDLL(SO)


def P(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_pair_equals_single_lane(hc, mode):
    kat = golden("kat_model.npz")
    rng = np.random.default_rng(mode)
    xs = np.concatenate([kat["x"], kat["x"] + 0.1 * rng.standard_normal(kat["x"].shape)])
    us = np.concatenate([kat["u"], 5 * rng.standard_normal(kat["u"].shape)])
    for x, u in zip(xs, us):
        x, u = np.ascontiguousarray(x), np.ascontiguousarray(u)
        xd, y = np.zeros(14), np.zeros(4)
        hc.hc_wb_dynamics(P(x), P(u), mode, P(xd), P(y))
        xd2, y2 = np.zeros((2, 14)), np.zeros((2, 4))
        hc.hc_wb_dynamics_pair(P(x), P(u), mode, P(xd2), P(y2))
        for lane in (0, 1):
            np.testing.assert_array_equal(xd2[lane], xd, err_msg=f"mode {mode} lane {lane}")
            np.testing.assert_array_equal(y2[lane], y, err_msg=f"mode {mode} lane {lane}")

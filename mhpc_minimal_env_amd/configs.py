"""The BASELINE.json workloads as problem descriptors (mapping: SURVEY.md App. C).

C1  1 SRB phase (mode 1), dt_fb = (float)0.0016, N = 50   -- MultiPhaseDDP(1) + SinglePhase<6,4,4>
C2  1 WB phase (mode 1), dt_wb = (float)(0.08f/120), N = 120
C3  2 WB (modes 1,2) + 2 SRB (modes 3,4), Gait(GaitType2D::PRONK) = default branch,
    uniform 0.08 s, dt = (float)0.001 -> N = 80 each; "trot" in BASELINE.json
C4  = C3, sharded over GPUs
C5  Gait() BOUND, 4 WB + 6 SRB; c5f32_desc() runs it in the fp32 instantiation (BASELINE.json)
demo  test_main.cpp: default MHPCUserParameters (4 WB + 4 SRB), Gait() BOUND, default x0
"""
from __future__ import annotations

import numpy as np

from . import locomotion as L


def c1_desc():
    d = L.make_problem_desc(0, 1, [1], [0.08], 0.001, 0.0016, 1.5)
    assert d.N[0] == 50, d.N[0]
    return d


def c2_desc():
    dt = float(np.float32(np.float32(0.08) / np.float32(120)))
    return L.make_problem_desc(1, 0, [1], [0.08], dt, 0.001, 1.5, N=[120])


def c3_desc():
    params = L.MHPCUserParameters(n_wbphase=2, n_fbphase=2, usrcmd=L.USRCMD(vel=1.5))
    return L.desc_from_params(params, L.Gait(L.GaitType2D.PRONK))


def c5_desc(precision: int = 64):
    params = L.MHPCUserParameters(n_wbphase=4, n_fbphase=6, usrcmd=L.USRCMD(vel=1.5))
    d = L.desc_from_params(params, L.Gait())
    d.precision = precision
    return d


def c5f32_desc():
    """C5 in the fp32 instantiation of the solve path (BASELINE.json configs[4])."""
    return c5_desc(32)


def demo_desc():
    """test_main.cpp's problem: default MHPCUserParameters (4 WB + 4 SRB), Gait() BOUND."""
    return L.desc_from_params(L.MHPCUserParameters(usrcmd=L.USRCMD(vel=1.5)), L.Gait())


def c3_at(cmode: int):
    """C3 at another point of its gait cycle: the layout MHPCLocomotion::build_problem makes
    for a controller whose current mode is cmode (the PRONK / default-branch gait)."""
    params = L.MHPCUserParameters(n_wbphase=2, n_fbphase=2, cmode=cmode, usrcmd=L.USRCMD(vel=1.5))
    return L.desc_from_params(params, L.Gait(L.GaitType2D.PRONK))


def c5_at(cmode: int, precision: int = 64):
    """C5 (bound) at current mode cmode."""
    params = L.MHPCUserParameters(n_wbphase=4, n_fbphase=6, cmode=cmode, usrcmd=L.USRCMD(vel=1.5))
    d = L.desc_from_params(params, L.Gait())
    d.precision = precision
    return d


def mixed_descs():
    """The mixed workload (north_star's batch axis over gait schedules): controllers at every
    point of the C3 trot cycle and at two points of the C5 bound cycle; problem b takes
    layout b % 6 (two thirds C3, one third C5)."""
    return [c3_at(1), c3_at(2), c3_at(3), c3_at(4), c5_at(1), c5_at(3)]


def x0_rows(descs, layout_of_problem, offset: int = 0):
    """Initial states of a mixed batch (rows of 14; an SRB-only problem's state in the first
    6 entries of its row, as mhpc_set_x0 reads it), the same stream as x0_for."""
    lop = np.asarray(layout_of_problem)
    x0 = L.random_x0(len(lop), offset=offset)
    for b, l in enumerate(lop):
        if descs[l].n_wb == 0:
            x0[b, :6] = x0[b, L.STATE_PROJ_ROWS]
            x0[b, 6:] = 0
    return np.ascontiguousarray(x0)


def x0_for(desc, batch: int, offset: int = 0):
    x0 = L.random_x0(batch, offset=offset)
    if desc.n_wb == 0:
        x0 = x0[:, L.STATE_PROJ_ROWS]
    return np.ascontiguousarray(x0)


def c2_eps(n: int = 256) -> np.ndarray:
    """C2 step sizes: j = 0..9 the reference's Armijo grid 1, 0.1, 0.1*0.1, ...
    (parity-pinned), j >= 10 eps = 0.1**(j / 25.5) (deterministic, unpinned)."""
    j = np.arange(n, dtype=np.float64)
    eps = np.power(0.1, j / 25.5)
    e = 1.0
    for k in range(min(n, 10)):  # eps *= alpha, exactly as forward_iteration steps it
        eps[k] = e
        e *= 0.1
    return eps

"""Host-side mirror of the reference's MHPC controller surface.

Same names, fields, defaults and argument meaning as the reference's C++ API:
  HSDDP_OPTION          MHPC_CompoundTypes.h:196-212
  USRCMD                MHPC_CompoundTypes.h:237-240
  MHPCUserParameters    MHPC_CompoundTypes.h:242-251   (alias MHPC_UserParameter)
  GaitType2D / Gait     Common/header/Gait.h:6-77
  MHPCLocomotion        Controller/MHPCLocomotion/MHPCLocomotion.{h,cpp}
but one MHPCLocomotion object drives a BATCH of independent problems on one GPU through
the C-ABI (include/mhpc_capi.h).  Numbers come only from the HIP library; there is no CPU
fallback in this module.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from enum import Enum
from typing import List, Optional

import numpy as np

from . import capi

PI = 3.141592653589793238  # MHPC_CPPTypes.h:18


def f32(v: float) -> float:
    """A reference `float` parameter promoted to double."""
    return float(np.float32(v))


def eigen_row(v) -> str:
    """One row as `ostream << vec.transpose()` prints it with Eigen's default IOFormat: each
    coefficient formatted like `ostream << double` (6 significant digits, %g), right-aligned
    to the widest coefficient of the row, separated by one space."""
    strs = ["%g" % float(x) for x in np.ravel(v)]
    w = max((len(t) for t in strs), default=0)
    return " ".join(t.rjust(w) for t in strs)


# ----------------------------------------------------------------------------------------
@dataclass
class HSDDP_OPTION:
    alpha: float = 0.1
    gamma: float = 0.01
    update_penalty: float = 8
    update_relax: float = 0.1
    update_regularization: float = 2
    update_ReB: float = 7
    max_DDP_iter: float = 3
    max_AL_iter: float = 2
    DDP_thresh: float = 1e-03
    AL_thresh: float = 1e-03
    AL_active: bool = True
    ReB_active: bool = True
    smooth_active: bool = False

    def to_c(self) -> capi.HsddpOption:
        o = capi.HsddpOption()
        for k in ("alpha", "gamma", "update_penalty", "update_relax", "update_regularization",
                  "update_ReB", "max_DDP_iter", "max_AL_iter", "DDP_thresh", "AL_thresh"):
            setattr(o, k, float(getattr(self, k)))
        o.AL_active = int(bool(self.AL_active))
        o.ReB_active = int(bool(self.ReB_active))
        o.smooth_active = int(bool(self.smooth_active))
        return o


@dataclass
class USRCMD:
    vel: float = 0.0
    height: float = 0.0
    roll: float = 0.0
    pitch: float = 0.0
    yaw: float = 0.0


@dataclass
class MHPCUserParameters:
    n_wbphase: int = 4
    n_fbphase: int = 4
    dt_wb: float = .001
    dt_fb: float = .001
    cmode: int = 1
    groundH: float = -0.404  # unused by the reference too (ground hard-coded)
    usrcmd: Optional[USRCMD] = None


MHPC_UserParameter = MHPCUserParameters  # the north star's spelling


class GaitType2D(Enum):
    STAND = 0
    BOUND = 1
    PRONK = 2


class Gait:
    """Gait.h:13-77.  Only BOUND is defined; every other type takes the default branch
    (uniform 0.08 s timings) exactly as the reference's switch does."""

    def __init__(self, gait: Optional[GaitType2D] = None):
        self._gait_mode = [1, 2, 3, 4]
        self._gait_name = "BOUND"
        if gait is None or gait == GaitType2D.BOUND:
            self._gait_timing = [f32(0.08), f32(0.1), f32(0.08), f32(0.1)]
        else:
            self._gait_timing = [f32(0.08)] * 4

    def get_next_mode(self, current_mode: int) -> int:
        for idx, m in enumerate(self._gait_mode):
            if m == current_mode:
                return self._gait_mode[(idx + 1) % len(self._gait_mode)]
        raise ValueError(f"mode {current_mode} not in gait")

    def get_mode_seq(self, current_mode: int, num_phases: int) -> List[int]:
        assert num_phases >= 1
        seq = [current_mode]
        for _ in range(num_phases - 1):
            seq.append(self.get_next_mode(seq[-1]))
        return seq

    def get_timings(self, mode_seq: List[int]) -> List[float]:
        return [self._gait_timing[m - 1] for m in mode_seq]

    def to_c(self) -> capi.GaitC:
        g = capi.GaitC()
        g.n_modes = len(self._gait_mode)
        for i, m in enumerate(self._gait_mode):
            g.modes[i] = m
        for i, t in enumerate(self._gait_timing):
            g.timings[i] = t
        return g


def c_round(v: float) -> int:
    """C `round()` (half away from zero)."""
    return int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)


def make_problem_desc(n_wb: int, n_fb: int, mode_seq: List[int], timings: List[float],
                      dt_wb: float, dt_fb: float, vel: float, height: float = 0.0,
                      N: Optional[List[int]] = None) -> capi.ProblemDesc:
    """MHPCLocomotion::build_problem (MHPCLocomotion.cpp:63-104): N = round(timing / dt)
    with float timings and float dt promoted to double."""
    d = capi.ProblemDesc()
    np_ = n_wb + n_fb
    if not 1 <= np_ <= capi.MHPC_MAX_PHASES:
        raise ValueError("number of phases out of range")
    d.n_wb, d.n_fb = n_wb, n_fb
    d.dt_wb, d.dt_fb = f32(dt_wb), f32(dt_fb)
    for p in range(np_):
        d.mode_seq[p] = mode_seq[p]
        if N is not None:
            d.N[p] = N[p]
        else:
            dt = d.dt_wb if p < n_wb else d.dt_fb
            d.N[p] = c_round(f32(timings[p]) / dt)
    d.vel_cmd = f32(vel)
    d.height_cmd = f32(height)
    d.precision = 64
    return d


def desc_from_params(params: MHPCUserParameters, gait: Gait) -> capi.ProblemDesc:
    n = params.n_wbphase + params.n_fbphase
    seq = gait.get_mode_seq(params.cmode, n)
    cmd = params.usrcmd or USRCMD()
    return make_problem_desc(params.n_wbphase, params.n_fbphase, seq, gait.get_timings(seq),
                             params.dt_wb, params.dt_fb, cmd.vel, cmd.height)


# Default initial condition (MHPCLocomotion.cpp:37-39)
Q0 = np.array([0.0927, -0.1093, -0.1542, 1.0957, -2.2033, 0.9742, -1.7098])
QD0 = np.array([0.9011, 0.2756, 0.7333, 0.0446, 0.0009, 1.3219, 2.7346])
X0_DEFAULT = np.concatenate([Q0, QD0])
STATE_PROJ_ROWS = [0, 1, 2, 7, 8, 9]  # _stateProj (MHPCLocomotion.cpp:32-34)

X0_SEED = 0x4D485043
_X0_AMP = np.array([0.01, 0.01] + [0.02] * 5 + [0.05] * 7)
_M64 = (1 << 64) - 1


def _splitmix64(state: int):
    state = (state + 0x9E3779B97F4A7C15) & _M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return state, z ^ (z >> 31)


def random_x0(batch: int, seed: int = X0_SEED, offset: int = 0) -> np.ndarray:
    """x0_b = x0_default + delta_b.  Problem b draws from its own
    splitmix64 stream, state0 = seed ^ (b * 0xD1B54A32D192ED03); U = (next >> 11) * 2^-53,
    delta = amp * (2U - 1).  `offset` = global index of the first problem (sharding)."""
    out = np.empty((batch, 14))
    for i in range(batch):
        b = offset + i
        st = (seed ^ ((b * 0xD1B54A32D192ED03) & _M64)) & _M64
        for j in range(14):
            st, z = _splitmix64(st)
            U = (z >> 11) * (1.0 / (1 << 53))
            out[i, j] = X0_DEFAULT[j] + _X0_AMP[j] * (2 * U - 1)
    return out


# ----------------------------------------------------------------------------------------
class SinglePhaseView:
    """One phase of the batch after a solve, with the public members of the reference's
    SinglePhaseAbstract (SinglePhaseAbstract.h:66-134): _modeidx, _phaseidx, _dt,
    _N_TIMESTEPS, _xsize/_usize/_ysize, and _V / _dV (phase cost, expected change) as
    [batch] arrays; get_nominal_ms_ptr() / get_CTG_info_ptr() return the phase's nominal
    (x, u, y) and cost-to-go (G = Vx, du, K) arrays [batch][N][...] (MHPC_CompoundTypes.h:7-22,
    88-101).  Read lazily from the device; valid until the next solve / update_problem."""

    def __init__(self, loco: "MHPCLocomotion", p: int):
        d = loco.desc
        self._loco, self._phaseidx = loco, p
        self._modeidx = int(d.mode_seq[p])
        self._N_TIMESTEPS = int(d.N[p])
        self._xsize, self._usize, self._ysize = d.xsize(p), 4, 4
        self._dt = float(d.dt_wb if p < d.n_wb else d.dt_fb)

    def get_modeidx(self) -> int:
        return self._modeidx

    @property
    def _V(self) -> np.ndarray:
        return self._loco.get_scalars()["V"][:, self._phaseidx]

    @property
    def _dV(self) -> np.ndarray:
        return self._loco.get_scalars()["dV"][:, self._phaseidx]

    def get_nominal_ms_ptr(self) -> dict:
        q = self._loco.get_phase(self._phaseidx)
        return {"x": q["x"], "u": q["u"], "y": q["y"]}

    def get_CTG_info_ptr(self) -> dict:
        q = self._loco.get_phase(self._phaseidx)
        return {"G": q["Vx"], "du": q["du"], "K": q["K"]}

    def get_terminal_state(self) -> np.ndarray:
        return self.get_nominal_ms_ptr()["x"][:, -1, :]


class MHPCLocomotion:
    """Batched MHPCLocomotion<double> over the C-ABI.

    MHPCLocomotion(params, gait, option)               (MHPCLocomotion.cpp:8-43)
    .initialization()                                    (:47-53)
    .solve_mhpc()                                        (:167-195)
    .print_debugInfo(dirname)                            (:293-380)
    Extensions: `batch`, `set_initial_condition(x0[batch][n])` before initialization
    (the reference always starts from its private default x0), `desc=` for layouts the
    reference's constructor cannot express (SRB-only C1, N > 110 C2)."""

    def __init__(self, params: Optional[MHPCUserParameters] = None, gait: Optional[Gait] = None,
                 option: Optional[HSDDP_OPTION] = None, batch: int = 1, device: int = 0,
                 desc: Optional[capi.ProblemDesc] = None):
        self.params = params or MHPCUserParameters(usrcmd=USRCMD(vel=1.5))
        self.gait = gait or Gait()
        self.option = option or HSDDP_OPTION()
        self.desc = desc if desc is not None else desc_from_params(self.params, self.gait)
        self.batch = int(batch)
        self.device = int(device)
        self._opt_c = self.option.to_c()
        L = capi.lib()
        h = __import__("ctypes").c_void_p()
        capi.check(L.mhpc_create(self.desc, self._opt_c, self.batch, self.device,
                                 __import__("ctypes").byref(h)), "mhpc_create")
        self._h = h
        self.descs = None  # per-problem descriptors once set_layouts mixes layouts
        self._default_x0()
        self.status = np.zeros(self.batch, dtype=np.int32)

    def _x0_row(self) -> int:
        ds = self.descs or [self.desc]
        return 14 if any(d.n_wb > 0 for d in ds) else 6

    def _default_x0(self):
        n0 = self._x0_row()
        x0 = X0_DEFAULT if n0 == 14 else X0_DEFAULT[STATE_PROJ_ROWS]
        self._x0 = np.tile(x0, (self.batch, 1)).astype(np.float64)

    # -- lifecycle ---------------------------------------------------------------------
    def set_initial_condition(self, x0: np.ndarray):
        x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(self.batch, -1))
        if x0.shape[1] != self._x0_row():
            raise ValueError("x0 has the wrong state size for phase 0")
        self._x0 = x0

    def initialization(self):
        L = capi.lib()
        capi.check(L.mhpc_set_x0(self._h, capi.dptr(self._x0)), "mhpc_set_x0")
        capi.check(L.mhpc_initialize(self._h), "mhpc_initialize")

    def solve_mhpc(self) -> np.ndarray:
        capi.check(capi.lib().mhpc_solve(self._h, capi.iptr(self.status)), "mhpc_solve")
        return self.status

    def update_problem(self, gait: Optional[Gait] = None):
        """MHPCLocomotion::update_problem (MHPCLocomotion.cpp:107-158) for every problem: the
        gait advances one mode, the phase buffers rotate (warm start of the next solve), the
        references follow the x0 given to set_initial_condition."""
        L = capi.lib()
        capi.check(L.mhpc_set_x0(self._h, capi.dptr(self._x0)), "mhpc_set_x0")
        g = (gait or self.gait).to_c()
        capi.check(L.mhpc_update_problem(self._h, __import__("ctypes").byref(g)),
                   "mhpc_update_problem")
        self._refresh_descs()

    # -- per-problem phase layouts: the batch axis over gait schedules ----------------------
    def set_layouts(self, descs, layout_of_problem=None):
        """mhpc_set_layouts: problem b gets descs[layout_of_problem[b]] (descs[b % len] when
        None) -- each controller of the batch at its own gait / gait point, as the reference
        builds one layout per MHPCLocomotion instance (MHPCLocomotion.cpp:63-104).  The
        initial states return to the default; set_initial_condition + initialization follow."""
        import ctypes
        arr = (capi.ProblemDesc * len(descs))(*descs)
        lop = (None if layout_of_problem is None
               else np.ascontiguousarray(layout_of_problem, dtype=np.int32))
        capi.check(capi.lib().mhpc_set_layouts(self._h, len(descs), arr, capi.iptr(lop)),
                   "mhpc_set_layouts")
        self._refresh_descs()
        self._default_x0()

    def update_problems(self, gaits, gait_of_problem=None, steps=None):
        """Per-problem update_problem (mhpc_update_problems): problem b takes steps[b] gait
        steps of gaits[gait_of_problem[b]] (0: keeps its layout); references follow the x0 of
        set_initial_condition for every problem."""
        import ctypes
        L = capi.lib()
        capi.check(L.mhpc_set_x0(self._h, capi.dptr(self._x0)), "mhpc_set_x0")
        gs = (capi.GaitC * len(gaits))(*[g.to_c() for g in gaits])
        gop = (None if gait_of_problem is None
               else np.ascontiguousarray(gait_of_problem, dtype=np.int32))
        st = None if steps is None else np.ascontiguousarray(steps, dtype=np.int32)
        capi.check(L.mhpc_update_problems(self._h, len(gaits), gs, capi.iptr(gop), capi.iptr(st)),
                   "mhpc_update_problems")
        self._refresh_descs()

    def problem_desc(self, b: int) -> capi.ProblemDesc:
        import ctypes
        d = capi.ProblemDesc()
        capi.check(capi.lib().mhpc_get_problem_desc(self._h, int(b), ctypes.byref(d)),
                   "mhpc_get_problem_desc")
        return d

    def num_layouts(self) -> int:
        import ctypes
        n = ctypes.c_int(0)
        capi.check(capi.lib().mhpc_num_layouts(self._h, ctypes.byref(n)), "mhpc_num_layouts")
        return n.value

    def max_phases(self) -> int:
        """Row length of get_scalars' per-phase arrays (mhpc_max_phases)."""
        import ctypes
        n = ctypes.c_int(0)
        capi.check(capi.lib().mhpc_max_phases(self._h, ctypes.byref(n)), "mhpc_max_phases")
        return n.value

    def _refresh_descs(self):
        ds = [self.problem_desc(b) for b in range(self.batch)]
        key = lambda d: bytes(d)
        self.descs = ds if any(key(d) != key(ds[0]) for d in ds) else None
        self.desc = ds[0]

    def get_phase_problems(self, p: int, first: int, count: int) -> dict:
        """Phase p of problems [first, first + count) (one phase shape over the range)."""
        d = self.descs[first] if self.descs else self.desc
        n, N = d.xsize(p), d.N[p]
        out = {k: np.zeros(s) for k, s in (
            ("x", (count, N, n)), ("u", (count, N, 4)), ("y", (count, N, 4)),
            ("K", (count, N, 4, n)), ("du", (count, N, 4)), ("Vx", (count, N, n)))}
        capi.check(capi.lib().mhpc_get_phase_problems(
            self._h, p, int(first), int(count),
            *[capi.dptr(out[k]) for k in ("x", "u", "y", "K", "du", "Vx")]), "mhpc_get_phase_problems")
        return out

    def problem_concatenated(self, b: int) -> dict:
        """Phase-concatenated arrays of one problem (the oracle's layout, row b)."""
        d = self.descs[b] if self.descs else self.desc
        parts = [self.get_phase_problems(p, b, 1) for p in range(d.n_phases)]
        return {
            "X": np.concatenate([q["x"].ravel() for q in parts]),
            "U": np.concatenate([q["u"].ravel() for q in parts]),
            "Y": np.concatenate([q["y"].ravel() for q in parts]),
            "K": np.concatenate([q["K"].ravel() for q in parts]),
            "DU": np.concatenate([q["du"].ravel() for q in parts]),
            "G": np.concatenate([q["Vx"].ravel() for q in parts]),
        }

    # MultiPhaseDDP's public members (MultiPhaseDDP.h:12-63), batched: [batch] arrays
    @property
    def _phases(self):
        return [SinglePhaseView(self, p) for p in range(self.desc.n_phases)]

    @property
    def _n_phases(self) -> int:
        return self.desc.n_phases

    @property
    def _actual_cost(self) -> np.ndarray:
        return self.get_scalars()["J"]

    @property
    def _exp_cost_change(self) -> np.ndarray:
        return self.get_scalars()["dV_exp"]

    @property
    def _tconstr_violation(self) -> np.ndarray:
        return self.get_scalars()["viol"]

    # -- cost / constraint parameters (CostBase.h:9-46, ConstraintsBase.h:11-50) -----------
    def set_cost_weights(self, w: "capi.CostWeights"):
        """Replace the diagonal cost weights (MHPCCost.cpp:24-75 values by default) for every
        later solve of this handle (mhpc_set_cost_weights)."""
        capi.check(capi.lib().mhpc_set_cost_weights(self._h, __import__("ctypes").byref(w)),
                   "mhpc_set_cost_weights")

    def get_cost_weights(self) -> "capi.CostWeights":
        w = capi.CostWeights()
        capi.check(capi.lib().mhpc_get_cost_weights(self._h, __import__("ctypes").byref(w)),
                   "mhpc_get_cost_weights")
        return w

    def set_constraint_params(self, c: "capi.ConstraintParams"):
        """Replace torque limit, friction coefficient and the AL / ReB initial parameters
        (MHPCConstraints.cpp:14-88 values by default); the initial values take effect at the
        next initialization() / update_problem() (mhpc_set_constraint_params)."""
        capi.check(capi.lib().mhpc_set_constraint_params(self._h, __import__("ctypes").byref(c)),
                   "mhpc_set_constraint_params")

    def get_constraint_params(self) -> "capi.ConstraintParams":
        c = capi.ConstraintParams()
        capi.check(capi.lib().mhpc_get_constraint_params(self._h, __import__("ctypes").byref(c)),
                   "mhpc_get_constraint_params")
        return c

    def get_exec(self) -> dict:
        """Execution horizon of solve_mhpc (MHPCLocomotion.cpp:176-194): the nominal and
        cost-to-go of phase 0, followed by phase 1 when there are two WB phases."""
        parts = [self.get_phase(0)] + ([self.get_phase(1)] if self.desc.n_wb > 1 else [])
        return {k: np.concatenate([q[k] for q in parts], axis=1) for k in parts[0]}

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            capi.lib().mhpc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- outputs -----------------------------------------------------------------------
    def get_phase(self, p: int) -> dict:
        n, N, B = self.desc.xsize(p), self.desc.N[p], self.batch
        out = {k: np.zeros(s) for k, s in (
            ("x", (B, N, n)), ("u", (B, N, 4)), ("y", (B, N, 4)), ("K", (B, N, 4, n)),
            ("du", (B, N, 4)), ("Vx", (B, N, n)))}
        capi.check(capi.lib().mhpc_get_phase(
            self._h, p, *[capi.dptr(out[k]) for k in ("x", "u", "y", "K", "du", "Vx")]),
            "mhpc_get_phase")
        return out

    def get_scalars(self) -> dict:
        B = self.batch
        P = self.max_phases()  # rows of the most phases over the problems' layouts
        out = {"J": np.zeros(B), "dV_exp": np.zeros(B), "viol": np.zeros(B),
               "V": np.zeros((B, P)), "dV": np.zeros((B, P)),
               "trace": np.zeros((B, capi.MHPC_TRACE_LEN), dtype=np.int32)}
        capi.check(capi.lib().mhpc_get_scalars(
            self._h, capi.dptr(out["J"]), capi.dptr(out["dV_exp"]), capi.dptr(out["viol"]),
            capi.dptr(out["V"]), capi.dptr(out["dV"]), capi.iptr(out["trace"])),
            "mhpc_get_scalars")
        return out

    def get_counters(self) -> dict:
        c = capi.Counters()
        capi.check(capi.lib().mhpc_get_counters(self._h, __import__("ctypes").byref(c)),
                   "mhpc_get_counters")
        return {k: getattr(c, k) for k, _ in capi.Counters._fields_}

    def rollout_costs(self, eps) -> dict:
        """Trial rollouts (forward_sweep_dynamics_only) at every step size in `eps` from the
        current nominal and gains, costs only: J, viol [batch][len(eps)] and the device ms."""
        eps = np.ascontiguousarray(eps, dtype=np.float64)
        J = np.zeros((self.batch, eps.shape[0]))
        viol = np.zeros_like(J)
        ms = __import__("ctypes").c_float(0)
        capi.check(capi.lib().mhpc_rollout_costs(self._h, int(eps.shape[0]), capi.dptr(eps),
                                                 capi.dptr(J), capi.dptr(viol),
                                                 __import__("ctypes").byref(ms)),
                   "mhpc_rollout_costs")
        return {"J": J, "viol": viol, "ms": ms.value}

    def set_profiling(self, on: bool = True):
        capi.check(capi.lib().mhpc_set_profiling(self._h, 1 if on else 0), "mhpc_set_profiling")

    def kernel_stats(self) -> dict:
        n = capi.MHPC_NUM_KERNELS
        ms, nl, by = np.zeros(n), np.zeros(n, dtype=np.int64), np.zeros(n)
        capi.check(capi.lib().mhpc_get_kernel_stats(
            self._h, capi.dptr(ms), nl.ctypes.data_as(__import__("ctypes").POINTER(
                __import__("ctypes").c_int64)), capi.dptr(by)), "mhpc_get_kernel_stats")
        fl = np.zeros(n)
        capi.check(capi.lib().mhpc_get_kernel_flops(self._h, capi.dptr(fl)), "mhpc_get_kernel_flops")
        return {capi.lib().mhpc_kernel_name(k).decode(): {"ms": float(ms[k]), "launches": int(nl[k]),
                                                          "alg_bytes": float(by[k]),
                                                          "alg_flops": float(fl[k])}
                for k in range(n)}

    def reset_kernel_stats(self):
        capi.check(capi.lib().mhpc_reset_kernel_stats(self._h), "mhpc_reset_kernel_stats")

    def set_kernel_variant(self, bws: str = "auto", rollout: str = "auto", overlap: str = "auto",
                           sub_batches: int = 0, ro_store: int = 0, sweep_bits: int = 0):
        """Pin the backward-sweep / line-search launch variant, the partials / sweep
        overlap, the number of concurrently scheduled sub-batches and the number of
        line-search trials that store their knot records (mhpc_set_kernel_variant); names in
        capi.BWS_VARIANTS / capi.RO_VARIANTS / capi.OVERLAP_VARIANTS, "auto" / 0 = chosen by
        batch size and phase layout (ro_store 0: the default).  sweep_bits: arithmetic of the
        backward sweep, 0 / 64 double (default), 32 float (fp32 handles only)."""
        L = capi.lib()
        if sweep_bits or getattr(self, "_sweep_bits_pinned", False):
            capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_SWEEP_BITS,
                                                 int(sweep_bits)), "mhpc_set_kernel_variant")
            self._sweep_bits_pinned = bool(sweep_bits)
        if ro_store or getattr(self, "_ro_store_pinned", False):
            capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_RO_STORE, int(ro_store)),
                       "mhpc_set_kernel_variant")
            self._ro_store_pinned = bool(ro_store)
        capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_SUBBATCH, int(sub_batches)),
                   "mhpc_set_kernel_variant")
        capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_OVERLAP,
                                             capi.OVERLAP_VARIANTS[overlap]), "mhpc_set_kernel_variant")
        capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_BWS,
                                             capi.BWS_VARIANTS[bws]), "mhpc_set_kernel_variant")
        capi.check(L.mhpc_set_kernel_variant(self._h, capi.MHPC_VARIANT_RO,
                                             capi.RO_VARIANTS[rollout]), "mhpc_set_kernel_variant")

    def concatenated(self) -> dict:
        """Phase-concatenated per-problem arrays (the oracle's layout)."""
        parts = [self.get_phase(p) for p in range(self.desc.n_phases)]
        B = self.batch
        return {
            "X": np.concatenate([q["x"].reshape(B, -1) for q in parts], axis=1),
            "U": np.concatenate([q["u"].reshape(B, -1) for q in parts], axis=1),
            "Y": np.concatenate([q["y"].reshape(B, -1) for q in parts], axis=1),
            "K": np.concatenate([q["K"].reshape(B, -1) for q in parts], axis=1),
            "DU": np.concatenate([q["du"].reshape(B, -1) for q in parts], axis=1),
            "G": np.concatenate([q["Vx"].reshape(B, -1) for q in parts], axis=1),
        }

    def get_cost_gradients(self, p: int) -> dict:
        """lx [batch][N-1][n] and Phix [batch][n] of phase p as the last partials evaluation
        left them (the reference's rcost[k].lx / tcost.Phix, written to cost.txt)."""
        n = self.desc.xsize(p)
        N = self.desc.N[p]
        lx = np.zeros((self.batch, N - 1, n))
        phix = np.zeros((self.batch, n))
        capi.check(capi.lib().mhpc_get_cost_gradients(self._h, p, capi.dptr(lx), capi.dptr(phix)),
                   "mhpc_get_cost_gradients")
        return {"lx": lx, "Phix": phix}

    def print_debugInfo(self, dirname: str = ".", problem: int = 0, verbose: bool = True):
        """MHPCLocomotion::print_debugInfo (MHPCLocomotion.cpp:293-380) for one problem:
        state.txt, control.txt, gradient.txt, cost.txt in Eigen's default row format
        (eigen_row), with the reference's row counts -- including its N_TIMESTEPS[i+2]
        indexing of the SRB phases in control / gradient / cost (exact for n_wbphase = 2;
        rows past an SRB phase's own N are the zero-initialised buffer)."""
        os.makedirs(dirname, exist_ok=True)
        d = self.desc
        nwb, nfb, P = d.n_wb, d.n_fb, d.n_phases
        parts = [self.get_phase(p) for p in range(P)]
        grads = [self.get_cost_gradients(p) for p in range(P)]
        Ns = [d.N[p] for p in range(P)]

        def n_rows(i):  # N_TIMESTEPS[i+2] (clamped where the reference would read past it)
            return Ns[i + 2] if i + 2 < P else Ns[nwb + i]

        def rows(arr, n_want, width):
            out = [np.ravel(arr[k]) if k < len(arr) else np.zeros(width) for k in range(n_want)]
            return out

        def write(fname, blocks):
            if verbose:
                print(f"********** Write to file {fname} ************")
            with open(os.path.join(dirname, fname), "w") as f:
                for blk in blocks:
                    for r in blk:
                        f.write(eigen_row(r) + "\n")

        st, ct, gr, co = [], [], [], []
        for i in range(nwb):
            q, g = parts[i], grads[i]
            st.append(rows(q["x"][problem], Ns[i], 14))
            ct.append(rows(q["u"][problem], Ns[i], 4))
            gr.append(rows(q["Vx"][problem], Ns[i], 14))
            co.append(rows(g["lx"][problem], Ns[i] - 1, 14) + [g["Phix"][problem]])
        for i in range(nfb):
            q, g = parts[nwb + i], grads[nwb + i]
            st.append(rows(q["x"][problem], Ns[nwb + i], 6))
            ct.append(rows(q["u"][problem], n_rows(i), 4))
            gr.append(rows(q["Vx"][problem], n_rows(i), 6))
            co.append(rows(g["lx"][problem], n_rows(i) - 1, 6) + [g["Phix"][problem]])
        write("state.txt", st)
        write("control.txt", ct)
        write("gradient.txt", gr)
        write("cost.txt", co)

"""ctypes mirror of include/mhpc_capi.h and the loader of the native library.

The product library is `mhpc_minimal_env_amd/libmhpc_amd.so` (HIP kernels for gfx950 +
the C-ABI host runtime), built in-tree by `__graft_entry__.build()`.  There is no
fallback: if the library is missing, `lib()` raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MHPC_AMD_LIB: alternate build of the same library (tuning experiments)
LIB_PATH = os.environ.get("MHPC_AMD_LIB") or os.path.join(HERE, "libmhpc_amd.so")

MHPC_MAX_PHASES = 16
MHPC_MAX_KNOTS = 1024
MHPC_MAX_LAYOUTS = 32
MHPC_TRACE_LEN = 64
MHPC_NUM_KERNELS = 7
MHPC_MAX_ROLLOUT_EPS = 4096

MHPC_OK = 0
MHPC_ERR_INVALID = 1

# mhpc_set_kernel_variant (include/mhpc_capi.h)
MHPC_VARIANT_BWS = 0
MHPC_VARIANT_RO = 1
BWS_VARIANTS = {"auto": 0, "rows4": 1, "rows2": 2, "rows1": 3, "pairs2": 4}
RO_VARIANTS = {"auto": 0, "pair": 1, "pipe_staged": 2, "pipe": 3, "fused_staged": 4, "fused": 5}
MHPC_VARIANT_OVERLAP = 2
OVERLAP_VARIANTS = {"auto": 0, "on": 1, "off": 2}
MHPC_VARIANT_SUBBATCH = 3
MHPC_MAX_SUBBATCH = 4
MHPC_VARIANT_RO_STORE = 4  # line-search trials storing their records (0 = default)
MHPC_VARIANT_SWEEP_BITS = 5  # backward-sweep arithmetic: 64 double (default) / 32 float (fp32)
MHPC_SOLVE_OK = 0
MHPC_SOLVE_REG_ABORT = 1
MHPC_SOLVE_NONFINITE = 2


class GaitC(ctypes.Structure):
    """mhpc_gait: mode cycle + per-mode durations (the reference's Gait)."""
    _fields_ = [
        ("n_modes", ctypes.c_int32),
        ("modes", ctypes.c_int32 * MHPC_MAX_PHASES),
        ("timings", ctypes.c_float * MHPC_MAX_PHASES),
    ]


class ProblemDesc(ctypes.Structure):
    _fields_ = [
        ("n_wb", ctypes.c_int32),
        ("n_fb", ctypes.c_int32),
        ("mode_seq", ctypes.c_int32 * MHPC_MAX_PHASES),
        ("N", ctypes.c_int32 * MHPC_MAX_PHASES),
        ("dt_wb", ctypes.c_double),
        ("dt_fb", ctypes.c_double),
        ("vel_cmd", ctypes.c_double),
        ("height_cmd", ctypes.c_double),
        ("precision", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]

    @property
    def n_phases(self) -> int:
        return self.n_wb + self.n_fb

    def xsize(self, p: int) -> int:
        return 14 if p < self.n_wb else 6

    def knots(self, p: int) -> int:
        return self.N[p]

    def lens(self):
        """Per-problem phase-concatenated lengths of (x, u, K) arrays."""
        lx = sum(self.N[p] * self.xsize(p) for p in range(self.n_phases))
        lu = sum(self.N[p] * 4 for p in range(self.n_phases))
        lk = sum(self.N[p] * 4 * self.xsize(p) for p in range(self.n_phases))
        return lx, lu, lk

    def describe(self) -> dict:
        return {
            "n_wb": self.n_wb, "n_fb": self.n_fb,
            "mode_seq": [self.mode_seq[p] for p in range(self.n_phases)],
            "N": [self.N[p] for p in range(self.n_phases)],
            "dt_wb": self.dt_wb, "dt_fb": self.dt_fb,
            "vel_cmd": self.vel_cmd, "height_cmd": self.height_cmd,
        }


class HsddpOption(ctypes.Structure):
    _fields_ = [
        ("alpha", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("update_penalty", ctypes.c_double),
        ("update_relax", ctypes.c_double),
        ("update_regularization", ctypes.c_double),
        ("update_ReB", ctypes.c_double),
        ("max_DDP_iter", ctypes.c_double),
        ("max_AL_iter", ctypes.c_double),
        ("DDP_thresh", ctypes.c_double),
        ("AL_thresh", ctypes.c_double),
        ("AL_active", ctypes.c_int32),
        ("ReB_active", ctypes.c_int32),
        ("smooth_active", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


def _mat(r, c):
    return (ctypes.c_double * c) * r


class CostWeights(ctypes.Structure):
    """mhpc_cost_weights: diagonal weights per mode (CostBase.h:9-46, MHPCCost.cpp:24-75)."""
    _fields_ = [
        ("wb_Q", _mat(4, 14)), ("wb_R", _mat(4, 4)), ("wb_S", _mat(4, 4)), ("wb_Qf", _mat(4, 14)),
        ("fb_Q", _mat(4, 6)), ("fb_R", _mat(4, 4)), ("fb_Qf", _mat(4, 6)),
    ]

    def as_dict(self) -> dict:
        import numpy as np
        return {k: np.ctypeslib.as_array(getattr(self, k)).copy() for k, _ in self._fields_}

    @classmethod
    def from_dict(cls, d: dict) -> "CostWeights":
        import numpy as np
        w = cls()
        for k, _ in cls._fields_:
            np.ctypeslib.as_array(getattr(w, k))[...] = np.asarray(d[k], dtype=np.float64)
        return w


class ConstraintParams(ctypes.Structure):
    """mhpc_constraint_params (ConstraintsBase.h:11-50, MHPCConstraints.cpp:14-88)."""
    _fields_ = [
        ("torque_limit", ctypes.c_double), ("friction_coeff", ctypes.c_double),
        ("sigma", ctypes.c_double * 4), ("delta", ctypes.c_double * 4),
        ("delta_min", ctypes.c_double * 4), ("eps_torque", ctypes.c_double * 4),
        ("eps_grf", ctypes.c_double * 4),
    ]

    def as_dict(self) -> dict:
        import numpy as np
        return {k: (float(getattr(self, k)) if t is ctypes.c_double
                    else np.ctypeslib.as_array(getattr(self, k)).copy()) for k, t in self._fields_}

    @classmethod
    def from_dict(cls, d: dict) -> "ConstraintParams":
        import numpy as np
        c = cls()
        for k, t in cls._fields_:
            if t is ctypes.c_double:
                setattr(c, k, float(d[k]))
            else:
                np.ctypeslib.as_array(getattr(c, k))[...] = np.asarray(d[k], dtype=np.float64)
        return c


class Counters(ctypes.Structure):
    _fields_ = [
        ("ddp_iters", ctypes.c_int64),
        ("bws_sweeps", ctypes.c_int64),
        ("bws_knots", ctypes.c_int64),
        ("ls_rollouts", ctypes.c_int64),
        ("fwd_sweeps", ctypes.c_int64),
        ("partial_sweeps", ctypes.c_int64),
        ("solve_ms", ctypes.c_double),
    ]


_DP = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int32)

# (name, restype, argtypes) -- every entry point declared in include/mhpc_capi.h
SIGNATURES = [
    ("mhpc_version", ctypes.c_char_p, []),
    ("mhpc_last_error", ctypes.c_char_p, []),
    ("mhpc_phase_dims", ctypes.c_int, [ctypes.POINTER(ProblemDesc), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("mhpc_create", ctypes.c_int, [ctypes.POINTER(ProblemDesc), ctypes.POINTER(HsddpOption),
                                   ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("mhpc_set_x0", ctypes.c_int, [ctypes.c_void_p, _DP]),
    ("mhpc_initialize", ctypes.c_int, [ctypes.c_void_p]),
    ("mhpc_solve", ctypes.c_int, [ctypes.c_void_p, _IP]),
    ("mhpc_get_phase", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _DP, _DP, _DP, _DP, _DP, _DP]),
    ("mhpc_get_phase_problems", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, _DP, _DP, _DP, _DP, _DP, _DP]),
    ("mhpc_get_scalars", ctypes.c_int, [ctypes.c_void_p, _DP, _DP, _DP, _DP, _DP, _IP]),
    ("mhpc_get_counters", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Counters)]),
    ("mhpc_get_cost_gradients", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _DP, _DP]),
    ("mhpc_get_cost_gradients_problems", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                        ctypes.c_int, _DP, _DP]),
    ("mhpc_update_problem", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GaitC)]),
    ("mhpc_update_problems", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(GaitC),
                                            _IP, _IP]),
    ("mhpc_get_desc", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ProblemDesc)]),
    ("mhpc_set_layouts", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ProblemDesc),
                                        _IP]),
    ("mhpc_get_problem_desc", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                             ctypes.POINTER(ProblemDesc)]),
    ("mhpc_num_layouts", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    ("mhpc_max_phases", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    ("mhpc_rollout_costs", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _DP, _DP, _DP,
                                          ctypes.POINTER(ctypes.c_float)]),
    ("mhpc_destroy", None, [ctypes.c_void_p]),
    ("mhpc_kernel_name", ctypes.c_char_p, [ctypes.c_int]),
    ("mhpc_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("mhpc_get_kernel_stats", ctypes.c_int, [ctypes.c_void_p, _DP,
                                             ctypes.POINTER(ctypes.c_int64), _DP]),
    ("mhpc_reset_kernel_stats", ctypes.c_int, [ctypes.c_void_p]),
    ("mhpc_get_kernel_flops", ctypes.c_int, [ctypes.c_void_p, _DP]),
    ("mhpc_set_kernel_variant", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("mhpc_default_cost_weights", ctypes.c_int, [ctypes.POINTER(CostWeights)]),
    ("mhpc_default_constraint_params", ctypes.c_int, [ctypes.POINTER(ConstraintParams)]),
    ("mhpc_set_cost_weights", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CostWeights)]),
    ("mhpc_get_cost_weights", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CostWeights)]),
    ("mhpc_set_constraint_params", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ConstraintParams)]),
    ("mhpc_get_constraint_params", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ConstraintParams)]),
    ("mhpc_eval_wb_dynamics", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _DP, _DP,
                                             _DP, _DP]),
    ("mhpc_eval_wb_dynamics_pair", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _DP,
                                                  _DP, _DP, _DP]),
    ("mhpc_eval_wb_touchdown", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _DP, _DP,
                                              _DP, _DP, _DP, _DP]),
    ("mhpc_eval_wb_dynamics_f32", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, _DP, _DP, _DP, _DP]),
    ("mhpc_eval_wb_partials", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _DP, _DP,
                                             _DP, _DP, _DP, _DP]),
    ("mhpc_eval_wb_impact", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _DP, _DP, _DP]),
    ("mhpc_eval_srb", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _DP, _DP, _DP, _DP, _DP, _DP, _DP]),
]

_lib = None


def lib():
    """Load libmhpc_amd.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP extension with "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != MHPC_OK:
        msg = lib().mhpc_last_error()
        raise RuntimeError(f"{what} failed with status {rc}: {msg.decode() if msg else ''}")


def dptr(a):
    return None if a is None else a.ctypes.data_as(_DP)


def iptr(a):
    return None if a is None else a.ctypes.data_as(_IP)


def default_cost_weights() -> CostWeights:
    w = CostWeights()
    check(lib().mhpc_default_cost_weights(ctypes.byref(w)), "mhpc_default_cost_weights")
    return w


def default_constraint_params() -> ConstraintParams:
    c = ConstraintParams()
    check(lib().mhpc_default_constraint_params(ctypes.byref(c)), "mhpc_default_constraint_params")
    return c

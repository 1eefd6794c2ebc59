"""TEST INFRASTRUCTURE ONLY -- ctypes access to the reference's own CasADi kernels.

`oracle/_ref/libmhpc_casadi_ref.so` is compiled (oracle/Makefile `ref`) straight from
/root/reference/CasadiGen/source/*.c.  This module calls those kernels exactly the way
the reference's adapter does (`casadi_interface`, CasadiGen/source/CasadiGen.cpp:4-79):
evaluate, then scatter each CSC-sparse output into a zero-initialised dense column-major
buffer.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(HERE, "_ref", "libmhpc_casadi_ref.so")

# name -> number of inputs (all outputs are discovered from *_n_out / *_sparsity_out)
FUNCS = {
    "Dyn_FL": 2, "Dyn_BS": 2, "Dyn_FS": 2,
    "Dyn_FL_par": 2, "Dyn_BS_par": 2, "Dyn_FS_par": 2,
    "Imp_F": 1, "Imp_B": 1, "Imp_F_par": 1, "Imp_B_par": 1,
    "FBDynamics": 4, "FBDynamics_par": 4,
    "WB_FL1_terminal_constr": 1, "WB_FL2_terminal_constr": 1,
    "Jacob_F": 1, "Jacob_B": 1,
}

_lib = None


def available() -> bool:
    return os.path.exists(REF_SO)


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{REF_SO} not built (make -C oracle ref)")
        _lib = ctypes.CDLL(REF_SO)
    return _lib


def _sparsity(name, i):
    f = getattr(lib(), name + "_sparsity_out")
    f.restype = ctypes.POINTER(ctypes.c_longlong)
    sp = f(ctypes.c_longlong(i))
    nrow, ncol = sp[0], sp[1]
    colptr = [sp[2 + c] for c in range(ncol + 1)]
    nnz = colptr[-1]
    rows = [sp[2 + ncol + 1 + k] for k in range(nnz)]
    return nrow, ncol, colptr, rows


def call(name: str, *args):
    """Evaluate CasADi function `name`; returns dense outputs as numpy arrays of shape
    (nrow, ncol) (column vectors squeezed to 1-D)."""
    L = lib()
    nout_f = getattr(L, name + "_n_out")
    nout_f.restype = ctypes.c_longlong
    nout = nout_f()
    ins = [np.ascontiguousarray(a, dtype=np.float64) for a in args]
    arg_arr = (ctypes.POINTER(ctypes.c_double) * max(len(ins), 1))()
    for i, a in enumerate(ins):
        arg_arr[i] = a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    sps = [_sparsity(name, i) for i in range(nout)]
    bufs = [np.zeros(max(len(sp[3]), 1)) for sp in sps]
    res_arr = (ctypes.POINTER(ctypes.c_double) * nout)()
    for i, b in enumerate(bufs):
        res_arr[i] = b.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    fn = getattr(L, name)
    fn.restype = ctypes.c_int
    rc = fn(arg_arr, res_arr, None, None, ctypes.c_int(0))
    if rc != 0:
        raise RuntimeError(f"{name} returned {rc}")
    outs = []
    for (nrow, ncol, colptr, rows), b in zip(sps, bufs):
        dense = np.zeros((nrow, ncol))
        for c in range(ncol):
            for k in range(colptr[c], colptr[c + 1]):
                dense[rows[k], c] = b[k]
        outs.append(dense[:, 0] if ncol == 1 else dense)
    return outs

"""ORACLE (test infrastructure and bench.py's second CPU line only) — Python binding of the
C++/OpenMP restatement in oracle/cpu_forward.cpp.  Nothing under ignnition_amd/ imports it.

    python -m oracle.cpu_oracle        # build oracle/_build/libign_oracle.so (g++ -O3 -fopenmp)

``cpu_forward(plan, graphs, params, threads, float64)`` runs the float32 (or float64) restatement of ComnetModel.call
(GM:384-658) on the host for the lowered plan (ignnition_amd.engine.MPPlan) and a list of feature
dicts or a BatchedGraphs, with the parameters by their Keras-style names."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "cpu_forward.cpp")
LIB = os.path.join(HERE, "_build", "libign_oracle.so")


def build(force: bool = False) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    # -ffast-math: vectorised expf / tanhf (libmvec) in the gates; a float32 restatement checked
    # against the float64 dense oracle at the parity tolerance (tests/test_cpu_oracle.py)
    cmd = ["g++", "-O3", "-march=x86-64-v3", "-ffast-math", "-fopenmp", "-std=c++17", "-shared", "-fPIC",
           "-I", os.path.join(REPO, "include"), SRC, "-o", LIB]
    subprocess.check_call(cmd)
    return LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError("oracle/_build/libign_oracle.so not built: python -m oracle.cpu_oracle")
        lib = C.CDLL(LIB)
        lib.ign_oracle_forward.restype = C.c_int
        lib.ign_oracle_forward.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.c_void_p,
                                           C.c_int32, C.c_int32]
        lib.ign_oracle_last_error.restype = C.c_char_p
        _lib = lib
    return _lib


class OracleError(RuntimeError):
    pass


def cpu_forward(plan, graphs, params: dict, threads: int = 0, float64: bool = False) -> np.ndarray:
    """float64=False: float32 arithmetic (TF's on the CPU; bench.py's line); True: float64 (the
    checker: float32 runs of this model differ from float64 by up to ~2e-4 on outliers)."""
    from ignnition_amd.engine import batch_desc
    lib = _load()
    pd, pkeep = plan.to_desc()
    bd, bkeep, (G, E, num, cnt, _) = batch_desc(plan, graphs)
    specs = plan.param_specs()
    arrs = [np.ascontiguousarray(np.asarray(params[name], np.float32).reshape(-1)) for name, _ in specs]
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    e = plan.readout_inputs[0]
    units = plan.dense[-1][1]
    out = np.empty(int(num[:, e].sum()) * units, np.float32)
    rc = lib.ign_oracle_forward(C.byref(pd), C.byref(bd), ptrs, len(arrs), out.ctypes.data, int(threads),
                                int(bool(float64)))
    if rc:
        raise OracleError("%d: %s" % (rc, lib.ign_oracle_last_error().decode()))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))

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
# the same source without -ffast-math: every float32 operation IEEE round-to-nearest (FMA
# contraction allowed, as in TF's Eigen kernels on an AVX2/FMA host), libm expf / tanhf, no
# reassociation -- the plain-float32 yardstick of the full-batch precision test
LIB_IEEE = os.path.join(HERE, "_build", "libign_oracle_ieee.so")

_FLAGS = {
    # -ffast-math: vectorised expf / tanhf (libmvec) in the gates; the timed CPU line, checked
    # against the float64 dense oracle at the parity tolerance (tests/test_cpu_oracle.py)
    LIB: ["-O3", "-march=x86-64-v3", "-ffast-math"],
    LIB_IEEE: ["-O3", "-march=x86-64-v3", "-fno-fast-math", "-fno-unsafe-math-optimizations"],
}


def build(force: bool = False) -> str:
    for lib, flags in _FLAGS.items():
        if not force and os.path.exists(lib) and os.path.getmtime(lib) >= os.path.getmtime(SRC):
            continue
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        cmd = ["g++", *flags, "-fopenmp", "-std=c++17", "-shared", "-fPIC",
               "-I", os.path.join(REPO, "include"), SRC, "-o", lib]
        subprocess.check_call(cmd)
    return LIB


_libs = {}


def _load(ieee: bool = False):
    path = LIB_IEEE if ieee else LIB
    if path not in _libs:
        if not os.path.exists(path):
            raise ImportError("%s not built: python -m oracle.cpu_oracle" % os.path.relpath(path, REPO))
        lib = C.CDLL(path)
        lib.ign_oracle_forward.restype = C.c_int
        lib.ign_oracle_forward.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.c_void_p,
                                           C.c_int32, C.c_int32]
        lib.ign_oracle_last_error.restype = C.c_char_p
        _libs[path] = lib
    return _libs[path]


class OracleError(RuntimeError):
    pass


def cpu_forward(plan, graphs, params: dict, threads: int = 0, float64: bool = False,
                ieee: bool = False) -> np.ndarray:
    """float64=False: float32 arithmetic (TF's on the CPU; bench.py's line); True: float64 (the
    checker: float32 runs of this model differ from float64 by up to ~2e-4 on outliers).
    ieee=True: the float32 arithmetic of the build without -ffast-math (libm expf / tanhf, no
    reassociation), the yardstick the engine's full-batch error is held to."""
    from ignnition_amd.engine import batch_desc
    lib = _load(ieee and not float64)
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

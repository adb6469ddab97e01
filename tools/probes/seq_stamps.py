"""Where the inference ordered update's waves spend their cycles (GPU box, diagnostic library):

    tools/build_ab.sh stamp -DIGN_SEQ_STAMP        # here (hipcc cross-compiles)
    IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_stamp.so python tools/probes/seq_stamps.py

Runs the 512 x synth50 RouteNet batch on one stream and reads the per-wave s_memtime sums of the last
seq_gru_h16 launch: tile prologue (header -> first step, incl. the state / first-row loads), the
split + h.U MFMA part of the steps, the gates (incl. the wait for the projected row), the epilogue
store.  The stamps serialise the schedule: read the shares, not the absolute time."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ignnition_amd import _lib, workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402


def main():
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", os.environ.get("TOPO", "synth50"),
                                                            int(os.environ.get("GRAPHS", "512")))
    plan = MPPlan.from_model_info(mi)
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(seed=0, bias_scale=0.05))
    b = Batch(eng, graphs)
    for _ in range(3):
        b.forward(to_host=False)
    eng.synchronize()
    fn = _lib.lib.ign_debug_seq_stamps
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(4096 * 8, np.uint64)
    rc = fn(buf.ctypes.data_as(C.c_void_p), buf.size)
    v = buf.reshape(4096, 8)
    v = v[v[:, 7] == 1].astype(np.float64)
    tot = v[:, 6]
    names = ["prologue", "mfma", "gates", "epilogue"]
    out = {"rc": rc, "waves": int(len(v)), "tiles": float(v[:, 4].sum()), "steps": float(v[:, 5].sum()),
           "wave_cycles_mean": float(tot.mean()), "wave_cycles_max": float(tot.max()),
           "wave_cycles_min": float(tot.min()),
           "share": {n: float(v[:, i].sum() / tot.sum()) for i, n in enumerate(names)},
           "cycles_per_tile": {n: float(v[:, i].sum() / v[:, 4].sum()) for i, n in enumerate(names)},
           "cycles_per_step": {n: float(v[:, i].sum() / v[:, 5].sum()) for i, n in enumerate(names[1:3], 1)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

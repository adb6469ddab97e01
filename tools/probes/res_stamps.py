"""Where the graph-resident forward's waves spend their cycles (GPU box, diagnostic library):

    tools/build_ab.sh rstamp -DIGN_RES_STAMP        # here
    IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so python tools/probes/res_stamps.py

Runs TOPO x GRAPHS (default GEANT2 x256: one workgroup per CU) on one stream and reads per-wave
s_memtime sums: init (features, iteration-0 projection), phase A work (ordered update tiles) and its
barrier wait, phase B work (sum update) and its barrier wait, over all T iterations; within phase B,
the cycles up to the end of B1 (message sums) and of B2 (GRU step), barrier waits included."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ignnition_amd import _lib, workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402


def main():
    n = int(os.environ.get("GRAPHS", "256"))
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs(os.environ.get("MODEL", "routenet"),
                                                            os.environ.get("TOPO", "geant2"), n)
    plan = MPPlan.from_model_info(mi)
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(seed=0, bias_scale=0.05))
    b = Batch(eng, graphs)
    for _ in range(3):
        b.forward(to_host=False)
    eng.synchronize()
    fn = _lib.lib.ign_debug_res_stamps
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int]
    W = int(os.environ.get("RES_WAVES", "16"))
    buf = np.zeros(256 * W * 8, np.uint64)
    rc = fn(buf.ctypes.data_as(C.c_void_p), buf.size)
    v = buf.reshape(256, W, 8)[:min(n, 256)].astype(np.float64)
    tot = v[:, :, 7]
    names = ["init", "A_work", "A_wait", "B_work", "B_wait"]
    out = {"rc": rc, "graphs": int(v.shape[0]), "cycles_per_graph_mean": float(tot.max(axis=1).mean()),
           "us_per_graph_at_100MHz": float(tot.max(axis=1).mean() / 100.0),
           "share_all_waves": {k: float(v[:, :, i].sum() / tot.sum()) for i, k in enumerate(names)},
           "per_wave_mean_cycles": {k: float(v[:, :, i].mean()) for i, k in enumerate(names)},
           "B1_cycles_per_wave_mean": float(v[:, :, 5].mean()),
           "B1_B2_cycles_per_wave_mean": float(v[:, :, 6].mean()),
           "A_work_per_wave": [float(x) for x in v[:, :, 1].mean(axis=0)],
           # phase A's wall cycles (work + barrier wait, the same span for every wave) per tile-step of
           # one SIMD (the graph's tile-steps over its 4 SIMDs), against tools/isa_mix.py's issue floor
           "phase_A_cycles_per_tile_step_per_simd": float((v[:, :, 1] + v[:, :, 2]).mean()) /
                                                     (b.resident_info()["tile_steps"] / n / 4.0),
           "B_work_per_wave": [float(x) for x in v[:, :, 3].mean(axis=0)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

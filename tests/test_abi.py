"""C-ABI boundary (CPU): libignmp.so loads, exports every symbol of include/ignmp.h,
validates plans and computes the parameter layout without a GPU (no compute calls)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from ignnition_amd import _lib, model_examples, workloads
from ignnition_amd.engine import MPPlan

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "ignmp.h")).read()
    return sorted(set(re.findall(r"\b(ign_[a-z0-9_]+)\s*\(", src)))


def test_every_header_symbol_exported():
    names = header_functions()
    assert len(names) >= 19
    assert sorted(_lib.SYMBOLS) == names
    for n in names:
        assert hasattr(_lib.lib, n), n


def test_abi_version_and_error_string():
    assert _lib.lib.ign_abi_version() == _lib.ABI_VERSION == 13
    rc = _lib.lib.ign_plan_create(None, 0, None)
    assert rc == -1
    assert b"null" in _lib.lib.ign_last_error()


def _plan(kind, **kw):
    desc, dims, mi = workloads.model(kind)
    return MPPlan.from_model_info(mi)


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_plan_layout_via_abi(kind):
    plan = _plan(kind)
    desc, keep = plan.to_desc()
    h = C.c_void_p()
    _lib.check(_lib.lib.ign_plan_create(C.byref(desc), 0, C.byref(h)))
    try:
        n = C.c_int32()
        _lib.check(_lib.lib.ign_plan_num_param_tensors(h, C.byref(n)))
        specs = plan.param_specs()
        assert n.value == len(specs)
        last = -1
        for i, (name, shape) in enumerate(specs):
            k, o, off, r, c = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32(), C.c_int32()
            _lib.check(_lib.lib.ign_plan_param_tensor(h, i, C.byref(k), C.byref(o), C.byref(off), C.byref(r), C.byref(c)))
            assert r.value * c.value == int(np.prod(shape)), name
            assert off.value % 64 == 0 and off.value > last
            last = off.value
        total = C.c_int64()
        _lib.check(_lib.lib.ign_plan_num_params(h, C.byref(total)))
        assert total.value >= last + 1
    finally:
        _lib.lib.ign_plan_destroy(h)


def test_plan_validation_errors():
    plan = _plan("routenet")
    plan.hidden[0] = 33   # GRU input 33 is not instantiated
    plan.cells = [(d, 33 if din == 32 and d == "path" else din, h) for d, din, h in plan.cells]
    desc, keep = plan.to_desc()
    h = C.c_void_p()
    rc = _lib.lib.ign_plan_create(C.byref(desc), 0, C.byref(h))
    assert rc in (-1, -2)
    assert _lib.lib.ign_last_error()


def test_feature_size_exceeds_hidden():
    plan = _plan("routenet")
    plan.features[0] = [("link_capacity", 40)]
    desc, keep = plan.to_desc()
    h = C.c_void_p()
    assert _lib.lib.ign_plan_create(C.byref(desc), 0, C.byref(h)) == -1
    assert b"exceeds" in _lib.lib.ign_last_error()


def test_compute_without_gpu_fails_loudly():
    from ignnition_amd.engine import device_count, Engine
    if device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(_lib.EngineError) as ei:
        Engine(_plan("routenet")).set_params(_plan("routenet").init_params(0))
    assert ei.value.code == -3


def test_batch_desc_index_width():
    """ABI 13: batch_desc passes int32 index arrays through (index_bytes 4, no widening copy) when
    every one of them is int32, and widens all of them to int64 (index_bytes 8) otherwise."""
    import numpy as np
    from ignnition_amd import workloads
    from ignnition_amd.engine import BatchedGraphs, MPPlan, batch_desc
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("qsize", "nsfnet", 2)
    plan = MPPlan.from_model_info(mi)
    bg = BatchedGraphs.from_dicts(graphs)
    ints = [k for k, (v, _) in bg.arrays.items() if v.dtype == np.int64]
    narrow = BatchedGraphs({k: (v.astype(np.int32) if k in ints else v, l) for k, (v, l) in bg.arrays.items()}, 2)
    d8, keep8, _ = batch_desc(plan, bg)
    d4, keep4, _ = batch_desc(plan, narrow)
    assert d8.index_bytes == 8 and d4.index_bytes == 4
    srcs4 = keep4[3]
    assert srcs4 and all(a.dtype == np.int32 for a in srcs4)
    assert all(np.shares_memory(a, narrow.get(k)[0]) for a, k in zip(srcs4, [s.keys[0] for s in plan.adj_slots]))
    mixed = dict(narrow.arrays)
    k0 = plan.adj_slots[0].keys[0]
    mixed[k0] = (bg.get(k0)[0], bg.get(k0)[1])   # one int64 array among int32 ones
    dm, keepm, _ = batch_desc(plan, BatchedGraphs(mixed, 2))
    assert dm.index_bytes == 8
    assert all(a.dtype == np.int64 for arrs in (keepm[3], keepm[4], keepm[5], keepm[7]) for a in arrs)
    for a4, a8 in zip(keep4[3] + keep4[4] + keep4[5] + keep4[7], keep8[3] + keep8[4] + keep8[5] + keep8[7]):
        np.testing.assert_array_equal(a4, a8)

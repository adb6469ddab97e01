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

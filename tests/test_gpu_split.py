"""SplitBatch (engine.py): a batch as sub-batches on several plans / HIP streams, launched before
any wait (bench.py's default step, DESIGN §3b'').  Graphs are independent (GM:712-724), so the
predictions must be bitwise those of one Batch over the same graphs, in graph order; the replicas
must follow every parameter update of the engine (set_params, adam_step)."""
import numpy as np
import pytest

from ignnition_amd import workloads
from ignnition_amd.engine import Batch, Engine, MPPlan, SplitBatch, device_count

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")


def _engine(kind, topo, n, seed=0):
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, topo, n)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(seed, bias_scale=0.05)
    eng = Engine(plan, 0)
    eng.set_params(prm)
    return eng, plan, graphs, labels


@pytest.mark.parametrize("kind,topo,n,parts", [("routenet", "synth50", 12, 2), ("routenet", "nsfnet", 5, 3),
                                               ("qsize", "synth50", 6, 2), ("routenet", "geant2", 3, 4)])
def test_split_batch_equals_one_batch(kind, topo, n, parts):
    eng, _, graphs, _ = _engine(kind, topo, n)
    whole = Batch(eng, graphs).forward()
    sb = SplitBatch(eng, graphs, parts)
    assert len(sb.parts) == min(parts, n)
    assert sb.num_graphs == n and sb.predictions == whole.shape[0]
    got = sb.forward()
    assert np.array_equal(got, whole)
    # async launches, then the host read: same bits again (the graph replay path)
    sb.forward(to_host=False)
    assert np.array_equal(sb.forward(), whole)
    assert sb.edges_per_forward == Batch(eng, graphs).edges_per_forward
    # timed forwards launch directly (no graph replay): same bits
    eng.set_timing(True)
    assert np.array_equal(sb.forward(), whole)
    eng.set_timing(False)


def test_split_batch_replicas_follow_parameter_updates():
    import torch
    eng, plan, graphs, _ = _engine("routenet", "nsfnet", 4)
    sb = SplitBatch(eng, graphs, 2)
    before = sb.forward()
    eng.set_params(plan.init_params(7, bias_scale=0.2))
    after = sb.forward()
    assert not np.array_equal(before, after)
    assert np.array_equal(after, Batch(eng, graphs).forward())
    # an optimizer step on the engine's device parameters reaches the replica too
    g = torch.full((eng.n_params,), 0.01, dtype=torch.float32, device="cuda")
    m, v = torch.zeros_like(g), torch.zeros_like(g)
    torch.cuda.synchronize()
    eng.adam_step(g, m, v, 0, 1e-2)
    stepped = sb.forward()
    assert not np.array_equal(stepped, after)
    assert np.array_equal(stepped, Batch(eng, graphs).forward())


def test_bench_line_with_sub_batch_streams():
    """bench.py's default step (two sub-batch streams) on a small batch: one JSON line whose
    roofline carries the timed region's figure and the isolated one; --streams 1 has no isolated leg."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = {}
    for streams in (2, 1):
        r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--graphs", "16", "--steps", "2",
                            "--warmup", "1", "--no-cpu", "--streams", str(streams)],
                           capture_output=True, text=True, timeout=300, cwd=repo)
        assert r.returncode == 0, r.stderr[-2000:]
        out = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(out) == 1
        lines[streams] = out[0]
    two, one = lines[2], lines[1]
    assert two["config"]["streams"] == 2 and one["config"]["streams"] == 1
    assert two["config"]["edges_per_step_per_gpu"] == one["config"]["edges_per_step_per_gpu"]
    assert two["value"] > 0 and one["value"] > 0
    iso = two["roofline"]["isolated"]
    assert iso["launches"] > 0 and 0 < iso["frac"] and "note" in two["roofline"]
    assert "isolated" not in one["roofline"]

"""north_star: "the RouteNet and Q-size examples run unchanged".  The examples' main.py
(RNM:20-48; code/main.py:55-59: create_model -> debug -> train_and_evaluate, then predict) is run
as a program, `python examples/<name>/main.py`, from a directory holding train_options.ini,
model_description.json and tar.gz datasets in the reference layout (examples/make_example.py;
synthetic data, the real datasets are not downloadable).  Nothing is patched: the program reads
./train_options.ini at import (FO:34-36) and finds its normalisation functions in __main__."""
import glob
import os
import re
import subprocess
import sys

import pytest

from examples.make_example import make

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind,script", [("routenet", "Routenet"), ("qsize", "Q-size")])
def test_example_main_runs_unchanged(tmp_path, kind, script):
    d = make(kind, str(tmp_path / kind), "nsfnet", 4)
    ini = os.path.join(d, "train_options.ini")
    text = open(ini).read()
    text = re.sub(r"train_steps: \d+", "train_steps: 20", text)
    text = re.sub(r"batch_size: \d+", "batch_size: 2", text)
    text = re.sub(r"eval_samples: \d+", "eval_samples: 4", text)
    open(ini, "w").write(text)
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "examples", script, "main.py")], cwd=d, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    ckpts = glob.glob(os.path.join(d, "CheckPoints", "experiment_*", "ckpt-*.safetensors"))
    assert ckpts, os.listdir(d)
    assert glob.glob(os.path.join(d, "CheckPoints", "experiment_*", "metrics.jsonl"))
    assert os.path.exists(os.path.join(os.path.dirname(d), "debug_model", "plan.json"))
    assert "eval at step 20" in r.stderr
    # predict (FO:169-236) prints one array of per-path predictions per sample of the predict set
    arrays = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("[")]
    assert len(arrays) >= 4, r.stdout[-2000:]
    nums = [float(x) for x in re.findall(r"-?\d+\.\d*(?:e[-+]?\d+)?", " ".join(arrays))]
    assert nums and all(abs(v) < 1e6 for v in nums)

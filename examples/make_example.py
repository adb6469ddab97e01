"""Write a runnable example directory: model_description.json, train_options.ini and synthetic
tar.gz datasets in the reference layout (the real datasets are not downloadable here).

    python examples/make_example.py routenet /tmp/rn_example [topology] [n_graphs]
    cd /tmp/rn_example && python <repo>/examples/Routenet/main.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from ignnition_amd import model_examples, synthetic  # noqa: E402

INI = """[PATHS]
train_dataset: {d}/data/train
eval_dataset: {d}/data/eval
predict_dataset: {d}/data/predict
json_path: {d}/model_description.json
model_dir: {d}/CheckPoints
debug_dir: {d}

[TRAINING_OPTIONS]
batch_size: 8
train_steps: 1000
shuffle_train_samples: True
shuffle_eval_samples: False
eval_samples: 10
save_checkpoints_secs: 300
keep_checkpoint_max: 20
throttle_secs: 300
execute_gpu: True
"""


def make(kind: str, out: str, topology: str = "nsfnet", n_graphs: int = 4) -> str:
    out = os.path.abspath(out)
    os.makedirs(out, exist_ok=True)
    desc = model_examples.routenet() if kind == "routenet" else model_examples.qsize()
    model_examples.write(desc, os.path.join(out, "model_description.json"))
    q = kind == "qsize"
    for split, first in (("train", 0), ("eval", 1000), ("predict", 2000)):
        synthetic.write_tar_dataset(synthetic.dataset(topology, n_graphs, qsize=q, first_id=first),
                                    os.path.join(out, "data", split))
    with open(os.path.join(out, "train_options.ini"), "w") as fh:
        fh.write(INI.format(d=out))
    return out


if __name__ == "__main__":
    kind = sys.argv[1] if len(sys.argv) > 1 else "routenet"
    out = sys.argv[2] if len(sys.argv) > 2 else "./example_" + kind
    topo = sys.argv[3] if len(sys.argv) > 3 else "nsfnet"
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    print(make(kind, out, topo, n))

"""Parameter checkpoints (safetensors, Keras-style tensor names).

Replaces the reference's Estimator checkpoints / Saver restore (FO:126-129, 141-145,
218-221), which need TensorFlow.  Tensor names follow the engine layout
(``path_update/kernel``, ``readout_model_0/1st_dense_layer/kernel`` ...).
"""

from __future__ import annotations

import numpy as np


def save_params(params: dict, path: str, metadata: dict | None = None):
    from safetensors.numpy import save_file
    save_file({k: np.ascontiguousarray(v, np.float32) for k, v in params.items()}, path,
              metadata={k: str(v) for k, v in (metadata or {}).items()})


def load_params(path: str) -> dict:
    from safetensors.numpy import load_file
    return dict(load_file(path))

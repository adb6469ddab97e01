"""Q-size example entry point — the reference's examples/Q-size/main.py workflow (QSM:20-48)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import ignnition_amd.framework_operations as ignnition  # noqa: E402


def normalization_queue_size(feature, feature_name):
    if feature_name == 'delay':
        feature = (np.log(feature) + 1.78) / 0.93
    if feature_name == 'traffic':
        feature = (feature - 0.28) / 0.15
    if feature_name == 'jitter':
        feature = (feature - 1.5) / 1.5
    if feature_name == 'link_capacity':
        feature = (feature - 27.0) / 14.86
    if feature_name == 'queue_sizes':
        feature = (feature - 16.5) / 15.5
    return feature


def main():
    model = ignnition.create_model()
    ignnition.debug(model)
    ignnition.train_and_evaluate(model)
    return ignnition.predict(model)


if __name__ == "__main__":
    main()

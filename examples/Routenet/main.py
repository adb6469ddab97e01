"""RouteNet example entry point — the reference's examples/Routenet/main.py workflow
(RNM:20-48) on the MI355X engine.  Run from a directory holding train_options.ini
(see examples/make_example.py).  Normalisation functions are numpy (the reference's use tf.math)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import ignnition_amd.framework_operations as ignnition  # noqa: E402


def normalization_routenet(feature, feature_name):
    if feature_name == 'traffic':
        feature = (feature - 170) / 130
    if feature_name == 'link_capacity':
        feature = (feature - 25000) / 40000
    return feature


def log(feature, feature_name):
    return np.log(feature)


def exp(feature, feature_name):
    return np.exp(feature)


def main():
    model = ignnition.create_model()
    ignnition.debug(model)
    ignnition.train_and_evaluate(model)
    return ignnition.predict(model)


if __name__ == "__main__":
    main()

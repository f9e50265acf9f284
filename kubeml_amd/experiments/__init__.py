"""Experiment harness (reference ml/experiments/: common/experiment.py, common/metrics.py,
common/utils.py, train.py, tf_train.py and the analysis notebooks)."""

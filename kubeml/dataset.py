"""reference python/kubeml/kubeml/dataset.py"""
from kubeml_amd.sdk.dataset import KubeDataset, _KubeArgs  # noqa: F401

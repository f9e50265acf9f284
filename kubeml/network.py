"""reference python/kubeml/kubeml/network.py"""
from kubeml_amd.sdk.model import KubeModel  # noqa: F401

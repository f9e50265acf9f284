"""Drop-in replacement for the reference's ``kubeml`` Python package
(python/kubeml/kubeml/__init__.py): ``from kubeml import KubeModel, KubeDataset``
keeps working for user functions written against the reference; the implementation
lives in :mod:`kubeml_amd` (resident MI355X workers, RCCL K-AVG, HIP kernels)."""
from kubeml_amd.sdk.dataset import KubeDataset
from kubeml_amd.sdk.model import KubeModel

__all__ = ["KubeModel", "KubeDataset"]
__version__ = "0.2.0"

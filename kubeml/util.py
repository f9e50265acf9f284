"""reference python/kubeml/kubeml/util.py"""
from kubeml_amd.api.types import STORAGE_SUBSET_SIZE  # noqa: F401
from kubeml_amd.sdk.util import get_gpu, get_subset_period, split_minibatches  # noqa: F401

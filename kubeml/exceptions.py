"""reference python/kubeml/kubeml/exceptions.py"""
from kubeml_amd.api.errors import (DataError, DatasetNotFoundError, InvalidArgsError,  # noqa: F401
                                   InvalidFormatError, KubeMLException, MergeError, StorageError)

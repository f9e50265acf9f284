"""Error envelope and exception classes shared by every component.

Envelope: ``{"error": str, "code": int}`` (reference ml/pkg/error/error.go:13-16 and
python/kubeml/kubeml/exceptions.py:1-14).  The SDK exception classes keep the
reference's names, messages and status codes (exceptions.py:15-48).
"""
from __future__ import annotations

from typing import Optional


class KubeMLException(Exception):
    def __init__(self, message, status_code=500):
        Exception.__init__(self, message)
        self.message = message
        self.status_code = status_code

    def to_dict(self):
        return {"error": self.message, "code": self.status_code}


class MergeError(KubeMLException):
    def __init__(self, e: Optional[Exception] = None):
        super().__init__(f"Error merging model: {e}", 500)


class DataError(KubeMLException):
    def __init__(self):
        super().__init__("Data not present in request", 400)


class InvalidFormatError(KubeMLException):
    def __init__(self):
        super().__init__("The data provided is not in an appropriate format", 400)


class StorageError(KubeMLException):
    def __init__(self, e: Exception):
        super().__init__(f"Could not access storage service: {str(e)}", 500)


class DatasetNotFoundError(KubeMLException):
    def __init__(self):
        super().__init__("Dataset not found in storage service", 404)


class InvalidArgsError(KubeMLException):
    def __init__(self, e: Exception):
        super().__init__(f"Error parsing function arguments: {str(e)}", 500)


class NotFoundError(KubeMLException):
    def __init__(self, what: str):
        super().__init__(f"{what} not found", 404)


class BadRequestError(KubeMLException):
    def __init__(self, what: str):
        super().__init__(what, 400)


def envelope(message: str, code: int) -> dict:
    return {"error": message, "code": code}


def check_function_error(status: int, body) -> Optional[KubeMLException]:
    """Parse a non-200 function/service response into an exception (error.go:36-59)."""
    if status == 200:
        return None
    if isinstance(body, dict) and "error" in body:
        return KubeMLException(str(body["error"]), int(body.get("code", status)))
    return KubeMLException(f"status {status}: {body!r}", status)

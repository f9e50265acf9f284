"""Small filesystem helpers shared by the JSON stores (atomic writes, name checks)."""
from __future__ import annotations

import json
import os
import tempfile

from ..api.errors import BadRequestError


def check_name(name: str, what: str = "name") -> str:
    if not name or "/" in name or "\\" in name or name.startswith(".") or len(name) > 200:
        raise BadRequestError(f"invalid {what} {name!r}")
    return name


def atomic_write(path: str, data: bytes):
    """Write-then-rename so a reader never sees a torn file."""
    d = os.path.dirname(path)
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp-")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(data)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


def write_json(path: str, obj):
    atomic_write(path, json.dumps(obj, indent=1).encode())


def read_json(path: str):
    with open(path) as f:
        return json.load(f)

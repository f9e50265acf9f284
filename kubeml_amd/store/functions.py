"""Function registry (replaces Fission packages/functions + HTTP triggers).

Reference: ``kubeml function create --name --code`` uploads a single Python file as a
Fission Package literal, creates a Function in env ``torch`` (concurrency 50, timeout
1000 s, idle 20 s, poolmgr) and an HTTPTrigger ``GET /{name}``
(ml/pkg/kubeml-cli/cmd/function.go:21-27, 71-145).

Here a function is the user's code file stored under ``<store>/functions/<name>.py``
with a JSON record; resident GPU workers import it once per job and call its
``main()`` (the Fission env's ``/specialize`` + ``/`` pair, ml/environment/server.py:60-128).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import asdict, dataclass
from typing import List

from ..api.errors import KubeMLException, NotFoundError
from ._fs import atomic_write, check_name, read_json, write_json

# reference defaults (function.go:21-27)
DEFAULT_ENV = "torch"
DEFAULT_CONCURRENCY = 50
DEFAULT_TIMEOUT = 1000
ARCHIVE_LITERAL_SIZE_LIMIT = 256 * 1024  # fission's literal package cap


@dataclass
class FunctionInfo:
    name: str
    environment: str = DEFAULT_ENV
    concurrency: int = DEFAULT_CONCURRENCY
    timeout: int = DEFAULT_TIMEOUT
    created: float = 0.0
    size: int = 0


class FunctionStore:
    def __init__(self, root: str):
        self.root = os.path.join(root, "functions")
        os.makedirs(self.root, exist_ok=True)
        self._lock = threading.Lock()

    def code_path(self, name: str) -> str:
        return os.path.join(self.root, check_name(name, "function name") + ".py")

    def _meta_path(self, name: str) -> str:
        return os.path.join(self.root, check_name(name, "function name") + ".json")

    def exists(self, name: str) -> bool:
        return os.path.exists(self.code_path(name))

    def create(self, name: str, code: bytes) -> FunctionInfo:
        with self._lock:
            if self.exists(name):
                raise KubeMLException(f"function {name} already exists", 400)
            if not code.strip():
                raise KubeMLException("empty function code", 400)
            try:
                compile(code, f"{name}.py", "exec")
            except SyntaxError as e:
                raise KubeMLException(f"function code does not compile: {e}", 400)
            atomic_write(self.code_path(name), code)
            info = FunctionInfo(name=name, created=time.time(), size=len(code))
            write_json(self._meta_path(name), asdict(info))
            return info

    def delete(self, name: str):
        with self._lock:
            if not self.exists(name):
                raise NotFoundError(f"function {name}")
            os.unlink(self.code_path(name))
            try:
                os.unlink(self._meta_path(name))
            except OSError:
                pass

    def get(self, name: str) -> FunctionInfo:
        if not self.exists(name):
            raise NotFoundError(f"function {name}")
        mp = self._meta_path(name)
        if os.path.exists(mp):
            return FunctionInfo(**read_json(mp))
        return FunctionInfo(name=name, created=os.path.getmtime(self.code_path(name)))

    def list(self) -> List[FunctionInfo]:
        out = []
        for f in sorted(os.listdir(self.root)):
            if f.endswith(".py") and not f.startswith("."):
                out.append(self.get(f[:-3]))
        return out

"""Storage service REST (reference python/storage/api.py:37-156, Flask + Mongo).

``POST /dataset/{name}`` with multipart files ``x-train, y-train, x-test, y-test``
(``.npy`` or ``.pkl``) → 64-sample shards in the :class:`ShardStore`;
``DELETE /dataset/{name}``; ``GET /health``.  Same responses:
``{"result": "Dataset created"}`` / ``{"error": ...}`` with 400 on a missing file or an
existing dataset, 404 on deleting a missing one.
"""
from __future__ import annotations

from ..api.errors import KubeMLException
from ..control.http import Response, Router, multipart_decode
from .shards import ShardStore

FIELDS = ("x-train", "y-train", "x-test", "y-test")


def create_from_multipart(store: ShardStore, name: str, body: bytes, content_type: str):
    try:
        files = multipart_decode(body, content_type)
    except KubeMLException:
        files = {}
    if not files:
        raise KubeMLException("Request does not include a file", 400)
    if store.exists(name):
        raise KubeMLException(f"Dataset {name} already exists", 400)
    missing = [f for f in FIELDS if f not in files]
    if missing:
        raise KubeMLException(f"missing files {missing}", 400)
    ext = files["x-train"][0].rsplit(".", 1)[-1].lower()
    if ext not in ("npy", "pkl"):
        raise KubeMLException("File extension not supported, must be one of [npy, pkl]", 400)
    arr = {k: (files[k][1], files[k][0]) for k in FIELDS}  # (bytes, filename) for shards.load_array
    store.create(name, arr["x-train"], arr["y-train"], arr["x-test"], arr["y-test"])
    return {"result": "Dataset created"}


def router(store: ShardStore) -> Router:
    r = Router("storage")

    def post(q):
        return create_from_multipart(store, q.params["name"], q.body, q.content_type)

    def delete(q):
        if not store.exists(q.params["name"]):
            return Response({"error": "Dataset does not exist"}, 404)
        store.delete(q.params["name"])
        return {"result": "Dataset deleted"}

    r.add("POST", "/dataset/{name}", post)
    r.add("DELETE", "/dataset/{name}", delete)
    r.add("GET", "/health", lambda q: "")
    return r

"""Minimal threaded HTTP/JSON server + client used by every control-plane role.

The reference's services are gorilla/mux routers (ml/pkg/*/api.go) and Flask apps
(python/storage/api.py, ml/environment/server.py).  The rebuild runs all roles in
one process and calls each other in-process; these HTTP endpoints exist so the
reference's wire surface (Appendix A of SURVEY.md) stays reachable — the CLI, the
experiments harness and external clients talk to them.

Stdlib only (``http.server.ThreadingHTTPServer``): no framework overhead on the
control path and nothing to install on the GPU box.
"""
from __future__ import annotations

import json
import logging
import re
import threading
import urllib.error
import urllib.parse
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api.errors import KubeMLException, envelope

log = logging.getLogger("kubeml.http")


class Request:
    def __init__(self, method: str, path: str, query: Dict[str, str], headers, body: bytes,
                 params: Dict[str, str]):
        self.method = method
        self.path = path
        self.query = query
        self.headers = headers
        self.body = body
        self.params = params

    def json(self):
        if not self.body:
            return None
        try:
            return json.loads(self.body)
        except ValueError:
            raise KubeMLException("request body is not valid JSON", 400)

    @property
    def content_type(self) -> str:
        return self.headers.get("Content-Type", "") if self.headers else ""


class Response:
    def __init__(self, body: Any = b"", status: int = 200, content_type: Optional[str] = None):
        if isinstance(body, (dict, list)) or (body is not None and not isinstance(body, (bytes, str))):
            self.body = json.dumps(body).encode()
            self.content_type = content_type or "application/json"
        elif isinstance(body, str):
            self.body = body.encode()
            self.content_type = content_type or "text/plain; charset=utf-8"
        else:
            self.body = body or b""
            self.content_type = content_type or "application/octet-stream"
        self.status = status


Handler = Callable[[Request], Any]


class Router:
    def __init__(self, name: str = "kubeml"):
        self.name = name
        self.routes: List[Tuple[str, "re.Pattern", Handler]] = []

    def add(self, methods: str, pattern: str, fn: Handler):
        rx = re.compile("^" + re.sub(r"\{(\w+)\}", r"(?P<\1>[^/]+)", pattern.rstrip("/") or "/") + "/?$")
        for m in methods.split("|"):
            self.routes.append((m.upper(), rx, fn))

    def route(self, methods: str, pattern: str):
        def deco(fn):
            self.add(methods, pattern, fn)
            return fn
        return deco

    def dispatch(self, method: str, path: str, query, headers, body: bytes) -> Response:
        allowed = False
        for m, rx, fn in self.routes:
            mt = rx.match(path)
            if not mt:
                continue
            allowed = True
            if m != method:
                continue
            req = Request(method, path, query, headers, body, {k: urllib.parse.unquote(v)
                                                                for k, v in mt.groupdict().items()})
            try:
                out = fn(req)
            except KubeMLException as e:
                return Response(e.to_dict(), e.status_code)
            except Exception as e:  # the reference envelope for unexpected errors (server.py:139-151)
                log.exception("%s %s failed", method, path)
                return Response(envelope(repr(e), 500), 500)
            return out if isinstance(out, Response) else Response(out if out is not None else b"")
        if allowed:
            return Response(envelope("method not allowed", 405), 405)
        return Response(envelope(f"no route {method} {path}", 404), 404)


class Server:
    """Serve a Router on ``host:port`` from a daemon thread."""

    def __init__(self, router: Router, host: str = "127.0.0.1", port: int = 0):
        self.router = router

        class _H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def _do(self):
                u = urllib.parse.urlsplit(self.path)
                q = {k: v[-1] for k, v in urllib.parse.parse_qs(u.query, keep_blank_values=True).items()}
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                resp = router.dispatch(self.command, u.path, q, self.headers, body)
                self.send_response(resp.status)
                self.send_header("Content-Type", resp.content_type)
                self.send_header("Content-Length", str(len(resp.body)))
                self.end_headers()
                if self.command != "HEAD":
                    self.wfile.write(resp.body)

            do_GET = do_POST = do_PUT = do_DELETE = do_HEAD = _do

            def log_message(self, fmt, *args):
                log.debug("%s " + fmt, router.name, *args)

        self.httpd = ThreadingHTTPServer((host, port), _H)
        self.httpd.daemon_threads = True
        self.host, self.port = self.httpd.server_address[:2]
        self._t: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def start(self) -> "Server":
        self._t = threading.Thread(target=self.httpd.serve_forever, name=f"http-{self.router.name}", daemon=True)
        self._t.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


# ------------------------------------------------------------------------------ client
class HttpError(KubeMLException):
    pass


def call(method: str, url: str, json_body: Any = None, data: Optional[bytes] = None,
         headers: Optional[Dict[str, str]] = None, timeout: float = 3600.0, raw: bool = False):
    """HTTP request; returns the decoded JSON (or text / bytes with ``raw``).  A non-2xx
    answer raises :class:`HttpError` carrying the server's error envelope."""
    h = dict(headers or {})
    if json_body is not None:
        data = json.dumps(json_body).encode()
        h.setdefault("Content-Type", "application/json")
    req = urllib.request.Request(url, data=data, method=method.upper(), headers=h)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            body = r.read()
            ctype = r.headers.get("Content-Type", "")
    except urllib.error.HTTPError as e:
        body = e.read()
        try:
            d = json.loads(body)
            msg, code = d.get("error", body.decode(errors="replace")), int(d.get("code", e.code))
        except ValueError:
            msg, code = body.decode(errors="replace"), e.code
        raise HttpError(msg, code)
    except urllib.error.URLError as e:
        raise HttpError(f"could not reach {url}: {e.reason}", 503)
    if raw:
        return body
    if "json" in ctype:
        return json.loads(body) if body else None
    return body.decode()


def multipart_encode(fields: Dict[str, Tuple[str, bytes]]) -> Tuple[bytes, str]:
    """Encode {field: (filename, bytes)} as multipart/form-data."""
    import uuid
    boundary = "kubeml" + uuid.uuid4().hex
    parts = []
    for name, (fname, blob) in fields.items():
        parts.append(f"--{boundary}\r\nContent-Disposition: form-data; name=\"{name}\"; filename=\"{fname}\"\r\n"
                     f"Content-Type: application/octet-stream\r\n\r\n".encode() + blob + b"\r\n")
    parts.append(f"--{boundary}--\r\n".encode())
    return b"".join(parts), f"multipart/form-data; boundary={boundary}"


def multipart_decode(body: bytes, content_type: str) -> Dict[str, Tuple[str, bytes]]:
    """Parse a multipart/form-data body into {field: (filename, bytes)}."""
    from email.parser import BytesParser
    from email.policy import HTTP
    if "multipart/form-data" not in content_type:
        raise KubeMLException("expected multipart/form-data", 400)
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + content_type.encode() + b"\r\n\r\n" + body)
    out = {}
    for part in msg.iter_parts():
        name = part.get_param("name", header="content-disposition")
        if not name:
            continue
        fname = part.get_filename() or name
        out[name] = (fname, part.get_payload(decode=True) or b"")
    return out

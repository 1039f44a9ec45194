"""REST config resolution -- ``ctrl.GetConfigOrDie()`` (``cmd/operator/start.go:152``).

Order [ext controller-runtime ``config.GetConfig``]: ``--kubeconfig`` flag,
``$KUBECONFIG``, in-cluster service account
(``KUBERNETES_SERVICE_HOST``/``_PORT`` + ``/var/run/secrets/kubernetes.io/serviceaccount``),
then ``~/.kube/config``.  Supported kubeconfig auth: bearer token / tokenFile,
client certificate + key (file or ``*-data``), basic auth, CA bundle or
``insecure-skip-tls-verify``, ``tls-server-name`` and ``proxy-url``-less
direct connections.  ``--qps``/``--burst`` are applied by the caller.

Token files rotate: the in-cluster service-account token is a projected,
kubelet-refreshed file (bound tokens expire; ``/var/run/secrets/.../token``).
[ext client-go ``transport.NewCachedFileTokenSource``] re-reads the file once
a minute (10 s leeway) and drops its cached token when a request comes back
401; :meth:`RestConfig.token` and :meth:`RestConfig.reset_token` do the same,
and the HTTP transport re-stamps its ``Authorization`` header when the token
changes (``runtime/http.py``).
"""
from __future__ import annotations

import base64
import os
import ssl
import tempfile
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
TOKEN_FILE_PERIOD = 60.0   # client-go fileTokenSource: a token read from a file is good for a minute
TOKEN_LEEWAY = 10.0        # client-go cachingTokenSource: refresh that long before expiry


class ConfigError(RuntimeError):
    pass


@dataclass
class RestConfig:
    host: str
    bearer_token: str = ""
    bearer_token_file: str = ""
    username: str = ""
    password: str = ""
    ca_file: str = ""
    ca_data: bytes = b""
    cert_file: str = ""
    key_file: str = ""
    cert_data: bytes = b""
    key_data: bytes = b""
    insecure: bool = False
    tls_server_name: str = ""
    qps: float = 30.0
    burst: int = 50
    user_agent: str = "cron-operator-amd"
    _tmp: List[str] = field(default_factory=list)
    _file_token: str = ""
    _file_token_refresh_at: float = 0.0   # monotonic; 0 = read on next use

    def token(self) -> str:
        """The bearer token; a ``tokenFile`` is re-read at most once per ``TOKEN_FILE_PERIOD -
        TOKEN_LEEWAY`` seconds.  A read error keeps the last good token (client-go logs and
        serves the cached one), falling back to the inline ``token``."""
        if self.bearer_token_file:
            now = time.monotonic()
            if now >= self._file_token_refresh_at:
                try:
                    with open(self.bearer_token_file) as fh:
                        self._file_token = fh.read().strip()
                    self._file_token_refresh_at = now + TOKEN_FILE_PERIOD - TOKEN_LEEWAY
                except OSError:
                    pass
            if self._file_token:
                return self._file_token
        return self.bearer_token

    def reset_token(self) -> None:
        """Forget the cached file token (client-go ``ResetTokenOlderThan`` after a 401)."""
        self._file_token_refresh_at = 0.0

    def _materialise(self, data: bytes, suffix: str) -> str:
        fd, path = tempfile.mkstemp(prefix="cron-operator-", suffix=suffix)
        with os.fdopen(fd, "wb") as fh:
            fh.write(data)
        self._tmp.append(path)
        return path

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.host.startswith("https://"):
            return None
        ctx = ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        elif self.ca_data:
            ctx.load_verify_locations(cadata=self.ca_data.decode())
        elif self.ca_file:
            ctx.load_verify_locations(cafile=self.ca_file)
        cert = self.cert_file or (self._materialise(self.cert_data, ".crt") if self.cert_data else "")
        key = self.key_file or (self._materialise(self.key_data, ".key") if self.key_data else "")
        if cert:
            ctx.load_cert_chain(cert, key or None)
        ctx.set_alpn_protocols(["http/1.1"])
        return ctx

    def auth_headers(self) -> Dict[str, str]:
        h = {"User-Agent": self.user_agent}
        tok = self.token()
        if tok:
            h["Authorization"] = f"Bearer {tok}"
        elif self.username:
            cred = base64.b64encode(f"{self.username}:{self.password}".encode()).decode()
            h["Authorization"] = f"Basic {cred}"
        return h


def _b64(s: Optional[str]) -> bytes:
    return base64.b64decode(s) if s else b""


def _resolve(path: str, base: str) -> str:
    if not path or os.path.isabs(path):
        return path
    return os.path.join(os.path.dirname(base), path)


def load_kubeconfig(path: str, context: Optional[str] = None) -> RestConfig:
    try:
        with open(path) as fh:
            doc: Dict[str, Any] = yaml.safe_load(fh) or {}
    except OSError as e:
        raise ConfigError(f"cannot read kubeconfig {path}: {e}") from None
    ctx_name = context or doc.get("current-context")
    ctxs = {c["name"]: c.get("context") or {} for c in doc.get("contexts") or []}
    if not ctx_name or ctx_name not in ctxs:
        raise ConfigError(f"context {ctx_name!r} not found in {path}")
    ctx = ctxs[ctx_name]
    clusters = {c["name"]: c.get("cluster") or {} for c in doc.get("clusters") or []}
    users = {u["name"]: u.get("user") or {} for u in doc.get("users") or []}
    cl = clusters.get(ctx.get("cluster", ""))
    if cl is None:
        raise ConfigError(f"cluster {ctx.get('cluster')!r} not found in {path}")
    us = users.get(ctx.get("user", ""), {})
    if "exec" in us or "auth-provider" in us:
        raise ConfigError("exec/auth-provider credential plugins are not supported; use a token or client cert")
    return RestConfig(
        host=cl.get("server", "").rstrip("/"),
        ca_file=_resolve(cl.get("certificate-authority", ""), path),
        ca_data=_b64(cl.get("certificate-authority-data")),
        insecure=bool(cl.get("insecure-skip-tls-verify", False)),
        tls_server_name=cl.get("tls-server-name", ""),
        bearer_token=us.get("token", ""),
        bearer_token_file=_resolve(us.get("tokenFile", ""), path),
        username=us.get("username", ""),
        password=us.get("password", ""),
        cert_file=_resolve(us.get("client-certificate", ""), path),
        key_file=_resolve(us.get("client-key", ""), path),
        cert_data=_b64(us.get("client-certificate-data")),
        key_data=_b64(us.get("client-key-data")),
    )


def in_cluster_config() -> Optional[RestConfig]:
    host = os.environ.get("KUBERNETES_SERVICE_HOST")
    port = os.environ.get("KUBERNETES_SERVICE_PORT")
    if not host or not port:
        return None
    if ":" in host and not host.startswith("["):
        host = f"[{host}]"
    return RestConfig(host=f"https://{host}:{port}", bearer_token_file=os.path.join(SA_DIR, "token"),
                      ca_file=os.path.join(SA_DIR, "ca.crt"))


def get_config(kubeconfig: str = "", context: Optional[str] = None) -> RestConfig:
    if kubeconfig:
        return load_kubeconfig(kubeconfig, context)
    env = os.environ.get("KUBECONFIG", "")
    if env:
        for p in env.split(os.pathsep):
            if p and os.path.exists(p):
                return load_kubeconfig(p, context)
    ic = in_cluster_config()
    if ic is not None:
        return ic
    home = os.path.join(os.path.expanduser("~"), ".kube", "config")
    if os.path.exists(home):
        return load_kubeconfig(home, context)
    raise ConfigError("could not locate a kubeconfig (--kubeconfig, $KUBECONFIG, in-cluster, ~/.kube/config)")


def write_kubeconfig(path: str, server: str, token: str = "", insecure: bool = False) -> None:
    """Minimal kubeconfig for a server (used for the fake apiserver)."""
    doc = {"apiVersion": "v1", "kind": "Config", "current-context": "fake",
           "clusters": [{"name": "fake", "cluster": {"server": server, "insecure-skip-tls-verify": insecure}}],
           "users": [{"name": "fake", "user": {"token": token} if token else {}}],
           "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "fake"}}]}
    with open(path, "w") as fh:
        yaml.safe_dump(doc, fh)

"""REST config resolution -- ``ctrl.GetConfigOrDie()`` (``cmd/operator/start.go:152``).

Order [ext controller-runtime ``config.GetConfig``]: ``--kubeconfig`` flag,
``$KUBECONFIG``, in-cluster service account
(``KUBERNETES_SERVICE_HOST``/``_PORT`` + ``/var/run/secrets/kubernetes.io/serviceaccount``),
then ``~/.kube/config``.  Supported kubeconfig auth: bearer token / tokenFile,
client certificate + key (file or ``*-data``), exec credential plugins, basic auth, CA bundle or
``insecure-skip-tls-verify``, ``tls-server-name``.  ``--qps``/``--burst`` are applied by the caller.

Proxies follow client-go: the kubeconfig's ``proxy-url`` for every request, else
``HTTPS_PROXY``/``HTTP_PROXY`` minus ``NO_PROXY`` (Go ``http.ProxyFromEnvironment``;
loopback servers are never proxied).  Only ``http://`` proxies are supported: plain
requests in absolute form, ``https`` servers through a ``CONNECT`` tunnel
(``runtime/fasthttp.py``), with ``user:password@`` sent as ``Proxy-Authorization``.

Token files rotate: the in-cluster service-account token is a projected,
kubelet-refreshed file (bound tokens expire; ``/var/run/secrets/.../token``).
[ext client-go ``transport.NewCachedFileTokenSource``] re-reads the file once
a minute (10 s leeway) and drops its cached token when a request comes back
401; :meth:`RestConfig.token` and :meth:`RestConfig.reset_token` do the same,
and the HTTP transport re-stamps its ``Authorization`` header when the token
changes (``runtime/http.py``).

``users[].user.exec`` credential plugins (``kubelogin``, ``aws eks get-token``,
``gke-gcloud-auth-plugin``, ...) follow [ext client-go
``plugin/pkg/client/auth/exec``]: the command runs with the kubeconfig's
``args``/``env`` plus ``KUBERNETES_EXEC_INFO`` (an ``ExecCredential`` request,
with the cluster when ``provideClusterInfo``), and its stdout must be an
``ExecCredential`` of the same ``apiVersion`` carrying a ``token`` and/or a
``clientCertificateData``/``clientKeyData`` pair.  The credential is cached
until its ``expirationTimestamp`` (forever without one) and fetched again after
a 401.  Plugins run non-interactively: ``interactiveMode: Always`` is refused.
"""
from __future__ import annotations

import base64
import ipaddress
import json
import os
import ssl
import subprocess
import tempfile
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import urlsplit

import yaml

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
TOKEN_FILE_PERIOD = 60.0   # client-go fileTokenSource: a token read from a file is good for a minute
TOKEN_LEEWAY = 10.0        # client-go cachingTokenSource: refresh that long before expiry
EXEC_API_VERSIONS = ("client.authentication.k8s.io/v1", "client.authentication.k8s.io/v1beta1")
EXEC_TIMEOUT = 60.0        # seconds a credential plugin may run


class ConfigError(RuntimeError):
    pass


@dataclass
class ExecCredentials:
    token: str = ""
    cert_data: bytes = b""
    key_data: bytes = b""
    expires_at: Optional[float] = None   # wall-clock seconds; None = until a 401


@dataclass
class ExecProvider:
    """A kubeconfig ``user.exec`` stanza (``ExecConfig``)."""
    command: str
    api_version: str
    args: List[str] = field(default_factory=list)
    env: List[Dict[str, str]] = field(default_factory=list)
    interactive_mode: str = "IfAvailable"
    provide_cluster_info: bool = False
    install_hint: str = ""
    cluster: Dict[str, Any] = field(default_factory=dict)   # the kubeconfig cluster, for provideClusterInfo

    @staticmethod
    def from_kubeconfig(ex: Dict[str, Any], cluster: Dict[str, Any]) -> "ExecProvider":
        cmd = ex.get("command") or ""
        if not cmd:
            raise ConfigError("exec plugin: command must be specified")
        api_version = ex.get("apiVersion") or ""
        if api_version not in EXEC_API_VERSIONS:
            raise ConfigError(f"exec plugin: invalid apiVersion {api_version!r}")
        mode = ex.get("interactiveMode") or ""
        if not mode:
            if api_version.endswith("/v1"):
                raise ConfigError("exec plugin: interactiveMode must be specified for "
                                  f"{api_version} to use exec authentication plugin")
            mode = "IfAvailable"
        if mode not in ("Never", "IfAvailable", "Always"):
            raise ConfigError(f"exec plugin: invalid interactiveMode {mode!r}")
        if mode == "Always":
            raise ConfigError("exec plugin cannot support interactive mode: the operator has no terminal")
        env = ex.get("env") or []
        for e in env:
            if not isinstance(e, dict) or "name" not in e:
                raise ConfigError("exec plugin: env entries need a name")
        return ExecProvider(command=cmd, api_version=api_version, args=[str(a) for a in ex.get("args") or []],
                            env=env, interactive_mode=mode,
                            provide_cluster_info=bool(ex.get("provideClusterInfo", False)),
                            install_hint=ex.get("installHint") or "", cluster=dict(cluster))

    def _exec_info(self) -> str:
        spec: Dict[str, Any] = {"interactive": False}
        if self.provide_cluster_info:
            c = self.cluster
            info: Dict[str, Any] = {"server": c.get("server", "")}
            for k in ("tls-server-name", "insecure-skip-tls-verify", "certificate-authority-data", "proxy-url",
                      "disable-compression"):
                if c.get(k):
                    info[k] = c[k]
            ext = next((e.get("extension") for e in c.get("extensions") or []
                        if e.get("name") == "client.authentication.k8s.io/exec"), None)
            if ext is not None:
                info["config"] = ext
            spec["cluster"] = info
        return json.dumps({"apiVersion": self.api_version, "kind": "ExecCredential", "spec": spec})

    def run(self) -> ExecCredentials:
        env = dict(os.environ)
        for e in self.env:
            env[e["name"]] = str(e.get("value", ""))
        env["KUBERNETES_EXEC_INFO"] = self._exec_info()
        try:
            p = subprocess.run([self.command, *self.args], env=env, stdin=subprocess.DEVNULL,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=EXEC_TIMEOUT, check=False)
        except FileNotFoundError:
            hint = f"\n\n{self.install_hint}" if self.install_hint else ""
            raise ConfigError(f"exec: executable {self.command} not found{hint}") from None
        except (OSError, subprocess.TimeoutExpired) as e:
            raise ConfigError(f"exec: executable {self.command} failed: {e}") from None
        if p.returncode != 0:
            err = p.stderr.decode(errors="replace").strip()
            raise ConfigError(f"exec: executable {self.command} failed with exit code {p.returncode}"
                              + (f": {err}" if err else ""))
        return self.parse(p.stdout)

    def parse(self, out: bytes) -> ExecCredentials:
        try:
            doc = json.loads(out)
        except ValueError as e:
            raise ConfigError(f"exec: decoding stdout: {e}") from None
        if not isinstance(doc, dict) or doc.get("kind") != "ExecCredential":
            raise ConfigError("exec: stdout is not an ExecCredential")
        if doc.get("apiVersion") != self.api_version:
            raise ConfigError(f"exec plugin is configured to use API version {self.api_version}, "
                              f"plugin returned version {doc.get('apiVersion')}")
        st = doc.get("status")
        if not isinstance(st, dict):
            raise ConfigError("exec plugin didn't return a status field")
        token = st.get("token") or ""
        cert, key = st.get("clientCertificateData") or "", st.get("clientKeyData") or ""
        if not token and not (cert and key):
            raise ConfigError("exec plugin didn't return a token or cert/key pair")
        if bool(cert) != bool(key):
            raise ConfigError("exec plugin returned only certificate or key, not both")
        exp = None
        if st.get("expirationTimestamp"):
            from ..api.meta import time_from_json
            try:
                t = time_from_json(str(st["expirationTimestamp"]))
            except ValueError:
                t = None
            if t is None:
                raise ConfigError(f"exec: bad expirationTimestamp {st['expirationTimestamp']!r}")
            exp = t.unix_nano() / 1e9
        return ExecCredentials(token=token, cert_data=cert.encode(), key_data=key.encode(), expires_at=exp)


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
    proxy_url: str = ""                   # kubeconfig ``proxy-url``: every request, no NO_PROXY
    qps: float = 150.0                    # cmd/main.py DEFAULT_QPS / DEFAULT_BURST
    burst: int = 300
    user_agent: str = "cron-operator-amd"
    exec_provider: Optional[ExecProvider] = None
    _file_token: str = ""
    _file_token_refresh_at: float = 0.0   # monotonic; 0 = read on next use
    _exec_creds: Optional[ExecCredentials] = None
    cert_generation: int = 0              # bumped when an exec plugin hands out a new client certificate

    @property
    def rotating(self) -> bool:
        """Credentials can change while the process runs (token file or exec plugin)."""
        return bool(self.bearer_token_file) or self.exec_provider is not None

    def exec_stale(self) -> bool:
        """An exec plugin is configured and its credential is missing or expired."""
        if self.exec_provider is None:
            return False
        c = self._exec_creds
        return c is None or (c.expires_at is not None and time.time() >= c.expires_at)

    def refresh_exec(self) -> None:
        """Run the plugin now if its credential is stale (blocking: the HTTP transport calls
        this in a worker thread so the event loop keeps serving leases and watches)."""
        if self.exec_stale():
            old = self._exec_creds
            new = self.exec_provider.run()  # type: ignore[union-attr]
            if old is None or (new.cert_data, new.key_data) != (old.cert_data, old.key_data):
                self.cert_generation += 1
            self._exec_creds = new

    def _exec(self) -> ExecCredentials:
        """The plugin's cached credential -- even when it has expired: refreshing runs the
        plugin (a subprocess, up to 60 s), which the HTTP transport does off the event loop
        before each request attempt (``HttpTransport._fresh_exec``).  Only the very first
        use, with nothing cached yet, runs the plugin here."""
        if self._exec_creds is None:
            self.refresh_exec()
        assert self._exec_creds is not None
        return self._exec_creds

    def client_cert(self) -> Tuple[bytes, bytes]:
        """PEM client certificate and key from an exec plugin, or empty."""
        if self.exec_provider is None:
            return b"", b""
        c = self._exec()
        return c.cert_data, c.key_data

    def token(self) -> str:
        """The bearer token; a ``tokenFile`` is re-read at most once per ``TOKEN_FILE_PERIOD -
        TOKEN_LEEWAY`` seconds.  A read error keeps the last good token (client-go logs and
        serves the cached one), falling back to the inline ``token``.  An exec plugin's token
        takes precedence over both (client-go wraps the transport with the exec authenticator)."""
        if self.exec_provider is not None:
            tok = self._exec().token
            if tok:
                return tok
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
        """Forget the cached file token (client-go ``ResetTokenOlderThan`` after a 401) and an
        exec plugin's credential (the exec authenticator refreshes on 401)."""
        self._file_token_refresh_at = 0.0
        if self._exec_creds is not None:
            self._exec_creds.expires_at = 0.0

    @staticmethod
    def _materialise(data: bytes, suffix: str) -> str:
        """Write PEM bytes to a private (0600) temp file for ``load_cert_chain``; the caller
        unlinks it as soon as the chain is loaded."""
        fd, path = tempfile.mkstemp(prefix="cron-operator-", suffix=suffix)
        with os.fdopen(fd, "wb") as fh:
            fh.write(data)
        return path

    def tls_material(self) -> Optional[Dict[str, Any]]:
        """The PEM material :meth:`ssl_context` is built from, for the native connections'
        own ``SSL_CTX`` (``ops/netconn_native.tls_context``): ``cadata``/``cafile``,
        ``certdata``/``keydata`` (bytes; files read), ``verify`` and ``check_hostname``."""
        if not self.host.startswith("https://"):
            return None
        cert_data, key_data = self.client_cert()
        if not cert_data:
            cert_data, key_data = self.cert_data, self.key_data
            if self.cert_file:
                with open(self.cert_file, "rb") as fh:
                    cert_data = fh.read()
                key_data = b""
                if self.key_file:
                    with open(self.key_file, "rb") as fh:
                        key_data = fh.read()
        return {"cadata": None if self.insecure else (self.ca_data or None),
                "cafile": None if self.insecure or self.ca_data else (self.ca_file or None),
                "certdata": cert_data or None, "keydata": key_data or None,
                "verify": not self.insecure, "check_hostname": not self.insecure}

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
        cert_data, key_data = self.client_cert()
        cert, key = "", ""
        if not cert_data:
            cert, key = self.cert_file, self.key_file
            cert_data = b"" if cert else self.cert_data
            key_data = b"" if key else self.key_data
        tmp: List[str] = []
        try:
            if cert_data:
                cert = self._materialise(cert_data, ".crt")
                tmp.append(cert)
            if key_data:
                key = self._materialise(key_data, ".key")
                tmp.append(key)
            if cert:
                ctx.load_cert_chain(cert, key or None)
        finally:
            for path in tmp:  # key material does not outlive the load
                try:
                    os.unlink(path)
                except OSError:
                    pass
        ctx.set_alpn_protocols(["http/1.1"])
        return ctx

    def proxy(self) -> str:
        """The proxy for this server: kubeconfig ``proxy-url`` (validated when the kubeconfig is
        loaded), else the environment.  An environment proxy of a scheme this client cannot
        speak (``https://``, ``socks5://``) is skipped with a warning -- the connection goes
        direct -- rather than failing every request."""
        if self.proxy_url:
            return self.proxy_url
        try:
            return proxy_from_environment(self.host)
        except ConfigError as e:
            from ..utils.logging import get_logger

            get_logger("kubeconfig").info("ignoring the environment proxy; connecting directly", reason=str(e))
            return ""

    def auth_headers(self, token: Optional[str] = None) -> Dict[str, str]:
        """Headers for every request; ``token`` saves a second :meth:`token` call when the caller
        just fetched it."""
        h = {"User-Agent": self.user_agent}
        tok = self.token() if token is None else token
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
    if "auth-provider" in us:
        raise ConfigError("auth-provider plugins are not supported (removed from client-go for gcp/azure); "
                          "use an exec credential plugin, a token or a client certificate")
    exec_provider = ExecProvider.from_kubeconfig(us["exec"], cl) if us.get("exec") else None
    return RestConfig(
        host=cl.get("server", "").rstrip("/"),
        ca_file=_resolve(cl.get("certificate-authority", ""), path),
        ca_data=_b64(cl.get("certificate-authority-data")),
        insecure=bool(cl.get("insecure-skip-tls-verify", False)),
        tls_server_name=cl.get("tls-server-name", ""),
        proxy_url=_check_proxy(cl.get("proxy-url", "")),
        bearer_token=us.get("token", ""),
        bearer_token_file=_resolve(us.get("tokenFile", ""), path),
        username=us.get("username", ""),
        password=us.get("password", ""),
        cert_file=_resolve(us.get("client-certificate", ""), path),
        key_file=_resolve(us.get("client-key", ""), path),
        cert_data=_b64(us.get("client-certificate-data")),
        key_data=_b64(us.get("client-key-data")),
        exec_provider=exec_provider,
    )


def _check_proxy(url: str) -> str:
    if url and urlsplit(url if "://" in url else "http://" + url).scheme != "http":
        raise ConfigError(f"proxy {url!r}: only http:// proxies are supported (CONNECT tunnels for https "
                          "servers)")
    return url


def _no_proxy_match(host: str, port: int, entries: str) -> bool:
    """Go ``httpproxy.Config``'s NO_PROXY rules: ``*``; an IP or CIDR; a domain name matching
    itself and its subdomains, or with a leading ``.`` (or ``*.``) its subdomains only; IPs and
    names optionally with ``:port``."""
    host = host.strip("[]").lower()
    try:
        ip = ipaddress.ip_address(host)
    except ValueError:
        ip = None
    for raw in entries.split(","):
        e = raw.strip().lower()
        if not e:
            continue
        if e == "*":
            return True
        if "/" in e:
            try:
                if ip is not None and ip in ipaddress.ip_network(e, strict=False):
                    return True
            except ValueError:
                pass
            continue
        e_port = 0
        h = e
        if e.startswith("["):
            h, _, rest = e[1:].partition("]")
            e_port = int(rest[1:]) if rest.startswith(":") and rest[1:].isdigit() else 0
        elif e.count(":") == 1:
            h, _, ps = e.partition(":")
            e_port = int(ps) if ps.isdigit() else 0
        if e_port and e_port != port:
            continue
        if ip is not None:
            try:
                if ipaddress.ip_address(h) == ip:
                    return True
            except ValueError:
                pass
            continue
        if h.startswith("*."):
            h = h[1:]
        if h.startswith("."):  # subdomains only
            if host.endswith(h):
                return True
        elif host == h or host.endswith("." + h):
            return True
    return False


def proxy_from_environment(server: str) -> str:
    """``http.ProxyFromEnvironment`` for ``server``: ``HTTPS_PROXY``/``HTTP_PROXY`` by the
    server's scheme (upper case first, then lower case), minus ``NO_PROXY`` matches; loopback
    servers never go through a proxy."""
    u = urlsplit(server)
    host = (u.hostname or "").lower()
    if host == "localhost" or host.endswith(".localhost"):
        return ""
    try:
        if ipaddress.ip_address(host).is_loopback:
            return ""
    except ValueError:
        pass
    names = ("HTTPS_PROXY", "https_proxy") if u.scheme == "https" else ("HTTP_PROXY", "http_proxy")
    proxy = next((os.environ[n] for n in names if os.environ.get(n)), "")
    if not proxy:
        return ""
    no_proxy = os.environ.get("NO_PROXY") or os.environ.get("no_proxy") or ""
    port = u.port or (443 if u.scheme == "https" else 80)
    if no_proxy and _no_proxy_match(host, port, no_proxy):
        return ""
    return _check_proxy(proxy)


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

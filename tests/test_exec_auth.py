"""kubeconfig ``users[].user.exec`` credential plugins (client-go ``plugin/pkg/client/auth/exec``).

The plugin here is a small Python script: it counts its runs, records the
``KUBERNETES_EXEC_INFO`` it was given, and prints an ``ExecCredential`` whose
token (and optional expiry / client certificate) come from files the test edits.
"""
from __future__ import annotations

import asyncio
import json
import os
import sys
import tempfile
import textwrap

import pytest
import yaml

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.apiserver.http import APIServerApp
from cron_operator_amd.runtime.client import Client
from cron_operator_amd.runtime.fasthttp import HttpPool
from cron_operator_amd.runtime.http import HttpTransport
from cron_operator_amd.runtime.kubeconfig import ConfigError, ExecProvider, load_kubeconfig
from cron_operator_amd.runtime.servers import self_signed_cert
from cron_operator_amd.testing.env import TestEnv

CM = GroupVersionResource("", "v1", "configmaps")
V1 = "client.authentication.k8s.io/v1"
V1B1 = "client.authentication.k8s.io/v1beta1"

PLUGIN = textwrap.dedent("""\
    import json, os, sys, time
    d = sys.argv[1]
    if os.path.exists(os.path.join(d, "sleep")):
        time.sleep(float(open(os.path.join(d, "sleep")).read()))
    n = int(open(os.path.join(d, "runs")).read()) if os.path.exists(os.path.join(d, "runs")) else 0
    open(os.path.join(d, "runs"), "w").write(str(n + 1))
    open(os.path.join(d, "info.json"), "w").write(os.environ["KUBERNETES_EXEC_INFO"])
    open(os.path.join(d, "env"), "w").write(os.environ.get("PLUGIN_FLAVOUR", ""))
    st = {"token": open(os.path.join(d, "token")).read().strip()}
    if os.path.exists(os.path.join(d, "expiry")):
        st["expirationTimestamp"] = open(os.path.join(d, "expiry")).read().strip()
    if os.path.exists(os.path.join(d, "crt")):
        st["clientCertificateData"] = open(os.path.join(d, "crt")).read()
        st["clientKeyData"] = open(os.path.join(d, "key")).read()
    print(json.dumps({"apiVersion": os.environ.get("PLUGIN_API", "%s"), "kind": "ExecCredential", "status": st}))
""" % V1)


def _kubeconfig(d: str, server: str, **exec_extra) -> str:
    with open(os.path.join(d, "plugin.py"), "w") as fh:
        fh.write(PLUGIN)
    ex = {"apiVersion": V1, "command": sys.executable, "args": [os.path.join(d, "plugin.py"), d],
          "env": [{"name": "PLUGIN_FLAVOUR", "value": "vanilla"}], "interactiveMode": "Never",
          "provideClusterInfo": True}
    ex.update(exec_extra)
    doc = {"apiVersion": "v1", "kind": "Config", "current-context": "c",
           "clusters": [{"name": "c", "cluster": {"server": server, "tls-server-name": "api.example",
                                                  "extensions": [{"name": "client.authentication.k8s.io/exec",
                                                                  "extension": {"audience": "cron"}}]}}],
           "users": [{"name": "u", "user": {"exec": ex}}],
           "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}]}
    p = os.path.join(d, "kubeconfig")
    with open(p, "w") as fh:
        yaml.safe_dump(doc, fh)
    return p


def _runs(d: str) -> int:
    return int(open(os.path.join(d, "runs")).read())


@pytest.mark.parametrize("fast", [True, False])
async def test_exec_plugin_token_cached_refreshed_on_expiry_and_401(fast):
    env = TestEnv()
    env.server.tokens = {"tok-1": {"username": "u"}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "token"), "w") as fh:
            fh.write("tok-1")
        cfg = load_kubeconfig(_kubeconfig(d, f"http://127.0.0.1:{port}"))
        c = Client(HttpTransport(cfg, fast=fast), qps=-1)
        try:
            await c.create(CM, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "a"}}, "default")
            await c.get(CM, "default", "a")
            assert _runs(d) == 1  # no expiry: cached
            info = json.load(open(os.path.join(d, "info.json")))
            assert info["apiVersion"] == V1 and info["kind"] == "ExecCredential"
            assert info["spec"]["interactive"] is False
            assert info["spec"]["cluster"]["server"] == f"http://127.0.0.1:{port}"
            assert info["spec"]["cluster"]["tls-server-name"] == "api.example"
            assert info["spec"]["cluster"]["config"] == {"audience": "cron"}
            assert open(os.path.join(d, "env")).read() == "vanilla"

            # the identity provider rotates: the cached token gets one 401, which forces a re-run
            with open(os.path.join(d, "token"), "w") as fh:
                fh.write("tok-2")
            env.server.tokens = {"tok-2": {"username": "u"}}
            with pytest.raises(errors.ApiError) as e:
                await c.get(CM, "default", "a")
            assert e.value.code == 401
            assert (await c.get(CM, "default", "a"))["metadata"]["name"] == "a"
            assert _runs(d) == 2

            # an expirationTimestamp in the past: every use re-runs (off the event loop for
            # requests) until a fresh one comes back
            with open(os.path.join(d, "token"), "w") as fh:
                fh.write("tok-3")
            with open(os.path.join(d, "expiry"), "w") as fh:
                fh.write("2000-01-01T00:00:00Z")
            env.server.tokens = {"tok-2": {"username": "u"}, "tok-3": {"username": "u"}}
            cfg._exec_creds.expires_at = 0.0  # the cached tok-2 credential expired
            await c.get(CM, "default", "a")
            assert _runs(d) >= 3 and cfg.token() == "tok-3"
            runs = _runs(d)
            with open(os.path.join(d, "expiry"), "w") as fh:
                fh.write("2999-01-01T00:00:00Z")
            env.server.tokens = {"tok-3": {"username": "u"}}
            await c.get(CM, "default", "a")
            await c.get(CM, "default", "a")
            assert _runs(d) == runs + 1  # fetched once more, then cached until 2999
        finally:
            await c.close()
            await app.stop()


async def test_slow_exec_plugin_does_not_block_the_event_loop():
    """A plugin that takes a while (an SSO round trip) runs in a worker thread: lease renewals
    and watches keep going, and concurrent requests wait for one run."""
    env = TestEnv()
    env.server.tokens = {"tok": {"username": "u"}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    with tempfile.TemporaryDirectory() as d:
        for name, text in (("token", "tok"), ("sleep", "0.6")):
            with open(os.path.join(d, name), "w") as fh:
                fh.write(text)
        c = Client(HttpTransport(load_kubeconfig(_kubeconfig(d, f"http://127.0.0.1:{port}"))), qps=-1)
        ticks = 0

        async def ticker():
            nonlocal ticks
            while True:
                await asyncio.sleep(0.05)
                ticks += 1

        t = asyncio.ensure_future(ticker())
        try:
            got = await asyncio.gather(*(c.get(CM, "default", "x") for _ in range(3)), return_exceptions=True)
            assert all(isinstance(g, errors.ApiError) and g.code == 404 for g in got)
            assert ticks >= 6 and _runs(d) == 1
        finally:
            t.cancel()
            await c.close()
            await app.stop()


def test_exec_plugin_client_certificate_loaded_and_rotated():
    with tempfile.TemporaryDirectory() as d:
        crt, key = self_signed_cert(d)
        for src, dst in ((crt, "crt"), (key, "key")):
            with open(src) as i, open(os.path.join(d, dst), "w") as o:
                o.write(i.read())
        with open(os.path.join(d, "token"), "w") as fh:
            fh.write("")
        cfg = load_kubeconfig(_kubeconfig(d, "https://127.0.0.1:1"))
        before = set(os.listdir(tempfile.gettempdir()))
        ctx = cfg.ssl_context()
        assert ctx is not None and cfg.cert_generation == 1
        # the PEM temp files used to load the chain are gone
        leaked = [f for f in set(os.listdir(tempfile.gettempdir())) - before if f.startswith("cron-operator-")]
        assert leaked == []
        assert cfg.token() == ""  # certificate-only credential
        # the same certificate again does not bump the generation; a new one does
        cfg._exec_creds.expires_at = 0.0
        cfg.refresh_exec()
        assert cfg.cert_generation == 1
        d2 = os.path.join(d, "two")
        os.mkdir(d2)
        crt2, key2 = self_signed_cert(d2)
        for src, dst in ((crt2, "crt"), (key2, "key")):
            with open(src) as i, open(os.path.join(d, dst), "w") as o:
                o.write(i.read())
        cfg._exec_creds.expires_at = 0.0
        cfg.client_cert()  # reads the cache: never runs the plugin on the caller's thread
        assert cfg.cert_generation == 1
        cfg.refresh_exec()  # what HttpTransport does in a worker thread before a request
        assert cfg.cert_generation == 2

        pool = HttpPool("https://127.0.0.1:1", ssl_context=ctx)
        pool.set_ssl(cfg.ssl_context())
        assert pool.ssl is not ctx and pool._ssl_gen == 1


@pytest.mark.parametrize("stanza,msg", [
    ({"apiVersion": V1, "command": "x"}, "interactiveMode must be specified"),
    ({"apiVersion": V1, "command": "x", "interactiveMode": "Always"}, "cannot support interactive mode"),
    ({"apiVersion": V1, "command": "x", "interactiveMode": "Sometimes"}, "invalid interactiveMode"),
    ({"apiVersion": "client.authentication.k8s.io/v1alpha1", "command": "x"}, "invalid apiVersion"),
    ({"apiVersion": V1, "interactiveMode": "Never"}, "command must be specified"),
    ({"apiVersion": V1, "command": "x", "interactiveMode": "Never", "env": [{"value": "v"}]}, "need a name"),
])
def test_exec_stanza_validation(stanza, msg):
    with pytest.raises(ConfigError, match=msg):
        ExecProvider.from_kubeconfig(stanza, {"server": "https://x"})


def test_exec_v1beta1_defaults_interactive_mode():
    p = ExecProvider.from_kubeconfig({"apiVersion": V1B1, "command": "x"}, {})
    assert p.interactive_mode == "IfAvailable"


@pytest.mark.parametrize("out,msg", [
    (b"not json", "decoding stdout"),
    (json.dumps({"apiVersion": V1, "kind": "Pod"}).encode(), "not an ExecCredential"),
    (json.dumps({"apiVersion": V1B1, "kind": "ExecCredential", "status": {"token": "t"}}).encode(),
     "plugin returned version"),
    (json.dumps({"apiVersion": V1, "kind": "ExecCredential"}).encode(), "didn't return a status"),
    (json.dumps({"apiVersion": V1, "kind": "ExecCredential", "status": {}}).encode(), "token or cert/key"),
    (json.dumps({"apiVersion": V1, "kind": "ExecCredential",
                 "status": {"token": "t", "clientCertificateData": "c"}}).encode(), "not both"),
    (json.dumps({"apiVersion": V1, "kind": "ExecCredential",
                 "status": {"token": "t", "expirationTimestamp": "soon"}}).encode(), "bad expirationTimestamp"),
])
def test_exec_output_validation(out, msg):
    p = ExecProvider(command="x", api_version=V1)
    with pytest.raises(ConfigError, match=msg):
        p.parse(out)


def test_exec_plugin_failures_are_config_errors():
    missing = ExecProvider(command="/nonexistent/kubelogin", api_version=V1, install_hint="brew install kubelogin")
    with pytest.raises(ConfigError, match="not found.*\n\nbrew install kubelogin"):
        missing.run()
    failing = ExecProvider(command=sys.executable, api_version=V1,
                           args=["-c", "import sys; sys.stderr.write('no creds'); sys.exit(3)"])
    with pytest.raises(ConfigError, match="exit code 3: no creds"):
        failing.run()


def test_auth_provider_still_rejected():
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "kc")
        doc = {"current-context": "c", "clusters": [{"name": "c", "cluster": {"server": "https://x"}}],
               "users": [{"name": "u", "user": {"auth-provider": {"name": "gcp"}}}],
               "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}]}
        with open(p, "w") as fh:
            yaml.safe_dump(doc, fh)
        with pytest.raises(ConfigError, match="auth-provider"):
            load_kubeconfig(p)


async def test_credential_expiring_during_retry_after_is_refreshed_off_the_loop():
    """A 429 with Retry-After, and the exec credential expires while the request waits it out:
    the retry refreshes the credential in a worker thread (never on the event-loop thread)
    and goes out with the new token."""
    import threading

    env = TestEnv()
    env.server.tokens = {"tok-1": {"username": "u"}, "tok-2": {"username": "u"}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "token"), "w") as fh:
            fh.write("tok-1")
        cfg = load_kubeconfig(_kubeconfig(d, f"http://127.0.0.1:{port}"))
        threads = []
        orig_run = cfg.exec_provider.run

        def run():
            threads.append(threading.current_thread())
            return orig_run()

        cfg.exec_provider.run = run
        c = Client(HttpTransport(cfg), qps=-1)
        try:
            with pytest.raises(errors.ApiError):
                await c.get(CM, "default", "x")  # first credential (tok-1)
            assert _runs(d) == 1
            env.server.faults.add(verb="get", resource="configmaps", code=429, reason="TooManyRequests",
                                  times=1, retry_after=1)
            with open(os.path.join(d, "token"), "w") as fh:
                fh.write("tok-2")
            loop = asyncio.get_running_loop()

            def rotate():  # during the Retry-After wait: tok-1 is revoked and its credential expires
                env.server.tokens = {"tok-2": {"username": "u"}}
                cfg._exec_creds.expires_at = 0.0

            loop.call_later(0.3, rotate)
            with pytest.raises(errors.ApiError) as e:
                await c.get(CM, "default", "x")
            assert e.value.code == 404  # retried with tok-2 (a stale tok-1 would be 401)
            assert _runs(d) == 2
            assert all(t is not threading.main_thread() for t in threads[1:]), threads
        finally:
            await c.close()
            await app.stop()

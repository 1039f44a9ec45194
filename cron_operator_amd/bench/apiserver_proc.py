"""Child-process fake apiserver for the benchmark (HTTP transport).

Prints ``LISTENING <url>`` once serving.  Uses a FakeClock the parent moves in
lockstep with the operator's clock through ``POST /debug/fake/clock``.

``--impl native`` (default): the C++ store and front end (``apiserver/native.py``,
``ops/csrc/apiserverd.cpp``) on a thread of its own, so the fixture stops bounding the
benchmark; ``--impl python``: :mod:`..apiserver.server` + :mod:`..apiserver.http` (the
envtest analog the test suite drives; also needed for ``--gc``).
"""
from __future__ import annotations

import argparse
import asyncio
import os
import signal

from ..api.v1alpha1.crd import crd
from ..apiserver.http import APIServerApp
from ..apiserver.server import APIServer
from ..trainingop.crds import kubeflow_crds
from ..utils.clock import FakeClock


async def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--start-ns", type=int, required=True)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--gc", action="store_true")
    ap.add_argument("--tls-dir", default="",
                    help="serve HTTPS with a self-signed certificate for CN=localhost written here "
                         "(tls.crt doubles as the client's CA)")
    ap.add_argument("--impl", choices=["native", "python"], default="native",
                    help="native: the C++ fake apiserver (_apiserverd); python: apiserver/server.py + http.py")
    ap.add_argument("--watch-window", type=int, default=200_000,
                    help="events per resource kept for watch resume (older resourceVersions answer 410)")
    a = ap.parse_args()
    if a.impl == "native" and not a.gc:
        await serve_native(a)
        return
    server = APIServer(FakeClock(a.start_ns), gc=a.gc, watch_window=a.watch_window)
    server.install_crd(crd())
    for c in kubeflow_crds():
        server.install_crd(c)
    app = APIServerApp(server)
    ctx = None
    if a.tls_dir:
        import ssl

        from ..runtime.servers import self_signed_cert

        cert, key = self_signed_cert(a.tls_dir, host="localhost")
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(cert, key)
    port = await app.start("127.0.0.1", a.port, ssl_context=ctx)
    print(f"LISTENING {'https' if ctx else 'http'}://127.0.0.1:{port}", flush=True)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    # exit if the parent goes away
    ppid = os.getppid()

    async def watchdog():
        while not stop.is_set():
            if os.getppid() != ppid:
                stop.set()
            await asyncio.sleep(1)

    dog = loop.create_task(watchdog())
    await stop.wait()
    dog.cancel()
    await app.stop()


async def serve_native(a: argparse.Namespace) -> None:
    from ..apiserver.native import NativeAPIServer

    srv = NativeAPIServer(a.start_ns, watch_window=a.watch_window)
    srv.install_crd(crd())
    for c in kubeflow_crds():
        srv.install_crd(c)
    cert = key = ""
    if a.tls_dir:
        from ..runtime.servers import self_signed_cert

        cert, key = self_signed_cert(a.tls_dir, host="localhost")
    port = srv.start("127.0.0.1", a.port, cert, key)
    print(f"LISTENING {'https' if cert else 'http'}://127.0.0.1:{port} native", flush=True)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    ppid = os.getppid()
    while not stop.is_set():  # exit if the parent goes away
        if os.getppid() != ppid:
            break
        try:
            await asyncio.wait_for(stop.wait(), 1.0)
        except asyncio.TimeoutError:
            pass
    srv.stop()


if __name__ == "__main__":
    prof = os.environ.get("CRON_BENCH_APISERVER_PROFILE")
    if prof:
        import cProfile

        cProfile.run("asyncio.run(main())", prof)
    else:
        asyncio.run(main())

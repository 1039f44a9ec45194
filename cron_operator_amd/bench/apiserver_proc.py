"""Child-process fake apiserver for the benchmark (HTTP transport).

Prints ``LISTENING <url>`` once serving.  Uses a FakeClock the parent moves in
lockstep with the operator's clock through ``POST /debug/fake/clock``.
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
    a = ap.parse_args()
    server = APIServer(FakeClock(a.start_ns), gc=a.gc)
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


if __name__ == "__main__":
    prof = os.environ.get("CRON_BENCH_APISERVER_PROFILE")
    if prof:
        import cProfile

        cProfile.run("asyncio.run(main())", prof)
    else:
        asyncio.run(main())

"""In-tree build of the native components.

``python -m cron_operator_amd.ops.build`` compiles every native extension next to
its Python wrapper (``cron_operator_amd/ops/_*.so``) so the artefacts travel with
the source tree (they are git-ignored, not gpurun-ignored).  Called by
``__graft_entry__.build()`` and lazily by the wrappers when a source file is
newer than its built library.

The operator is CPU control plane (no kernels, no
collectives), so the native pieces are host C++17 built with the system g++ and
linked against the running CPython's headers -- no hipcc involved.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import Dict, List

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"

# extension name -> sources
EXTENSIONS: Dict[str, List[str]] = {
    "_cron_engine": ["cron_engine.cpp"],
    "_fastjson": ["fastjson.cpp"],
    "_httpcodec": ["httpcodec.cpp"],
    "_netconn": ["netconn.cpp"],
    "_aioloop": ["aioloop.cpp"],
    "_promlite": ["promlite.cpp"],
    "_workqueue": ["workqueue.cpp"],
    "_apiserverd": ["apiserverd.cpp"],
}
# headers each extension includes (a change rebuilds it)
HEADERS: Dict[str, List[str]] = {
    "_httpcodec": ["httpframe.h"],
    "_netconn": ["httpframe.h"],
    "_apiserverd": ["jdom.h"],
}
# extra linker inputs: _netconn speaks TLS through the system OpenSSL and builds its own SSL_CTX
# (TlsContext); an ssl.SSLContext is used only when CPython's _ssl resolves to the same libssl
# (checked at configure() with dlopen/dlsym)
LIBS: Dict[str, List[str]] = {
    "_netconn": ["-lssl", "-lcrypto", "-ldl"],
    # the fake apiserver serves HTTPS itself (deployment-shaped runs) and runs its own thread
    "_apiserverd": ["-lssl", "-lcrypto", "-pthread"],
}


def ext_path(name: str) -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return HERE / f"{name}{suffix}"


def _compiler() -> str:
    for cand in (os.environ.get("CXX"), "g++", "c++", "clang++"):
        if cand and shutil.which(cand):
            return cand
    raise RuntimeError("no C++ compiler found (tried $CXX, g++, c++, clang++)")


def needs_build(name: str) -> bool:
    out = ext_path(name)
    if not out.exists():
        return True
    mtime = out.stat().st_mtime
    deps = EXTENSIONS[name] + HEADERS.get(name, [])
    return any((CSRC / s).stat().st_mtime > mtime for s in deps if (CSRC / s).exists())


def build_extension(name: str, force: bool = False, verbose: bool = False) -> Path:
    out = ext_path(name)
    srcs = [CSRC / s for s in EXTENSIONS[name]]
    missing = [str(s) for s in srcs if not s.exists()]
    if missing:
        raise FileNotFoundError(f"sources missing for {name}: {missing}")
    if not force and not needs_build(name):
        return out
    inc = sysconfig.get_paths()["include"]
    tmp = out.with_suffix(out.suffix + f".tmp{os.getpid()}")
    cmd = [
        _compiler(), "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
        "-Wall", "-Wno-missing-field-initializers", "-Wno-cast-function-type",
        f"-I{inc}", *map(str, srcs), "-o", str(tmp), *LIBS.get(name, []),
    ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"building {name} failed:\n{res.stderr}")
    os.replace(tmp, out)  # atomic: concurrent importers never see a half-written .so
    return out


def build_all(force: bool = False, verbose: bool = False) -> List[Path]:
    return [build_extension(n, force=force, verbose=verbose) for n in EXTENSIONS
            if all((CSRC / s).exists() for s in EXTENSIONS[n])]


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print(p)

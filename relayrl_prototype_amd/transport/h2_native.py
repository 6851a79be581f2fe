"""Loader of the native gRPC server module ``_h2grpc`` (csrc/net/h2grpc.cpp).

The module links nghttp2 as the image ships it (``/opt/conda/lib/libnghttp2.so.14``, which
depends on libc only).  It is built without an rpath -- a search path into /opt/conda/lib would
also resolve libstdc++ there, an older one than the process's -- so the library is preloaded
here by its full path (RTLD_GLOBAL), after which the module's DT_NEEDED entry resolves to it.
``load()`` returns the module, or None with the reason in ``ERROR`` (the gRPC transport then
serves with grpc.aio and says so)."""
from __future__ import annotations

import ctypes
import glob
import os
from typing import Optional

ERROR: Optional[str] = None
_MOD = None


def load():
    global ERROR, _MOD
    if _MOD is not None or ERROR is not None:
        return _MOD
    if os.environ.get("RRL_GRPC_NATIVE", "1") == "0":
        ERROR = "disabled by RRL_GRPC_NATIVE=0"
        return None
    prefix = os.environ.get("RRL_NGHTTP2_PREFIX", "/opt/conda")
    libs = sorted(glob.glob(os.path.join(prefix, "lib", "libnghttp2.so.*")))
    try:
        if libs:
            ctypes.CDLL(libs[0], mode=ctypes.RTLD_GLOBAL)
        from .. import _h2grpc  # noqa: F401

        _MOD = _h2grpc
    except (ImportError, OSError) as e:
        ERROR = f"{type(e).__name__}: {e}"
    return _MOD

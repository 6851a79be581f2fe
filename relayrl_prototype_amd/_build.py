"""In-tree build of the native extensions (no hipify, no JIT cache).

Two shared objects are produced next to this file:

* ``_hip_ops<EXT>``  -- the gfx950 HIP kernels (``csrc/kernels/*.hip``, compiled by
  ``hipcc --offload-arch=gfx950`` with a C ABI) linked with the PyTorch binding
  ``csrc/bindings/hip_ops.cpp`` (host compiler, PyTorch-ROCm headers).
* ``_native<EXT>``   -- the host runtime in C++ (``csrc/host/*.cpp``): safetensors /
  trajectory codec, ZMTP transport, vectorised CPU environments; pybind11 only.

The reference builds its native core with cargo + PyO3 (relayrl_framework/Cargo.toml,
build.rs); this is the MI355X-native equivalent.  Usage::

    python -m relayrl_prototype_amd._build            # build both
    python -m relayrl_prototype_amd._build --target native
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("RRL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

HIP_OPS = os.path.join(PKG_DIR, "_hip_ops" + EXT)
NATIVE = os.path.join(PKG_DIR, "_native" + EXT)
H2GRPC = os.path.join(PKG_DIR, "_h2grpc" + EXT)
# nghttp2 (HTTP/2 framing + HPACK) as the image ships it; the native gRPC server links it
NGHTTP2_PREFIX = os.environ.get("RRL_NGHTTP2_PREFIX", "/opt/conda")


def _jobs() -> int:
    env = os.environ.get("MAX_JOBS")
    if env and env.isdigit():
        return max(1, int(env))
    return max(1, min(8, os.cpu_count() or 1))


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, verbose):
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _py_includes():
    inc = [sysconfig.get_paths()["include"]]
    try:
        import pybind11

        inc.append(pybind11.get_include())
    except ImportError:  # pragma: no cover
        pass
    return inc


def _torch_flags():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [
        os.path.join(tdir, "include"),
        os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
    ]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM"]
    libdir = os.path.join(tdir, "lib")
    ldflags = [f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-ltorch_python", f"-Wl,-rpath,{libdir}"]
    return inc, cflags, ldflags


# Compiler flags for the HIP kernels: no SLP vectorisation -- packed f32 VALU (v_pk_fma_f32 /
# v_pk_mul_f32) beside MFMAs costs ~22 cycles more than two plain FMAs on gfx950, and the
# packed temporaries raised register pressure (spills in the value/policy-grad kernel).
HIP_FLAGS = ["-fno-slp-vectorize"]
FILE_FLAGS = {}


def build_hip(verbose=False, force=False) -> str:
    kdir = os.path.join(CSRC, "kernels")
    srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    headers = sorted(glob.glob(os.path.join(kdir, "*.h")))
    binding = os.path.join(CSRC, "bindings", "hip_ops.cpp")
    odir = os.path.join(BUILD, "hip")
    os.makedirs(odir, exist_ok=True)
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(odir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                         "-munsafe-fp-atomics", *HIP_FLAGS, *FILE_FLAGS.get(os.path.basename(s), []), "-I", kdir,
                         "-c", s,
                         "-o", o])
    # host runtime linked into this module: the host-env rollout driver (csrc/runtime) and the
    # env pools it steps from C++ (csrc/host/vecenv.cpp, a private copy: hidden symbols)
    hdir, rdir = os.path.join(CSRC, "host"), os.path.join(CSRC, "runtime")
    rt_headers = sorted(glob.glob(os.path.join(hdir, "*.h"))) + sorted(glob.glob(os.path.join(rdir, "*.h")))
    for s in sorted(glob.glob(os.path.join(rdir, "*.cpp"))) + [os.path.join(hdir, "vecenv.cpp")]:
        o = os.path.join(odir, "rt_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + rt_headers):
            jobs.append([CXX, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread",
                         "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", hdir, "-I", rdir, "-c", s, "-o", o])
    tinc, tcf, tld = _torch_flags()
    bindings = [binding] + sorted(b for b in glob.glob(os.path.join(CSRC, "bindings", "*_ops.cpp")) if b != binding)
    for bsrc in bindings:
        bo = os.path.join(odir, os.path.basename(bsrc) + ".o")
        objs.append(bo)
        if force or _newer(bo, [bsrc] + rt_headers):
            cmd = [CXX, "-O2", "-std=c++17", "-fPIC", "-DTORCH_EXTENSION_NAME=_hip_ops",
                   "-DTORCH_API_INCLUDE_EXTENSION_H", "-I/opt/rocm/include", "-I", hdir, "-I", rdir] + tcf
            for i in tinc + _py_includes():
                cmd += ["-I", i]
            cmd += ["-c", bsrc, "-o", bo]
            jobs.append(cmd)
    with cf.ThreadPoolExecutor(_jobs()) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or _newer(HIP_OPS, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread"] + objs + ["-o", HIP_OPS] + tld,
             verbose)
    return HIP_OPS


def build_native(verbose=False, force=False) -> str:
    hdir = os.path.join(CSRC, "host")
    srcs = sorted(glob.glob(os.path.join(hdir, "*.cpp"))) + [os.path.join(CSRC, "bindings", "native.cpp"),
                                                             os.path.join(CSRC, "bindings", "pickle_native.cpp")]
    headers = sorted(glob.glob(os.path.join(hdir, "*.h")))
    odir = os.path.join(BUILD, "native")
    os.makedirs(odir, exist_ok=True)
    objs, jobs = [], []
    for s in srcs:
        if not os.path.exists(s):
            continue
        o = os.path.join(odir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            cmd = [CXX, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread", "-I", hdir]
            for i in _py_includes():
                cmd += ["-I", i]
            cmd += ["-c", s, "-o", o]
            jobs.append(cmd)
    with cf.ThreadPoolExecutor(_jobs()) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if objs and (force or _newer(NATIVE, objs)):
        _run([CXX, "-shared", "-fPIC", "-pthread"] + objs + ["-o", NATIVE], verbose)
    return NATIVE


def build_h2(verbose=False, force=False):
    """``_h2grpc``: the native gRPC server (csrc/net/h2grpc.cpp) -- a module of its own because
    it links nghttp2; skipped (the transport falls back to grpc.aio) where nghttp2 is absent."""
    inc = os.path.join(NGHTTP2_PREFIX, "include")
    lib = os.path.join(NGHTTP2_PREFIX, "lib")
    if not os.path.exists(os.path.join(inc, "nghttp2", "nghttp2.h")) or not glob.glob(os.path.join(lib, "libnghttp2.so*")):
        print(f"[build] nghttp2 not found under {NGHTTP2_PREFIX}: _h2grpc skipped", flush=True)
        return None
    ndir = os.path.join(CSRC, "net")
    srcs = [os.path.join(ndir, "h2grpc.cpp"), os.path.join(CSRC, "bindings", "h2grpc_bind.cpp")]
    deps = srcs + [os.path.join(ndir, "h2grpc.h")]
    if not (force or _newer(H2GRPC, deps)):
        return H2GRPC
    cmd = [CXX, "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread", "-I", ndir, "-I", inc]
    for i in _py_includes():
        cmd += ["-I", i]
    # no rpath: a search path of /opt/conda/lib would also resolve libstdc++ there (an older one);
    # transport/h2_native.py preloads libnghttp2 (it needs libc only) by its full path instead
    cmd += srcs + [f"-L{lib}", "-lnghttp2", "-o", H2GRPC]
    _run(cmd, verbose)
    return H2GRPC


def build(targets=("native", "hip", "h2"), verbose=False, force=False):
    out = []
    if "native" in targets:
        out.append(build_native(verbose, force))
    if "h2" in targets:
        p = build_h2(verbose, force)
        if p:
            out.append(p)
    if "hip" in targets:
        out.append(build_hip(verbose, force))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", choices=["all", "hip", "native", "h2"], default="all")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    t = ("native", "hip", "h2") if a.target == "all" else (a.target,)
    for p in build(t, verbose=a.verbose, force=a.force):
        print(p)


if __name__ == "__main__":
    sys.exit(main())

"""Build libisg.so (all HIP kernels + C-ABI) in-tree for gfx950.

    python -m instancesegmentation_amd.build_lib      (or __graft_entry__.build())

hipcc cross-compiles on a CPU-only host; the resulting .so travels to the GPU box
with the repo snapshot (it is git-ignored, not gpurun-ignored).
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libisg.so")
SOURCES = ["conv_mfma.hip", "pw_gemm.hip", "tap_conv.hip", "tap_wgrad.hip", "thin_conv.hip", "halo_conv.hip", "wgrad.hip", "dw_convt.hip", "eltwise.hip", "maskops.hip", "infer_ops.hip", "kp_stem.hip", "down_conv.hip", "mask_head.hip", "api.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O2", "-fno-unroll-loops", "-std=c++17", "-fPIC", "-Wall",
         "-Wno-unused-function", "-Wno-pass-failed"]


_INCLUDE = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def _deps(src, seen=None):
    """`src` and every quoted header it includes, transitively (so an edit to stage.h,
    common.h or isg.h rebuilds exactly the objects that include it)."""
    seen = set() if seen is None else seen
    src = os.path.normpath(src)
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    with open(src, errors="replace") as f:
        text = f.read()
    for inc in _INCLUDE.findall(text):
        _deps(os.path.join(os.path.dirname(src), inc), seen)
    return seen


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in _deps(src))


def build(verbose=False, jobs=4):
    objdir = os.path.join(HERE, "build_obj")
    os.makedirs(objdir, exist_ok=True)
    procs = []
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        if _stale(obj, src):
            lang = ["-x", "hip"] if s.endswith(".cpp") else []
            cmd = [HIPCC] + FLAGS + lang + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            procs.append((s, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                              stderr=subprocess.STDOUT)))
            if len(procs) >= jobs:
                _wait(procs)
    _wait(procs)
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return LIB


def _wait(procs):
    err = None
    for name, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            err = f"hipcc failed on {name}:\n{out.decode(errors='replace')}"
    procs.clear()
    if err:
        raise RuntimeError(err)


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))

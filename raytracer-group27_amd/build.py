"""Build librt_amd.so in-tree: host C++ with g++, the HIP megakernel with hipcc for gfx950.

Every object is compiled with -ffp-contract=off (no FMA contraction) and without fast-math so
host and device arithmetic follow the reference's IEEE float/double op order bit for bit.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "librt_amd.so")

HOST_SRCS = ["obj_loader.cpp", "scene.cpp", "bvh_build.cpp", "rt_api_host.cpp", "bmp.cpp", "png_decode.cpp"]
HIP_SRCS = ["rt_runtime.hip", "rt_post.hip", "rt_build.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function"]


def _run(cmd):
    print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(src, obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def build(force=False, verbose_resource=False, defines=(), out=None):
    """defines / out (developer A/B builds, e.g. RT_MAX_LEAF=2): compiled into a separate object directory
    and library, the in-tree librt_amd.so untouched."""
    global BUILD, LIB
    if defines or out:
        tag = "_".join(d.replace("=", "") for d in defines) or "alt"
        BUILD = os.path.join(HERE, "build", "ab_" + tag)
        LIB = out or os.path.join(HERE, "build", f"lib_{tag}.so")
    extra_d = [f"-D{d}" for d in defines]
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))]
    headers.append(os.path.join(HERE, "..", "include", "rt_amd.h"))
    objs = []
    for s in HOST_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _stale(src, obj, headers):
            _run(["g++"] + COMMON + extra_d + ["-c", src, "-o", obj])
        objs.append(obj)
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _stale(src, obj, headers):
            extra = ["-Rpass-analysis=kernel-resource-usage"] if verbose_resource else []
            _run([HIPCC, "-x", "hip", f"--offload-arch={ARCH}"] + COMMON + extra_d + ["-Wno-unused-result",
                 "-Wno-unused-value"] + extra + ["-c", src, "-o", obj])
        objs.append(obj)
    if force or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        _run([HIPCC, "-shared", "-fPIC", "-o", LIB] + objs + ["-lz"])
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resource="--resource" in sys.argv,
          defines=[a[2:] for a in sys.argv[1:] if a.startswith("-D")])

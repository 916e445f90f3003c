"""Build librt_amd.so in-tree: host C++ with g++, the HIP megakernel with hipcc for gfx950.

Every object is compiled with -ffp-contract=off (no FMA contraction) and without fast-math so
host and device arithmetic follow the reference's IEEE float/double op order bit for bit.

Provenance: source_hash() is the SHA-256 of the sources the library is built from (csrc/, the C-ABI
header and this file, whose flags decide the code); the build compiles it into the library
(rt_source_hash, include/rt_amd.h), and build() rebuilds whenever the in-tree library's hash is not
the tree's, so the library that travels to the GPU box is the one of the committed sources.
"""
import concurrent.futures
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "librt_amd.so")

HOST_SRCS = ["obj_loader.cpp", "scene.cpp", "bvh_build.cpp", "rt_api_host.cpp", "bmp.cpp", "png_decode.cpp"]
HIP_SRCS = ["rt_runtime.hip", "rt_post.hip", "rt_build.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function"]
# HIP sources: every automatic variable defined at its declaration.  The kernels read no variable before writing it
# (the clang static analyzer, -Wuninitialized and the machine verifier find nothing), but their optimised IR keeps
# undef values on paths that do not use them, and the 4-wave recursion-tree build that faulted in rounds 4-5 ran the
# faulting C4 batch green once built this way (profiles/r06/fault/): no kernel is compiled with undefs
HIP_FLAGS = ["-ftrivial-auto-var-init=pattern"]


def _sources():
    """(name, path) of every file the library's code depends on, in a fixed order."""
    out = [("csrc/" + f, os.path.join(CSRC, f)) for f in sorted(os.listdir(CSRC))
           if f.endswith((".hip", ".cpp", ".h"))]
    out.append(("include/rt_amd.h", os.path.join(INCLUDE, "rt_amd.h")))
    out.append(("build.py", os.path.abspath(__file__)))
    return out


def _toolchain():
    """What besides the sources decides the code: the offload arch, the hipcc path and the ROCm release
    (read from /opt/rocm/.info/version, no subprocess), so a library built for another arch or toolchain
    does not pass for this tree's."""
    try:
        with open(os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(HIPCC))), ".info", "version")) as f:
            rel = f.read().strip()
    except OSError:
        rel = ""
    return f"arch={ARCH};hipcc={HIPCC};rocm={rel}"


def source_hash(defines=()):
    """SHA-256 (16 hex digits) of the library's sources: each file's name and bytes, then any -D defines,
    then the toolchain (_toolchain)."""
    h = hashlib.sha256()
    for name, path in _sources():
        with open(path, "rb") as f:
            data = f.read()
        h.update(name.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    for d in defines:
        h.update(b"-D" + d.encode() + b"\0")
    h.update(_toolchain().encode())
    return h.hexdigest()[:16]


def library_hash(path=None):
    """The source hash compiled into a built library, read from the file's bytes (the stamp string
    "RT_SOURCE_HASH:<16 hex>" that rt_source_hash returns from), so checking it loads nothing."""
    try:
        with open(path or LIB, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"RT_SOURCE_HASH:")
    if i < 0:
        return None
    return data[i + 15:i + 31].decode("ascii", "replace")


def _run(cmd):
    print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(src, obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def build(force=False, verbose_resource=False, defines=(), out=None, flags=()):
    """Build the library if its embedded source hash differs from the tree's (or force).
    defines / flags / out (developer A/B builds, e.g. RT_MAX_LEAF=2, or extra hipcc flags for the HIP sources):
    compiled into a separate object directory and library, the in-tree librt_amd.so untouched."""
    global BUILD, LIB
    if defines or flags or out:
        tag = "_".join([d.replace("=", "") for d in defines] +
                       ["".join(ch for ch in f if ch.isalnum()) for f in flags]) or "alt"
        BUILD = os.path.join(HERE, "build", "ab_" + tag)
        LIB = out or os.path.join(HERE, "build", f"lib_{tag}.so")
    want = source_hash(tuple(defines) + tuple("flag:" + f for f in flags))
    if not force and os.path.exists(LIB) and library_hash(LIB) == want:
        return LIB
    # the tree differs from what the library was built from: every object is rebuilt (no mtime trust)
    force = True
    extra_d = [f"-D{d}" for d in defines]
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))]
    headers.append(os.path.join(INCLUDE, "rt_amd.h"))
    jobs, objs = [], []
    for s in HOST_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _stale(src, obj, headers):
            jobs.append(["g++"] + COMMON + extra_d + ["-c", src, "-o", obj])
        objs.append(obj)
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        if force or _stale(src, obj, headers):
            extra = ["-Rpass-analysis=kernel-resource-usage"] if verbose_resource else []
            jobs.append([HIPCC, "-x", "hip", f"--offload-arch={ARCH}"] + COMMON + HIP_FLAGS + list(flags) + extra_d + ["-Wno-unused-result",
                        "-Wno-unused-value"] + extra + ["-c", src, "-o", obj])
        objs.append(obj)
    # the provenance stamp: one generated translation unit holding the source hash
    stamp = os.path.join(BUILD, "rt_source_hash.cpp")
    with open(stamp, "w") as f:
        f.write('#include <cstddef>\n#include <cstring>\n'
                # a whole, kept array (a static one may be emitted only from the part the copy reads)
                f'extern "C" __attribute__((used)) const char rt_source_stamp[] = "RT_SOURCE_HASH:{want}";\n'
                'extern "C" int rt_source_hash(char* buf, size_t len) {\n'
                '    const size_t n = sizeof(rt_source_stamp) - 15;  // the 16 digits and the NUL\n'
                '    if (!buf || len < n) return -1;\n'
                '    std::memcpy(buf, rt_source_stamp + 15, n);\n'
                '    return 0;\n}\n')
    jobs.append(["g++"] + COMMON + ["-c", stamp, "-o", stamp + ".o"])
    objs.append(stamp + ".o")
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(len(jobs), 8) or 1) as ex:
        for fut in [ex.submit(_run, j) for j in jobs]:
            fut.result()
    _run([HIPCC, "-shared", "-fPIC", "-o", LIB] + objs + ["-lz"])
    got = library_hash(LIB)
    if got != want:
        raise RuntimeError(f"built {LIB} reports source hash {got}, expected {want}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resource="--resource" in sys.argv,
          defines=[a[2:] for a in sys.argv[1:] if a.startswith("-D")],
          flags=[a[2:] for a in sys.argv[1:] if a.startswith("-F")])

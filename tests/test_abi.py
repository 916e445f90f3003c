"""The C-ABI library loads, exports exactly what include/rt_amd.h declares, and fails loudly
(no CPU fallback) where there is no GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "rt_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|long)\s+(rt_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_every_binding(R):
    assert header_functions() == sorted(R.EXPORTS)


def test_library_exports_every_symbol(R):
    L = R.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    # raw dlsym through a fresh handle as well
    raw = ctypes.CDLL(R.LIB_PATH)
    for name in header_functions():
        getattr(raw, name)


def test_abi_version_and_struct_sizes(R):
    assert R.lib().rt_abi_version() == 5
    assert ctypes.sizeof(R.rt_stats) == 112
    assert ctypes.sizeof(R.rt_material) == 40
    assert ctypes.sizeof(R.rt_ray) == 28
    assert ctypes.sizeof(R.rt_hit) == 52
    assert ctypes.sizeof(R.rt_params) == 80
    assert ctypes.sizeof(R.rt_texture) == 24


def test_library_built_from_this_tree(R):
    """Provenance: the source hash compiled into the library (rt_source_hash) is the hash of this tree's
    sources (build.py source_hash), and the file stamp build.py reads agrees with the C-ABI call."""
    import build

    p = R.provenance(strict=False)
    assert p["match"], p
    assert build.library_hash(R.LIB_PATH) == p["library_source_hash"]


def test_library_reads_no_environment(R):
    """Render paths are chosen by the scene and explicit context options (rt_ctx_set_option), never
    by environment variables: the library imports no getenv / secure_getenv."""
    import subprocess

    nm = subprocess.run(["nm", "-D", "--undefined-only", R.LIB_PATH], capture_output=True, text=True, check=True)
    assert not re.search(r"\b(secure_)?getenv\b", nm.stdout)


def test_no_cpu_fallback_without_gpu(R):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the -m gpu tests")
    s = R.Scene()
    s.load_obj(os.path.join(R.data_dir(), "cube.obj"))
    with pytest.raises(R.RtError, match="no HIP device"):
        R.Context(s)


def test_error_reporting(R):
    s = R.Scene()
    with pytest.raises(R.RtError, match="does not exist"):
        s.load_obj("/nonexistent/file.obj")


def test_camera_matches_oracle_bitwise(R, O):
    for W, H in [(256, 256), (1920, 1080), (3840, 2160), (7, 3)]:
        cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
        mine = np.array(list(cam.position) + list(cam.quat) + [cam.half_height, cam.half_width], np.float32)
        ref = O.Oracle.camera((0, 0, 0), R.default_euler(), 3.0, R.default_fovy(), R.aspect_of(W, H))
        assert mine.tobytes() == ref.tobytes()


def test_ipc_export_of_2gib_refused(R):
    """rt_ipc_alloc refuses buffers of 2 GiB or more before touching a device (this ROCm's importing
    hipIpcOpenMemHandle never returns for them: 2 145 386 496 B maps, 2 147 483 648 B hangs, tools/ipc_probe.py
    --bytes), so an exporter can fall back to the gather exchange instead of hanging its importers."""
    for nbytes in (2 ** 31, 3 * 2 ** 30):
        with pytest.raises(R.RtError, match="2 GiB or more"):
            R.IpcBuffer(0, nbytes=nbytes)

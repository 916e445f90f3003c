"""The C++ facade (include/rt_facade.hpp) compiles against the C-ABI and drives it the way the
reference's main.cpp drives BoundingVolumeHierarchy / getFinalColor / renderRayTracing."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_example(tmp_path):
    exe = str(tmp_path / "facade_example")
    lib_dir = os.path.join(REPO, "raytracer-group27_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "facade_example.cpp"), "-L", lib_dir, "-lrt_amd",
                    f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True)
    return exe


def test_facade_builds_and_fails_loudly_without_gpu(R, tmp_path):
    import torch

    exe = build_example(tmp_path)
    if torch.cuda.is_available():
        pytest.skip("GPU present: see test_facade_runs_on_gpu")
    r = subprocess.run([exe, R.data_dir()], capture_output=True, text=True)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "no HIP device" in r.stdout


@pytest.mark.gpu
def test_facade_runs_on_gpu(R, tmp_path):
    exe = build_example(tmp_path)
    bmp = str(tmp_path / "render.bmp")
    r = subprocess.run([exe, R.data_dir(), bmp], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hit=1" in r.stdout and "frame_sum=" in r.stdout
    assert "views_identical=3/3" in r.stdout, r.stdout
    data = open(bmp, "rb").read()
    assert data[:2] == b"BM" and len(data) == 54 + 32 * 3 * 24

"""Developer tool: median kernel ms of configs with a given build of librt_amd.so, so two builds
can be compared on one GPU box (run once per library, alternating).
Usage: python tools/ab_lib.py path/to/librt_amd.so C3 C5"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

R.LIB_PATH = os.path.abspath(sys.argv[1])


class _Lenient(R.C.CDLL):  # an older build lacks newer entry points: bind those to None
    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return R.C.CFUNCTYPE(R.C.c_int)(lambda: -1)


R.C.CDLL = _Lenient
for cfg in sys.argv[2:]:
    s, p, W, H, _ = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    ctx.render(cam, p, W, H)
    ms = [ctx.render(cam, p, W, H)[1].kernel_ms for _ in range(int(os.environ.get("AB_ROUNDS", "5")))]
    print(f"{os.path.basename(os.path.dirname(R.LIB_PATH))} {cfg} median {np.median(ms):.3f} ms", flush=True)
    ctx.close()

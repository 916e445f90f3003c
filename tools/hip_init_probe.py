"""Probe (developer tool): rt_create and torch both see the device whatever the order of
`import rt_amd` / R.lib() / torch CUDA use.  python tools/hip_init_probe.py ORDER
(ORDER: lib-torch | torch-lib | lib-only)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
order = sys.argv[1]
import rt_amd as R  # noqa: E402

if order == "torch-lib":
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
R.lib()
if order == "lib-torch":
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
scene, prm, W, H, _ = R.build_config("C2")
try:
    ctx = R.Context(scene, device=0)
    print(order, "rt_create ok", flush=True)
except Exception as e:  # noqa: BLE001
    print(order, "rt_create FAILED", e, flush=True)
    sys.exit(1)
if order != "lib-only":
    import torch
    x = torch.ones(4, device="cuda")
    print(order, "torch tensor ok", float(x.sum()), flush=True)

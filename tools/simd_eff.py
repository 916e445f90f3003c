"""Developer tool: SIMD efficiency of the persistent kernels from the counting build.
Per config and variant: lane node visits / (64 x wave node steps), same for triangle records
and for state-machine advances (one per query).  Usage: python tools/simd_eff.py C3 whole:1=1 df:1=2
(variant name : rt_ctx_set_option key=value pairs, e.g. 1=2 selects the dynamic-fetch kernel)
SE_VIEWS=V renders a turntable batch of V views in one launch (rt_render_views_device) instead of one frame."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

args = sys.argv[1:]
if "--lib" in args:  # another build of the library (A/B of builds)
    i = args.index("--lib")
    R.LIB_PATH = os.path.abspath(args[i + 1])
    del args[i:i + 2]
cfgs = [a for a in args if a.startswith("C") and ":" not in a] or ["C3"]
variants = [(a.split(":", 1)[0], dict(x.split("=") for x in a.split(":", 1)[1].split(",") if x))
            for a in args if ":" in a] or [("default", {})]
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    V = int(os.environ.get("SE_VIEWS", "1"))
    if V > 1:
        import torch
        cams = R.turntable_cameras(V, R.aspect_of(W, H))
        buf = torch.zeros(V * R.local_band_elems(W, H, 8, 1), dtype=torch.float32, device="cuda")
    for name, env in variants:
        for k, v in {R.OPT_KERNEL: 0, R.OPT_VARIANT: -1, R.OPT_COOP: -1, R.OPT_COOP_MAX: 0, R.OPT_REFILL: 0, R.OPT_FAN: 1, R.OPT_INTERLEAVE: -1, R.OPT_FAN_CAP: 0, R.OPT_DUAL_STEP: -1}.items():
            ctx.set_option(k, v)
        for k, v in env.items():
            ctx.set_option(int(k), int(v))
        R.set_counting(True)
        if V > 1:
            st = ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
        else:
            _, st = ctx.render(cam, p, W, H)
        R.set_counting(False)
        c = ctx.debug_counters(58)
        rays, nodes, tris, hits, wn, wt, wa = (int(x) for x in c[:7])
        print(f"{cfg} {name}: rays={rays} nodes/ray={nodes / rays:.2f} tris/ray={tris / rays:.2f} "
              f"eff_node={nodes / max(1, 64 * wn):.3f} eff_tri={tris / max(1, 64 * wt):.3f} "
              f"eff_adv={rays / max(1, 64 * wa):.3f} wave_steps/ray: node={wn / rays:.3f} tri={wt / rays:.3f} "
              f"adv={wa / rays:.3f} cycA={int(c[8]) / max(1, int(c[8]) + int(c[9])):.2f} "
              f"(advance {int(c[10]) / max(1, int(c[8])):.2f}, job fetch {int(c[11]) / max(1, int(c[8])):.2f}) "
              f"iterations by tracing lanes 1-16/17-32/33-64: "
              f"{[round(int(c[k]) / max(1, sum(int(c[j]) for j in (13, 14, 15))), 3) for k in (13, 14, 15)]} "
              f"revisits/ray={int(c[16]) / rays:.3f} (share of visits {int(c[16]) / max(1, nodes):.3f}, "
              f"popped slots/revisit {int(c[17]) / max(1, int(c[16])):.2f}, still hit {int(c[18]) / max(1, int(c[16])):.2f}) "
              f"ref_slab/ray={int(c[19]) / rays:.3f} wave ref_slab/ray={int(c[20]) / rays:.4f} "
              f"lane iterations/ray={int(c[23]) / rays:.2f} (node + record {int(c[22]) / max(1, int(c[23])):.3f}, "
              f"held to a record with a node to visit {int(c[21]) / max(1, int(c[23])):.3f}) (opaque kernel)",
              flush=True)
        if int(c[53]):  # the opaque kernel's camera queries that hit nothing: their share of the visits
            print(f"{cfg} {name}: camera misses ({int(c[27])} queries): node visits {int(c[53])} "
                  f"({int(c[53]) / max(1, nodes):.3f} of all), records {int(c[54])} ({int(c[54]) / max(1, tris):.3f}), "
                  f"{int(c[53]) / max(1, int(c[27])):.2f} nodes per miss", flush=True)
        if int(c[50]) + int(c[51]) + int(c[52]):  # the tree kernel's phase A in parts (share of all wave cycles)
            tot = max(1, int(c[8]) + int(c[9]))
            print(f"{cfg} {name}: phase A parts: finished samples / segments {int(c[50]) / tot:.3f}, owners resuming "
                  f"{int(c[51]) / tot:.3f}, fan hand-out {int(c[52]) / tot:.3f} (of all wave cycles)", flush=True)
    ctx.close()

import sys, time, os
sys.path.insert(0,'raytracer-group27_amd'); sys.path.insert(0,'oracle')
import numpy as np
import rt_amd as R, oracle as O
for name, W, H in [('C1',64,64),('C2',64,48)]:
    s, p, _, _, desc = R.build_config(name)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W,H))
    ctx = R.Context(s)
    print(name, ctx.info())
    img, st = ctx.render(cam, p, W, H)
    ref, rays = O.Oracle(s).render(p, W, H)
    d = np.abs(img-ref)
    print(name, 'rays gpu', st.rays, 'oracle', rays, 'Linf', d.max(), 'nbad', int((d>1e-5).sum()), 'ms', st.kernel_ms)

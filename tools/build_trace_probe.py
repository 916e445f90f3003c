import sys; sys.path.insert(0, "raytracer-group27_amd")
import rt_amd as R
R.LIB_PATH = sys.argv[1]
s, p, W, H, d = R.build_config("C3")
for i in range(3):
    c = R.Context(s); print(sys.argv[1], [round(x, 1) for x in c.create_ms()], c.build_info(), flush=True); c.close()

import sys, os, numpy as np
sys.path[:0] = ["/root/repo/3d-ray-tracer-vulkan_amd", "/root/repo"]
from rtamd import configs
k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = configs.get(k)
b = cfg.build()
cam = cfg.camera()
d = f"/tmp/sim/cfg{k}"
os.makedirs(d, exist_ok=True)
np.asarray(b.model_vertex_data).tofile(d + "/verts.bin")
np.asarray(b.model_material_data).tofile(d + "/mats.bin")
np.asarray(b.flat_bvh_data).tofile(d + "/nodes.bin")
open(d + "/cam.bin", "wb").write(bytes(cam.ubo_bytes()))
open(d + "/meta.txt", "w").write(f"{cfg.width} {cfg.height} {cfg.max_bounces}\n")
print(cfg.name, os.path.getsize(d + "/verts.bin"), os.path.getsize(d + "/nodes.bin"))

"""Root-entry depth on the accel walk's CPU model (analysis aid, not part of
the product): orc_accel_root(d) enters the first d records of a
layout's leftmost path without their slab test (the kernel: d = 1); per-pixel,
per-bounce visits from the model's profile, lockstep wave steps of 16 x 4
tiles (the most records any alive lane walks per bounce).  Config 5 samples
rows 1000-1539 (its top rows are sky).
Usage: root_depth_model.py CONFIG
"""
import sys, numpy as np, ctypes as C
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, '3d-ray-tracer-vulkan_amd'), ROOT]
from rtamd import configs, _lib
from oracle import oracle_lib as O
k=int(sys.argv[1])
cfg=configs.get(k); b=cfg.build()
rec,info=_lib.accel_records(b,8)
args=(b.model_vertex_data,b.model_material_data,b.flat_bvh_data,cfg.camera().ubo_bytes(),cfg.width,cfg.height,cfg.max_bounces)
tile=(0,1000,cfg.width,540) if k==5 else None
L=O.lib(accel=True)
for d in (0,1,2,3):
    L.orc_accel_root(d)
    rgba,rad,c,prof=O.render_accel(*args,rec,info,profile=True,tile=tile)
    vis=(prof & 0xFFFFF).astype(np.int64)
    alive=vis>0
    steps=np.where(alive, vis - d, 0)    # records walked (the first d counted, not walked)
    H,W,B=steps.shape
    T=steps[:H//4*4,:W//16*16].reshape(H//4,4,W//16,16,B)
    ws=T.max(axis=(1,3)).sum()
    print('config',k,'depth',d,'visits',int(vis.sum()),'lane steps',int(steps.sum()),'wave steps',int(ws))
L.orc_accel_root(1)

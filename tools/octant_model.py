"""Fewer of the 8 layouts walked on the accel walk's CPU model (analysis aid;
DESIGN.md §5, option accel_octants): orc_accel_octants(mask) keeps the octant
bits of mask when choosing a ray's layout; wave steps of 16 x 4 tiles as in
root_depth_model.py.
Usage: octant_model.py CONFIG
"""
import sys, numpy as np
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
base=None
for mask in (7,3,5,6,1,2,4,0):
    L.orc_accel_octants(mask)
    rgba,rad,c,prof=O.render_accel(*args,rec,info,profile=True,tile=tile)
    vis=(prof & 0xFFFFF).astype(np.int64)
    steps=np.where(vis>0, vis-1, 0)
    H,W,B=steps.shape
    ws=steps[:H//4*4,:W//16*16].reshape(H//4,4,W//16,16,B).max(axis=(1,3)).sum()
    base=base or ws
    print('config',k,'mask',mask,'layouts',2**bin(mask).count('1'),'lane steps',int(steps.sum()),'wave steps',int(ws),'%.3f'%(ws/base))
L.orc_accel_octants(7)

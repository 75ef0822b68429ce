"""Workgroup-local compaction of the paths still alive between bounces, on
the accel walk's CPU model (analysis aid, not part of the product).  From the
model's per-pixel, per-bounce node visits (oracle/rt_accel_model.c profile),
16 x 4 wave tiles in groups of G consecutive tiles: the lockstep wave steps of
the kernel as built (each wave alone, the most visits of its alive lanes per
bounce), of the group's alive paths packed into waves of 64 in lane order,
and of the same with the per-bounce barrier such an exchange needs (every
active wave of the group lives as long as the group's slowest wave).
Usage: compact_model.py CONFIG [G]   
"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, '3d-ray-tracer-vulkan_amd'), ROOT]
from rtamd import configs, _lib
from oracle import oracle_lib as O
k=int(sys.argv[1]); G=int(sys.argv[2]) if len(sys.argv)>2 else 4
cfg=configs.get(k); b=cfg.build()
rec,info=_lib.accel_records(b,8)
args=(b.model_vertex_data,b.model_material_data,b.flat_bvh_data,cfg.camera().ubo_bytes(),cfg.width,cfg.height,cfg.max_bounces)
tile=None
if k==5: tile=(0,0,cfg.width,540)
rgba,rad,c,prof=O.render_accel(*args,rec,info,profile=True,tile=tile)
vis=(prof & 0xFFFFF).astype(np.int64)   # rows,w,B ; 0 = not alive in that bounce
H,W,B=vis.shape
# 16x4 tiles
T=vis[:H//4*4,:W//16*16].reshape(H//4,4,W//16,16,B).transpose(0,2,1,3,4).reshape(-1,64,B)  # tiles x 64 lanes x B
base=T.max(axis=1).sum()
# groups of G consecutive tiles (raster within a row of tiles)
n=T.shape[0]//G*G
Tg=T[:n].reshape(-1,G*64,B)
comp=0; bar=0
for g in range(Tg.shape[0]):
    for bb in range(B):
        v=Tg[g,:,bb]; a=v[v>0]
        if a.size==0: continue
        # pack in lane order into waves of 64
        mx=[a[i:i+64].max() for i in range(0,a.size,64)]
        comp+=sum(mx)
        bar+=len(mx)*max(mx)
lanes=T.sum()
print('config',k,'G',G,'wave steps base',int(base),'compacted',int(comp),'ratio %.3f'%(comp/base),'with barrier ratio %.3f'%(bar/base),'util base %.3f comp %.3f'%(lanes/(64*base), lanes/(64*comp)))

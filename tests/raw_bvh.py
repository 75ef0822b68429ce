"""Hand-built BVHs in the reference's flat layout (BVHFlattener.java:51-90 record format),
for shapes the reference's own builder never makes."""
import struct
from types import SimpleNamespace

import numpy as np


def raw_bvh_scene(n, shape, seed):
    """Triangles in front of the default camera under a hand-built BVH of the
    given shape: "left" = left-deep chain (right children are leaves), "right"
    = right-deep chain, "random" = random split points.  Any tree in the
    reference's preorder layout is a valid upload (VulkanEngine takes the
    buffer as is); deep chains overflow the walk's 8-entry t_enter stack."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-14, 14, (n, 1, 3))
    tv = (c + rng.uniform(-4, 4, (n, 3, 3))).astype(np.float32)
    mats = np.concatenate([rng.uniform(0.2, 0.9, (n, 3)), rng.integers(0, 3, (n, 1))], 1).astype(np.float32)
    lo, hi = tv.min(1), tv.max(1)

    def build(ids):
        if len(ids) == 1:
            return ids[0]
        if shape == "left":
            k = len(ids) - 1
        elif shape == "right":
            k = 1
        else:
            k = int(rng.integers(1, len(ids)))
        return (build(ids[:k]), build(ids[k:]))

    recs, order = [], []

    def rec(node):
        my = len(recs)
        recs.append(None)
        if isinstance(node, tuple):
            ids = []

            def leaves(x):
                if isinstance(x, tuple):
                    leaves(x[0]), leaves(x[1])
                else:
                    ids.append(x)
            leaves(node)
            bmin, bmax = lo[ids].min(0), hi[ids].max(0)
            li = rec(node[0])
            ri = rec(node[1])
            tail = struct.pack("<ii", li, ri)
        else:
            bmin, bmax = lo[node], hi[node]
            tail = struct.pack("<ii", -(len(order) + 1), -1)
            order.append(node)
        recs[my] = struct.pack("<4f4f", *bmin, 0.0, *bmax, 0.0) + tail + b"\0" * 8
        return my

    rec(build(list(range(n))))
    verts = np.zeros((n, 3, 4), np.float32)
    verts[:, :, :3] = tv[order]
    return SimpleNamespace(model_vertex_data=verts.reshape(-1), model_material_data=mats[order].reshape(-1),
                           flat_bvh_data=np.frombuffer(b"".join(recs), np.uint8).copy(), triangle_count=n)


def trailing_subtree_scene(first, second):
    """first's buffers with second's whole tree appended after the root's
    subtree: a valid upload (every node in preorder, every leaf's triangle in
    the buffers) whose trailing nodes the reference's DFS never reaches
    (compute_dynamic_ray.comp:185-210 starts at node 0 and stops when its
    stack is empty).  second's triangles follow first's in the vertex and
    material buffers."""
    n0 = len(first.flat_bvh_data) // 48
    t0 = len(first.model_vertex_data) // 12
    nodes = np.frombuffer(bytes(second.flat_bvh_data), np.uint8).copy().view(np.int32).reshape(-1, 12)
    leaf = nodes[:, 9] < 0
    nodes[leaf, 8] = nodes[leaf, 8] - t0                 # -(tri + 1) -> -(tri + t0 + 1)
    nodes[~leaf, 8] += n0
    nodes[~leaf, 9] += n0
    return SimpleNamespace(
        model_vertex_data=np.concatenate([np.asarray(first.model_vertex_data, np.float32).reshape(-1),
                                          np.asarray(second.model_vertex_data, np.float32).reshape(-1)]),
        model_material_data=np.concatenate([np.asarray(first.model_material_data, np.float32).reshape(-1),
                                            np.asarray(second.model_material_data, np.float32).reshape(-1)]),
        flat_bvh_data=np.concatenate([np.frombuffer(bytes(first.flat_bvh_data), np.uint8),
                                      nodes.view(np.uint8).reshape(-1)]),
        triangle_count=first.triangle_count + second.triangle_count)

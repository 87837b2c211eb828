"""Copies of a mesh scene's records with each group object's mesh moved in its own object
space, p -> s * p + X0, and the object's inverse adjusted (inv' = [s I | X0] inv), so the
world-space scene is the same up to rounding.  Used to check that the traversal index
keeps its quality for meshes far from the origin or larger than binary16's range
(ptmi_bvh.cpp root frame) and stays exact there (live-reference parity).

Triangle edges are recomputed from the moved vertices (e1 = p2 - p1, e2 = p3 - p1, as
the Go scene build does, shapes.go NewTriangle); vertex normals are left unchanged
(a uniform scale does not turn them).
"""
import numpy as np

from ptmi import layout


def moved(objs, tris, grps, offset=(0.0, 0.0, 0.0), scale=1.0):
    objs = objs.copy()
    tris = tris.copy()
    grps = grps.copy()
    x0 = np.array(list(offset) + [0.0], dtype=np.float64)
    s = float(scale)

    def pt(a):  # points (w = 1 or unused): s * p + X0 on x, y, z
        out = a.copy()
        out[..., :3] = a[..., :3] * s + x0[:3]
        return out

    for f in ("p1", "p2", "p3"):
        tris[f] = pt(tris[f])
    tris["e1"][..., :3] = tris["p2"][..., :3] - tris["p1"][..., :3]
    tris["e2"][..., :3] = tris["p3"][..., :3] - tris["p1"][..., :3]
    grps["bb_min"] = pt(grps["bb_min"])
    grps["bb_max"] = pt(grps["bb_max"])
    for o in objs:
        if int(o["type"]) != layout.TYPE_GROUP:
            continue
        o["bb_min"] = pt(o["bb_min"][None])[0]
        o["bb_max"] = pt(o["bb_max"][None])[0]
        a = np.eye(4)
        a[:3, :3] *= s
        a[:3, 3] = x0[:3]
        inv = a @ o["inverse"].reshape(4, 4)
        o["inverse"] = inv.reshape(16)
        o["inverse_transpose"] = inv.T.reshape(16)
        o["transform"] = np.linalg.inv(inv).reshape(16)
    return objs, tris, grps

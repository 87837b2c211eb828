"""Restatement of the reference's Wavefront OBJ/MTL reader (internal/app/obj/objparser.go)
for building the BVH benchmark scenes (teapot, gopher).

Documented deviations from the Go code (both are non-determinism / environment
fixes, not semantic changes):
  * groups are attached to the root in FILE order; Go iterates a map
    (objparser.go:208-214), which is randomised per run;
  * ``mtllib`` is resolved relative to the OBJ file; Go reads it relative to the
    process CWD (objparser.go:36).
"""
import os

import numpy as np

from . import geom, shapes


class Mtl:
    """material.Mtl (material/mtl.go)."""

    def __init__(self, name):
        self.name = name
        self.ambient = [0.0] * 4
        self.diffuse = [0.0] * 4
        self.specular = [0.0] * 4
        self.shininess = 0.0
        self.transparency = 0.0
        self.refractive_index = 0.0


def _pf(s):
    """strconv.ParseFloat with the error ignored (-> 0)."""
    try:
        return float(s)
    except ValueError:
        return 0.0


def _atoi(s):
    try:
        return int(s)
    except ValueError:
        return 0


def parse_mtl(data):
    """ParseMtl (objparser.go:225-273)."""
    out = {}
    current = None
    for row in data.split("\n"):
        if row.strip() == "":
            continue
        parts = row.strip().split()
        k = parts[0]
        if k == "newmtl":
            current = parts[1]
            out[current] = Mtl(current)
        elif k == "Ns":
            out[current].shininess = _pf(parts[1])
        elif k in ("Ka", "Kd", "Ks"):
            c = geom.color(_pf(parts[1]), _pf(parts[2]), _pf(parts[3]))
            setattr(out[current], {"Ka": "ambient", "Kd": "diffuse", "Ks": "specular"}[k], c)
        elif k == "Ni":
            out[current].refractive_index = _pf(parts[1])
        elif k == "d":
            out[current].transparency = 1 - _pf(parts[1])
    return out


def to_material(mtl):
    """toMaterial (objparser.go:180-190): color = Ka + Kd + Ks, w = 1."""
    m = shapes.Material(geom.tuple3(0, 0, 0), geom.tuple3(0, 0, 0), 0.0)
    r = mtl.ambient[0] + mtl.diffuse[0] + mtl.specular[0]
    g = mtl.ambient[1] + mtl.diffuse[1] + mtl.specular[1]
    b = mtl.ambient[2] + mtl.diffuse[2] + mtl.specular[2]
    m.color = geom.color(r, g, b)
    m.refractive_index = mtl.refractive_index
    return m


class Obj:
    def __init__(self):
        self.vertices = [geom.point(0, 0, 0)]
        self.normals = [geom.vector(0, 0, 0)]
        self.groups = {}
        self.ignored_lines = 0

    def to_group(self):
        """Obj.ToGroup (objparser.go:206-215), file order."""
        g = shapes.Group()
        g.label = "ROOT"
        for v in self.groups.values():
            g.add_child(v)
        return g


def parse_obj(data, base_dir="."):
    """ParseObj (objparser.go:13-135)."""
    out = Obj()
    mats = {}
    current = "DefaultGroup"
    current_material = shapes.new_default_material()
    out.groups[current] = shapes.Group()
    out.groups[current].label = current
    pending = {}  # group name -> list of triangles (added in bulk, same order)

    def flush(name):
        tris = pending.pop(name, None)
        if tris:
            out.groups[name].add_children(tris)

    for row in data.split("\n"):
        if row.strip() == "":
            out.ignored_lines += 1
            continue
        parts = row.strip().split()
        k = parts[0]
        if k == "mtllib":
            with open(os.path.join(base_dir, parts[1])) as f:
                mats = parse_mtl(f.read())
        elif k == "usemtl":
            current_material = to_material(mats[parts[1]])
            out.groups[current].set_material(current_material)
        elif k == "v":
            out.vertices.append(geom.point(_pf(parts[1]), _pf(parts[2]), _pf(parts[3])))
        elif k == "vn":
            out.normals.append(geom.vector(_pf(parts[1]), _pf(parts[2]), _pf(parts[3])))
        elif k == "f":
            lst = pending.setdefault(current, [])
            if "/" not in row:
                for i in range(2, len(parts) - 1):
                    lst.append(shapes.new_triangle_3p(out.vertices[_atoi(parts[1])],
                                                      out.vertices[_atoi(parts[i])],
                                                      out.vertices[_atoi(parts[i + 1])]))
            else:
                for i in range(2, len(parts) - 1):
                    s1, s2, s3 = parts[1].split("/"), parts[i].split("/"), parts[i + 1].split("/")
                    n1 = n2 = n3 = 0
                    if len(s1) == 3:
                        n1, n2, n3 = _atoi(s1[2]), _atoi(s2[2]), _atoi(s3[2])
                    tri = shapes.Triangle(out.vertices[_atoi(s1[0])], out.vertices[_atoi(s2[0])],
                                          out.vertices[_atoi(s3[0])], out.normals[n1],
                                          out.normals[n2], out.normals[n3])
                    tri.material = current_material
                    lst.append(tri)
        elif k in ("g", "o"):
            flush(current)
            current = parts[1]
            if current not in out.groups:
                out.groups[current] = shapes.Group()
                out.groups[current].label = parts[1]
        else:
            out.ignored_lines += 1
    for name in list(pending):
        flush(name)
    return out


def compute_vertex_normals(tris):
    """ComputeVertexNormals (objparser.go:137-178): O(n^2) fuzzy (0.01) vertex match,
    normals summed in triangle order, then geom.Normalize."""
    P = np.array([[t.p1, t.p2, t.p3] for t in tris], dtype=np.float64)  # (n,3,4)
    N = [t.n for t in tris]
    n = len(tris)
    new = []
    for i in range(n):
        res = []
        for k in range(3):
            p = P[i, k]
            close = np.all(np.abs(P - p) < 0.01, axis=2)  # (n,3): TupleEquals per vertex
            match = np.any(close, axis=1)
            match[i] = False
            acc = list(N[i])
            for j in np.nonzero(match)[0]:
                acc = geom.add(acc, N[j])
            res.append(geom.normalize(acc))
        new.append(res)
    for t, (a, b, c) in zip(tris, new):
        t.n1, t.n2, t.n3 = a, b, c

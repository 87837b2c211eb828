"""Adversarial BVH meshes for the parity tests (synthetic OBJ text fed through
ptmi's restatement of the Go scene pipeline: ParseObj, ComputeVertexNormals,
Divide(50), BuildCLGroup -- scenes.teapot_scene with obj_path).

They target the exactness arguments of the BVH path:
  * "flat"   -- a planar grid (z = 0): every reference node box has zero
                thickness, so the reference's line-box test (tmin < tmax) fails
                whenever the z slab binds; ptmi's own index finds those hits
                and must drop them through the exact gate check;
  * "stairs" -- axis-aligned faces sharing edges and vertices: rays through
                shared edges, boxes touching faces exactly;
  * "dupes"  -- every triangle listed twice: exact t ties between different
                triangle indices (tie-break by index, both gated);
  * "far"    -- "stairs" plus two small grids at x = +-1e5, past binary16's
                range: the traversal boxes above them carry +-infinity bounds
                (ptmi_bvh.cpp), which must stay conservative;
  * "big"    -- a 34,848-triangle tilted planar grid: more triangles than 16-bit
                child codes address, so the scene takes the wide codes and the generic
                instantiation with its 32-bit traversal stack;
  * "bumpy"  -- the same grid as a bumpy height field: lines along it meet up to ~200
                triangles, past the reference's 64-entry ctx arrays (tracer.cl:97-99;
                its kernel faults on this scene), so it is checked against the oracle
                only (pyoracle.max_candidates names the limit).
"""
import os
import tempfile

from ptmi import layout, scenes


def _grid(nx, ny, x0, y0, s, z, faces, verts, flip=False):
    base = len(verts)
    for j in range(ny + 1):
        for i in range(nx + 1):
            verts.append((x0 + i * s, y0 + j * s, z))
    for j in range(ny):
        for i in range(nx):
            a = base + j * (nx + 1) + i + 1
            b, c, d = a + 1, a + nx + 1, a + nx + 2
            faces += [(a, b, d), (a, d, c)] if not flip else [(a, d, b), (a, c, d)]


def obj_text(kind):
    verts, faces = [], []
    if kind == "far":
        text, _ = obj_text("stairs")
        for line in text.splitlines():
            if line.startswith("v "):
                verts.append(tuple(float(x) for x in line.split()[1:]))
            elif line.startswith("f "):
                faces.append(tuple(int(x) for x in line.split()[1:]))
        _grid(2, 2, 1.0e5, -1.0, 0.5, 0.0, faces, verts)
        _grid(2, 2, -1.0e5 - 1.0, -1.0, 0.5, -1.0, faces, verts)
    elif kind == "flat":
        _grid(24, 24, -6.0, -1.0, 0.5, 0.0, faces, verts)
    elif kind == "stairs":
        for k in range(8):  # step k: top (y = k/2 + 1/2) and riser (z = -k/2) faces, 4x4 quads each
            y, z = 0.5 * k, -0.5 * k
            base = len(verts)
            for j in range(5):
                for i in range(5):
                    verts.append((-4.0 + 2.0 * i, y + 0.5, z - 0.125 * j))  # tread
            for j in range(4):
                for i in range(4):
                    a = base + j * 5 + i + 1
                    faces += [(a, a + 1, a + 6), (a, a + 6, a + 5)]
            base = len(verts)
            for j in range(5):
                for i in range(5):
                    verts.append((-4.0 + 2.0 * i, y + 0.125 * j, z))  # riser
            for j in range(4):
                for i in range(4):
                    a = base + j * 5 + i + 1
                    faces += [(a, a + 1, a + 6), (a, a + 6, a + 5)]
    elif kind in ("big", "bumpy"):  # 34,848 triangles: child codes past 16 bits (32-bit stack)
        n = 132
        base = len(verts)
        for j in range(n + 1):
            for i in range(n + 1):
                x, y = -6.0 + 12.0 * i / n, -1.0 + 12.0 * j / n
                z = 0.25 * ((i * 7 + j * 13) % 5) / 4.0 if kind == "bumpy" else 0.05 * y - 0.5
                verts.append((x, y, z))
        for j in range(n):
            for i in range(n):
                a = base + j * (n + 1) + i + 1
                faces += [(a, a + 1, a + n + 2), (a, a + n + 2, a + n + 1)]
    elif kind == "dupes":
        _grid(12, 12, -6.0, -1.0, 1.0, 0.0, faces, verts)
        _grid(12, 12, -6.0, -1.0, 1.0, -2.0, faces, verts, flip=True)
        faces = faces + list(faces)  # every triangle twice
    else:
        raise ValueError(kind)
    lines = ["v %.17g %.17g %.17g" % v for v in verts]
    lines += ["g mesh"]
    lines += ["f %d %d %d" % f for f in faces]
    return "\n".join(lines) + "\n", len(faces)


def scene_inputs(kind, width, height, aperture=0.0, focal_length=0.0):
    """-> (objects, triangles, groups, camera) records of the adversarial scene."""
    text, _ = obj_text(kind)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "%s.obj" % kind)
        with open(p, "w") as f:
            f.write(text)
        sc = scenes.teapot_scene(width, height, aperture, focal_length, obj_path=p)
    objs, tris, grps = layout.build_scene_buffer_cl(sc.objects)
    return objs, tris, grps, layout.camera_record(sc.camera)

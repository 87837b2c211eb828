"""Restatement of the reference's scene-graph shapes (internal/app/shapes) and of its
BVH build (shapes/bvh.go), producing exactly the numbers Go would.

Only what feeds the kernel's input records is restated: transforms
(``SetTransform`` post-multiplies then inverts, sphere.go:60-64), materials,
bounding boxes (boundingbox.go) and ``Divide`` / ``PartitionChildren`` /
``MakeSubGroup`` / ``SplitBounds`` (bvh.go:8-119).

Bounding-box code follows Go's sequential ``Add`` semantics exactly (strict ``>`` /
``<`` compares, so NaN never enters and on ±0 ties the first value seen wins);
the per-triangle work is vectorised with numpy, whose elementwise float64 ops are
the same IEEE operations Go performs one by one.
"""
import numpy as np

from . import geom

INF = float("inf")


class Material:
    """material.Material (material/material.go:7-21)."""

    def __init__(self, color=None, emission=None, refractive_index=1.0, reflectivity=0.0):
        self.color = list(color) if color is not None else geom.tuple3(1, 1, 1)
        self.emission = list(emission) if emission is not None else geom.tuple3(0, 0, 0)
        self.refractive_index = float(refractive_index)
        self.reflectivity = float(reflectivity)
        self.textured = False
        self.texture_id = 0
        self.texture_scale_x = 0.0
        self.texture_scale_y = 0.0
        self.textured_nm = False
        self.texture_id_nm = 0
        self.texture_scale_x_nm = 0.0
        self.texture_scale_y_nm = 0.0
        self.is_env_map = False

    def copy(self):
        m = Material(self.color, self.emission, self.refractive_index, self.reflectivity)
        m.__dict__.update({k: v for k, v in self.__dict__.items() if k not in ("color", "emission")})
        return m


def new_default_material():
    return Material(geom.tuple3(1, 1, 1), geom.tuple3(0, 0, 0), 1.0)


def new_diffuse(r, g, b):
    return Material(geom.tuple3(r, g, b), geom.tuple3(0, 0, 0), 1.0)


def new_glass():
    return Material(geom.tuple3(1, 1, 1), geom.tuple3(0, 0, 0), 1.52, 0.05)


def new_mirror():
    return Material(geom.tuple3(1, 1, 1), geom.tuple3(0, 0, 0), 1.0, 1.0)


def new_light_bulb():
    return Material(geom.tuple3(1, 1, 1), geom.tuple3(8, 8, 8), 1.0)


class Basic:
    """shapes.Basic + the common SetTransform/SetMaterial methods."""
    TYPE = 999

    def __init__(self, material):
        self.label = ""
        self.transform = geom.identity()
        self.inverse = geom.identity()
        self.inverse_transpose = geom.identity()
        self.material = material

    def set_transform(self, m):
        self.transform = geom.multiply(self.transform, m)
        self.inverse = geom.inverse(self.transform)
        self.inverse_transpose = geom.transpose(self.inverse)

    def set_material(self, m):
        self.material = m


class Plane(Basic):
    TYPE = 0

    def __init__(self):  # plane.go:12-29 (RefractiveIndex 0 until SetMaterial)
        super().__init__(Material(geom.tuple3(0, .5, 1), geom.tuple3(0, 0, 0), 0.0))


class Sphere(Basic):
    TYPE = 1

    def __init__(self):  # sphere.go:15-31
        super().__init__(Material(geom.tuple3(1, .5, .5), geom.tuple3(0, 0, 0), 1.0))


class Cylinder(Basic):
    TYPE = 2

    def __init__(self, min_y=-INF, max_y=INF, closed=False):  # cylinder.go:10-41
        super().__init__(new_default_material())
        self.min_y = float(min_y)
        self.max_y = float(max_y)
        self.closed = closed


class Cube(Basic):
    TYPE = 3

    def __init__(self):  # cube.go:9-23
        super().__init__(new_default_material())


# ----------------------------------------------------------------------------
# Triangles live in one growable store so box math can be vectorised.
# ----------------------------------------------------------------------------

class Triangle:
    """shapes.Triangle (triangle.go).  Points/normals are 4-float lists."""
    TYPE = None

    def __init__(self, p1, p2, p3, n1=None, n2=None, n3=None, label="Triangle"):
        self.p1, self.p2, self.p3 = list(p1), list(p2), list(p3)
        self.e1 = geom.sub(self.p2, self.p1)
        self.e2 = geom.sub(self.p3, self.p1)
        self.n = geom.normalize(geom.cross(self.e2, self.e1))
        self.n1 = list(n1) if n1 is not None else list(self.n)
        self.n2 = list(n2) if n2 is not None else list(self.n)
        self.n3 = list(n3) if n3 is not None else list(self.n)
        self.material = new_default_material()
        self.label = label
        self.transform = geom.identity()


def new_triangle_3p(p1, p2, p3):
    return Triangle(p1, p2, p3, label="Triangle3P")


def new_triangle_n(p1, p2, p3):
    return Triangle(p1, p2, p3, label="TriangleN")


# ----------------------------------------------------------------------------
# Sequential min/max with Go's BoundingBox.Add semantics.
# ----------------------------------------------------------------------------

def _seq_min(vals, axis):
    """Go ``if cur > v { cur = v }`` starting from +Inf, along ``axis``."""
    m = np.fmin.reduce(vals, axis=axis)
    with np.errstate(invalid="ignore"):
        mask = vals == np.expand_dims(m, axis)
    idx = np.argmax(mask, axis=axis)
    out = np.take_along_axis(vals, np.expand_dims(idx, axis), axis=axis).squeeze(axis)
    return np.where(np.isnan(m), INF, out)


def _seq_max(vals, axis):
    m = np.fmax.reduce(vals, axis=axis)
    with np.errstate(invalid="ignore"):
        mask = vals == np.expand_dims(m, axis)
    idx = np.argmax(mask, axis=axis)
    out = np.take_along_axis(vals, np.expand_dims(idx, axis), axis=axis).squeeze(axis)
    return np.where(np.isnan(m), -INF, out)


def _box_of_points(pts):
    """NewEmptyBoundingBox then Add(p) for pts[..., k, 0:3] in order.
    Returns (...,2,4) with w = 1 (NewPoint)."""
    shp = pts.shape[:-2]
    out = np.empty(shp + (2, 4))
    out[..., 0, :3] = _seq_min(pts[..., :3], axis=-2)
    out[..., 1, :3] = _seq_max(pts[..., :3], axis=-2)
    out[..., :, 3] = 1.0
    return out


def _mul_by_tuple_np(m, pts):
    """geom.MultiplyByTuple vectorised over pts[..., 4] (matrix.go:51-61)."""
    m = np.asarray(m, dtype=np.float64).reshape(4, 4)
    out = np.empty_like(pts)
    with np.errstate(invalid="ignore"):
        for r in range(4):
            a = m[r, 0] * pts[..., 0]
            b = m[r, 1] * pts[..., 1]
            c = m[r, 2] * pts[..., 2]
            d = m[r, 3] * pts[..., 3]
            out[..., r] = ((a + b) + c) + d
    return out


def _transform_box_np(boxes, m):
    """TransformBoundingBox (boundingbox.go:72-94) over boxes[...,2,4]."""
    mn, mx = boxes[..., 0, :], boxes[..., 1, :]
    one = np.ones(mn.shape[:-1])

    def P(x, y, z):
        return np.stack([x, y, z, one], axis=-1)
    corners = np.stack([
        mn,
        P(mn[..., 0], mn[..., 1], mx[..., 2]),
        P(mn[..., 0], mx[..., 1], mn[..., 2]),
        P(mn[..., 0], mx[..., 1], mx[..., 2]),
        P(mx[..., 0], mn[..., 1], mn[..., 2]),
        P(mx[..., 0], mn[..., 1], mx[..., 2]),
        P(mx[..., 0], mx[..., 1], mn[..., 2]),
        mx,
    ], axis=-2)
    return _box_of_points(_mul_by_tuple_np(m, corners))


def _tri_points(tris):
    return np.array([[t.p1, t.p2, t.p3] for t in tris], dtype=np.float64).reshape(len(tris), 3, 4)


def _merge_into(box, boxes):
    """box.MergeWith(b) for b in boxes[n,2,4], in order (boundingbox.go:41-44):
    Add(b.Min) then Add(b.Max); the running Min/Max are the reductions' seeds."""
    pts = boxes.reshape(-1, 4)
    out = np.empty((2, 4))
    out[0, :3] = _seq_min(np.concatenate([box[0][None, :3], pts[:, :3]]), axis=0)
    out[1, :3] = _seq_max(np.concatenate([box[1][None, :3], pts[:, :3]]), axis=0)
    out[0, 3] = box[0][3]
    out[1, 3] = box[1][3]
    return out


def _empty_box():
    """NewEmptyBoundingBox (boundingbox.go:13-18)."""
    return np.array([[INF, INF, INF, 1.0], [-INF, -INF, -INF, 1.0]])


class Group:
    """shapes.Group (group.go) with its bounding box bookkeeping."""
    TYPE = 4

    def __init__(self):
        self.label = ""
        self.transform = geom.identity()
        self.inverse = geom.identity()
        self.inverse_transpose = geom.identity()
        self.material = Material(geom.tuple3(0, 0, 0), geom.tuple3(0, 0, 0), 0.0)  # zero Material{}
        self.children = []
        self.bbox = _empty_box()

    def set_transform(self, m):
        self.transform = geom.multiply(self.transform, m)
        self.inverse = geom.inverse(self.transform)
        self.inverse_transpose = geom.transpose(self.inverse)

    def set_material(self, m):
        self.material = m

    def add_child(self, s):
        self.add_children([s])

    def add_children(self, shapes):
        """AddChild per shape: append + BoundingBox.MergeWith(BoundsOf(s))."""
        if not shapes:
            return
        self.children.extend(shapes)
        self.bbox = _merge_into(self.bbox, _bounds_of_list(shapes))

    def bounds(self):
        """Group.Bounds(): BoundingBox = BoundsOf(g)."""
        self.bbox = bounds_of(self)


def _bounds_of_list(shapes):
    """BoundsOf(s) for each shape, in order -> (n,2,4)."""
    out = np.empty((len(shapes), 2, 4))
    tri_idx = [i for i, s in enumerate(shapes) if isinstance(s, Triangle)]
    if tri_idx:
        out[tri_idx] = _box_of_points(_tri_points([shapes[i] for i in tri_idx]))
    for i, s in enumerate(shapes):
        if isinstance(s, Triangle):
            continue
        out[i] = bounds_of(s)
    return out


def bounds_of_many(shapes):
    return _bounds_of_list(shapes)


def parent_space_bounds_list(shapes):
    """ParentSpaceBounds for each shape (boundingbox.go:67-70) -> (n,2,4)."""
    out = np.empty((len(shapes), 2, 4))
    tri_idx = [i for i, s in enumerate(shapes) if isinstance(s, Triangle)]
    if tri_idx:
        boxes = _box_of_points(_tri_points([shapes[i] for i in tri_idx]))
        out[tri_idx] = _transform_box_np(boxes, geom.identity())
    for i, s in enumerate(shapes):
        if isinstance(s, Triangle):
            continue
        out[i] = _transform_box_np(bounds_of(s)[None], s.transform)[0]
    return out


def bounds_of(s):
    """BoundsOf (boundingbox.go:96-116)."""
    if isinstance(s, Group):
        if not s.children:
            return _empty_box()
        return _merge_into(_empty_box(), parent_space_bounds_list(s.children))
    if isinstance(s, Triangle):
        return _box_of_points(_tri_points([s]))[0]
    return np.array([[-1.0, -1.0, -1.0, 1.0], [1.0, 1.0, 1.0, 1.0]])


def split_bounds(b):
    """SplitBounds (bvh.go:8-44)."""
    dx = b[1][0] - b[0][0]
    dy = b[1][1] - b[0][1]
    dz = b[1][2] - b[0][2]
    greatest = dx
    for v in (dy, dz):          # shapes.max (basic.go): strict '>' scan
        if v > greatest:
            greatest = v
    x0, y0, z0 = b[0][0], b[0][1], b[0][2]
    x1, y1, z1 = b[1][0], b[1][1], b[1][2]
    if greatest == dx:
        x0 = x0 + dx / 2.0
        x1 = x0
    elif greatest == dy:
        y0 = y0 + dy / 2.0
        y1 = y0
    else:
        z0 = z0 + dz / 2.0
        z1 = z0
    left = np.array([list(b[0]), [x1, y1, z1, 1.0]])
    right = np.array([[x0, y0, z0, 1.0], list(b[1])])
    return left, right


def _contains_box(b, cb):
    """BoundingBox.ContainsBox vectorised over cb[n,2,4]."""
    def cp(p):
        return ((b[0][0] <= p[:, 0]) & (b[0][1] <= p[:, 1]) & (b[0][2] <= p[:, 2]) &
                (b[1][0] >= p[:, 0]) & (b[1][1] >= p[:, 1]) & (b[1][2] >= p[:, 2]))
    return cp(cb[:, 0]) & cp(cb[:, 1])


def partition_children(g):
    """PartitionChildren (bvh.go:46-70)."""
    left = Group()
    right = Group()
    lb, rb = split_bounds(bounds_of(g))
    cbs = parent_space_bounds_list(g.children)
    in_left = _contains_box(lb, cbs)
    in_right = _contains_box(rb, cbs) & ~in_left
    left_list = [c for c, f in zip(g.children, in_left) if f]
    right_list = [c for c, f in zip(g.children, in_right) if f]
    remain = [c for c, fl, fr in zip(g.children, in_left, in_right) if not fl and not fr]
    left.add_children(left_list)
    right.add_children(right_list)
    g.children = remain
    g.bounds()
    left.bounds()
    right.bounds()
    return left, right


class _Counter:
    subgroup = 0


def reset_subgroup_counter():
    _Counter.subgroup = 0


def make_sub_group(g, shapes):
    """MakeSubGroup (bvh.go:74-84): label 'Subgroup N' from a process-global counter."""
    _Counter.subgroup += 1
    sg = Group()
    sg.material = g.material
    sg.label = "Subgroup %d" % _Counter.subgroup
    sg.add_children(shapes)
    g.add_child(sg)


def divide(s, threshold):
    """Divide (bvh.go:86-119)."""
    if not isinstance(s, Group):
        return
    if threshold <= len(s.children):
        left, right = partition_children(s)
        if left.children:
            make_sub_group(s, left.children)
        if right.children:
            make_sub_group(s, right.children)
    for c in list(s.children):
        divide(c, threshold)

"""The reference's own known-answer tests for the scene side (Go unit tests of the
code that builds the kernel's input records), run against both restatements:
  * the native C++ host side (pathtracer-ocl_amd/host, libptmi_host.so's sources):
    tests/host_kat/host_kat.cpp, built by __graft_entry__.build();
  * the Python mirror (pathtracer-ocl_amd/ptmi), below.
Sources of the known answers:
  geom/matrix_test.go:187-254          Inverse, multiply by inverse
  shapes/bvh_test.go:9-153             SplitBounds / PartitionChildren / MakeSubGroup / Divide
  obj/objparser_test.go:13-233         ParseObj, ParseMtl
  shapes/boundingbox_test.go:203-263   IntersectRayWithBox truth tables, re-derived for
                                       the kernel's box test (tracer.cl:250-280: EPSILON
                                       1e-4 instead of Go's 0.01) on the oracle's restatement
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
from ptmi import geom, objparser, shapes

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HOST_KAT = os.path.join(ROOT, "tests", "host_kat", "build", "host_kat")


def test_cpp_host_side_passes_reference_kats():
    if not os.path.exists(HOST_KAT):
        pytest.fail("tests/host_kat not built (run __graft_entry__.build())")
    r = subprocess.run([HOST_KAT], capture_output=True, text=True, timeout=60)
    lines = r.stdout.splitlines()
    assert len(lines) == 20 and all(l.startswith("PASS") for l in lines), r.stdout
    assert r.returncode == 0


def _in_epsilon(expected, actual, eps=0.01):  # assert.InEpsilon with geom.Epsilon
    expected, actual = np.asarray(expected), np.asarray(actual)
    return np.all(np.abs(expected - actual) / np.abs(expected) <= eps)


@pytest.mark.parametrize("m,expected", [
    ([-5, 2, 6, -8, 1, -5, 1, 8, 7, 7, -6, -7, 1, -3, 7, 4],
     [0.21805, 0.45113, 0.24060, -0.04511, -0.80827, -1.45677, -0.44361, 0.52068,
      -0.07895, -0.22368, -0.05263, 0.19737, -0.52256, -0.81391, -0.30075, 0.30639]),
    ([8, -5, 9, 2, 7, 5, 6, 1, -6, 0, 9, 6, -3, 0, -9, -4],
     [-0.15385, -0.15385, -0.28205, -0.53846, -0.07692, 0.12308, 0.02564, 0.03077,
      0.35897, 0.35897, 0.43590, 0.92308, -0.69231, -0.69231, -0.76923, -1.92308]),
    ([9, 3, 0, 9, -5, -2, -6, -3, -4, 9, 6, 4, -7, 6, 6, 2],
     [-0.04074, -0.07778, 0.14444, -0.22222, -0.07778, 0.03333, 0.36667, -0.33333,
      -0.02901, -0.14630, -0.10926, 0.12963, 0.17778, 0.06667, -0.26667, 0.33333]),
])
def test_inverse(m, expected):
    m = [float(v) for v in m]
    assert _in_epsilon(expected, geom.inverse(m))


def test_inverse_cofactors_and_determinant():
    m = [float(v) for v in (-5, 2, 6, -8, 1, -5, 1, 8, 7, 7, -6, -7, 1, -3, 7, 4)]
    assert geom._det4(m) == 532.0 and geom._cof4(m, 2, 3) == -160.0 and geom._cof4(m, 3, 2) == 105.0


def test_multiply_by_inverse():
    m1 = [float(v) for v in (3, -9, 7, 3, 3, -8, 2, -9, -4, 4, 4, 1, -6, 5, -1, 1)]
    m2 = [float(v) for v in (8, 2, 2, 2, 3, -1, 7, 0, 7, 0, 5, 4, 6, -2, 0, 5)]
    back = geom.multiply(geom.multiply(m1, m2), geom.inverse(m2))
    assert all(abs(a - b) < 0.01 for a, b in zip(back, m1))


def _box(x0, y0, z0, x1, y1, z1):
    return np.array([[x0, y0, z0, 1.0], [x1, y1, z1, 1.0]])


@pytest.mark.parametrize("box,lmax,rmin", [
    (_box(-1, -4, -5, 9, 6, 5), (4, 6, 5), (4, -4, -5)),
    (_box(-1, -2, -3, 9, 5.5, 3), (4, 5.5, 3), (4, -2, -3)),
    (_box(-1, -2, -3, 5, 8, 3), (5, 3, 3), (-1, 3, -3)),
    (_box(-1, -2, -3, 5, 3, 7), (5, 3, 2), (-1, -2, 2)),
])
def test_split_bounds(box, lmax, rmin):
    left, right = shapes.split_bounds(box)
    assert list(left[0]) == list(box[0]) and list(left[1]) == list(lmax) + [1.0]
    assert list(right[0]) == list(rmin) + [1.0] and list(right[1]) == list(box[1])


def _sphere(m=None):
    s = shapes.Sphere()
    if m is not None:
        s.set_transform(m)
    return s


def test_partition_children_of_group():
    s1, s2, s3 = _sphere(geom.translate(-2, 0, 0)), _sphere(geom.translate(2, 0, 0)), _sphere()
    g = shapes.Group()
    for s in (s1, s2, s3):
        g.add_child(s)
    g.bounds()
    left, right = shapes.partition_children(g)
    assert left.children == [s1] and right.children == [s2] and g.children == [s3]


def test_make_sub_group():
    s1, s2 = _sphere(), _sphere()
    g = shapes.Group()
    shapes.make_sub_group(g, [s1, s2])
    assert len(g.children) == 1 and isinstance(g.children[0], shapes.Group)
    assert g.children[0].children == [s1, s2]


def test_divide_primitive_does_nothing():
    s = _sphere()
    shapes.divide(s, 1)
    assert isinstance(s, shapes.Sphere)


def test_subdivide_group_partitions_its_children():
    s1, s2 = _sphere(geom.translate(-2, -2, 0)), _sphere(geom.translate(-2, 2, 0))
    s3 = _sphere(geom.scale(4, 4, 4))
    g = shapes.Group()
    g.add_children([s1, s2, s3])
    shapes.divide(g, 1)
    assert g.children[0] is s3
    sub = g.children[1]
    assert isinstance(sub, shapes.Group) and len(sub.children) == 2
    assert sub.children[0].children == [s1] and sub.children[1].children == [s2]


def test_divide_threshold_keeps_small_groups():  # bvh_test.go TestName
    s1, s2, s3 = _sphere(geom.translate(-2, 0, 0)), _sphere(geom.translate(2, 1, 0)), _sphere(geom.translate(2, -1, 0))
    subgr = shapes.Group()
    subgr.add_children([s1, s2, s3])
    s4 = _sphere()
    g = shapes.Group()
    g.add_children([subgr, s4])
    shapes.divide(g, 3)
    assert g.children[0] is subgr and g.children[1] is s4
    assert len(subgr.children) == 2
    assert subgr.children[0].children == [s1] and subgr.children[1].children == [s2, s3]


OBJ3 = "\nv -1 1 0\nv -1 0 0\nv 1 0 0\nv 1 1 0\n"


def test_parse_gibberish():
    data = ("There was a young lady named Bright\nwho traveled much faster than light.\nShe set out one day\n"
            "in a relative way,\nand came back the previous night.")
    assert objparser.parse_obj(data).ignored_lines == 5


def test_parse_vertices():
    o = objparser.parse_obj("\nv -1 1 0\nv -1.0000 0.5000 0.0000\nv 1 0 0\nv 1 1 0\n")
    assert [list(v) for v in o.vertices[1:]] == [[-1, 1, 0, 1], [-1, 0.5, 0, 1], [1, 0, 0, 1], [1, 1, 0, 1]]


def _pts(t):
    return [list(t.p1), list(t.p2), list(t.p3)]


@pytest.mark.parametrize("data,want", [
    (OBJ3 + "f 1 2 3\nf 1 3 4\n", [(1, 2, 3), (1, 3, 4)]),
    ("\nv -1 1 0\nv -1 0 0\nv 1 0 0\nv 1 1 0\nv 0 2 0\nf 1 2 3 4 5", [(1, 2, 3), (1, 3, 4), (1, 4, 5)]),
])
def test_parse_faces_and_polygons(data, want):
    o = objparser.parse_obj(data)
    g = o.groups["DefaultGroup"]
    assert [_pts(t) for t in g.children] == [[list(o.vertices[i]) for i in w] for w in want]


def test_triangles_in_groups():
    o = objparser.parse_obj(OBJ3 + "g FirstGroup\nf 1 2 3\ng SecondGroup\nf 1 3 4")
    t1, t2 = o.groups["FirstGroup"].children[0], o.groups["SecondGroup"].children[0]
    assert _pts(t1) == [list(o.vertices[i]) for i in (1, 2, 3)]
    assert _pts(t2) == [list(o.vertices[i]) for i in (1, 3, 4)]


def test_normal_data():
    o = objparser.parse_obj("\nvn 0 0 1\nvn 0.707 0 -0.707\nvn 1 2 3")
    assert [list(n) for n in o.normals[1:]] == [[0, 0, 1, 0], [0.707, 0, -0.707, 0], [1, 2, 3, 0]]


def test_faces_with_normals():
    o = objparser.parse_obj("\nv 0 1 0\nv -1 0 0\nv 1 0 0\nvn -1 0 0\nvn 1 0 0\nvn 0 1 0\n"
                            "f 1//3 2//1 3//2\nf 1/0/3 2/102/1 3/14/2")
    t1, t2 = o.groups["DefaultGroup"].children
    assert _pts(t1) == [list(o.vertices[i]) for i in (1, 2, 3)]
    assert [list(t1.n1), list(t1.n2), list(t1.n3)] == [list(o.normals[i]) for i in (3, 1, 2)]
    for a in ("p1", "p2", "p3", "e1", "e2", "n", "n1", "n2", "n3"):
        assert list(getattr(t1, a)) == list(getattr(t2, a)), a


def test_parse_gopher_materials():
    blocks = [("Body", "0.000000 0.429367 0.640000"), ("Eye-White", "0.800000 0.800000 0.800000"),
              ("Material", "0.640000 0.640000 0.640000"), ("Material.001", "0.000000 0.000000 0.000000"),
              ("NoseTop", "0.000000 0.000000 0.000000"), ("SkinColor", "0.609017 0.353452 0.144174"),
              ("Tooth", "0.640000 0.640000 0.640000")]
    data = "# Blender MTL File: 'gopher.blend'\n# Material Count: 7\n\n" + "\n".join(
        "newmtl %s\nNs 96.078431\nKa 0.000000 0.000000 0.000000\nKd %s\nKs 0.500000 0.500000 0.500000\n"
        "Ni 1.000000\nd 1.000000\nillum 2\n" % b for b in blocks)
    mats = objparser.parse_mtl(data)
    assert len(mats) == 7
    assert list(mats["Body"].diffuse[:3]) == [0.0, 0.429367, 0.64]


# shapes/boundingbox_test.go:203-263 -- (origin, direction, hit) for the unit cube and
# for the box (5,-2,0)-(11,4,7); directions normalised as the Go test does.
CUBE_CASES = [((5, 0.5, 0), (-1, 0, 0), True), ((-5, 0.5, 0), (1, 0, 0), True), ((0.5, 5, 0), (0, -1, 0), True),
              ((0.5, -5, 0), (0, 1, 0), True), ((0.5, 0, 5), (0, 0, -1), True), ((0.5, 0, -5), (0, 0, 1), True),
              ((0, 0.5, 0), (0, 0, 1), True), ((-2, 0, 0), (2, 4, 6), False), ((0, -2, 0), (6, 2, 4), False),
              ((0, 0, -2), (4, 6, 2), False), ((2, 0, 2), (0, 0, -1), False), ((0, 2, 2), (0, -1, 0), False),
              ((2, 2, 0), (-1, 0, 0), False)]
BOX_CASES = [((15, 1, 2), (-1, 0, 0), True), ((-5, -1, 4), (1, 0, 0), True), ((7, 6, 5), (0, -1, 0), True),
             ((9, -5, 6), (0, 1, 0), True), ((8, 2, 12), (0, 0, -1), True), ((6, 0, -5), (0, 0, 1), True),
             ((8, 1, 3.5), (0, 0, 1), True), ((9, -1, -8), (2, 4, 6), False), ((8, 3, -4), (6, 2, 4), False),
             ((9, -1, -2), (4, 6, 2), False), ((4, 0, 9), (0, 0, -1), False), ((8, 6, -1), (0, -1, 0), False),
             ((12, 5, 4), (-1, 0, 0), False)]


@pytest.mark.parametrize("mn,mx,cases", [((-1, -1, -1), (1, 1, 1), CUBE_CASES), ((5, -2, 0), (11, 4, 7), BOX_CASES)])
def test_kernel_box_test_truth_tables(mn, mx, cases):
    """The kernel's intersectRayWithBox (tracer.cl:270-280), as the oracle restates it,
    gives the Go truth table's answers: every direction component is 0 or well above
    both epsilons, so Go's 0.01 and the kernel's 1e-4 classify the axes alike."""
    if not pyoracle.cpu_available():
        pytest.skip("oracle not built")
    for o, d, want in cases:
        dn = geom.normalize(geom.vector(*d))
        assert pyoracle.ray_box((*o, 1.0), dn, mn, mx) == want, (o, d)

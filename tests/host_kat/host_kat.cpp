// host_kat.cpp -- TEST INFRASTRUCTURE: the reference's own known-answer tests for
// the scene side, run against the native C++ restatement (pathtracer-ocl_amd/host):
//   geom/matrix_test.go:187-254        Inverse (three matrices), multiply by inverse
//   shapes/bvh_test.go:9-153           SplitBounds, PartitionChildren, MakeSubGroup, Divide
//   obj/objparser_test.go:13-233       ParseObj: gibberish, vertices, faces, polygons,
//                                      groups, normals, faces with normals
// Go test identity checks (s.ID()) become pointer identity.  Prints one line per
// case and exits with the number of failures.  Built by tests/host_kat/Makefile.
#include <cmath>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../../pathtracer-ocl_amd/host/geom.h"
#include "../../pathtracer-ocl_amd/host/shapes.h"

using namespace ptmi_host;

namespace {

int failures = 0;
std::string g_detail;

bool check(bool c, const std::string& what) {
    if (!c && g_detail.empty()) g_detail = what;
    return c;
}

// assert.InEpsilon(expected, actual, Epsilon = 0.01): relative error
bool in_epsilon(double e, double a) { return std::fabs(e - a) / std::fabs(e) <= 0.01; }

bool tup_eq(const Tup& a, const Tup& b) { return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3]; }

bool inverse_case(const Mat& m, const Mat& expected) {
    const Mat inv = inverse(m);
    bool ok = true;
    for (int i = 0; i < 16; i++) ok = check(in_epsilon(expected[i], inv[i]), "index " + std::to_string(i)) && ok;
    return ok;
}

Box box(double x0, double y0, double z0, double x1, double y1, double z1) {  // NewBoundingBoxF
    Box b;
    b.mn = point(x0, y0, z0);
    b.mx = point(x1, y1, z1);
    return b;
}

bool split_case(const Box& b, const Tup& lmin, const Tup& lmax, const Tup& rmin, const Tup& rmax) {
    Box l, r;
    split_bounds(b, l, r);
    return check(tup_eq(l.mn, lmin) && tup_eq(l.mx, lmax) && tup_eq(r.mn, rmin) && tup_eq(r.mx, rmax), "split");
}

Shape* sphere_at(Arena& A, const Mat& m) {
    Shape* s = A.sphere();
    s->set_transform(m);
    return s;
}

const char* kObj3 = "\nv -1 1 0\nv -1 0 0\nv 1 0 0\nv 1 1 0\n";

}  // namespace

int main() {
    std::vector<std::pair<std::string, std::function<bool()>>> cases = {
        {"matrix_test.go:TestInverse",
         [] {
             const Mat m{-5, 2, 6, -8, 1, -5, 1, 8, 7, 7, -6, -7, 1, -3, 7, 4};
             return check(detail::det4(m.data()) == 532.0, "determinant") &&
                    check(detail::cof4(m.data(), 2, 3) == -160.0, "cofactor(2,3)") &&
                    check(detail::cof4(m.data(), 3, 2) == 105.0, "cofactor(3,2)") &&
                    inverse_case(m, {0.21805, 0.45113, 0.24060, -0.04511, -0.80827, -1.45677, -0.44361, 0.52068,
                                     -0.07895, -0.22368, -0.05263, 0.19737, -0.52256, -0.81391, -0.30075, 0.30639});
         }},
        {"matrix_test.go:TestInverse2",
         [] {
             return inverse_case({8, -5, 9, 2, 7, 5, 6, 1, -6, 0, 9, 6, -3, 0, -9, -4},
                                 {-0.15385, -0.15385, -0.28205, -0.53846, -0.07692, 0.12308, 0.02564, 0.03077,
                                  0.35897, 0.35897, 0.43590, 0.92308, -0.69231, -0.69231, -0.76923, -1.92308});
         }},
        {"matrix_test.go:TestInverse3",
         [] {
             return inverse_case({9, 3, 0, 9, -5, -2, -6, -3, -4, 9, 6, 4, -7, 6, 6, 2},
                                 {-0.04074, -0.07778, 0.14444, -0.22222, -0.07778, 0.03333, 0.36667, -0.33333,
                                  -0.02901, -0.14630, -0.10926, 0.12963, 0.17778, 0.06667, -0.26667, 0.33333});
         }},
        {"matrix_test.go:TestMultiplyByInverse",
         [] {
             const Mat m1{3, -9, 7, 3, 3, -8, 2, -9, -4, 4, 4, 1, -6, 5, -1, 1};
             const Mat m2{8, 2, 2, 2, 3, -1, 7, 0, 7, 0, 5, 4, 6, -2, 0, 5};
             const Mat back = multiply(multiply(m1, m2), inverse(m2));
             bool ok = true;
             for (int i = 0; i < 16; i++) ok = check(eq(back[i], m1[i]), "index " + std::to_string(i)) && ok;
             return ok;
         }},
        {"bvh_test.go:TestSplitPerfectCube",
         [] {
             return split_case(box(-1, -4, -5, 9, 6, 5), point(-1, -4, -5), point(4, 6, 5), point(4, -4, -5),
                               point(9, 6, 5));
         }},
        {"bvh_test.go:TestSplitXWideBoundingBox",
         [] {
             return split_case(box(-1, -2, -3, 9, 5.5, 3), point(-1, -2, -3), point(4, 5.5, 3), point(4, -2, -3),
                               point(9, 5.5, 3));
         }},
        {"bvh_test.go:TestSplitYWideBoundingBox",
         [] {
             return split_case(box(-1, -2, -3, 5, 8, 3), point(-1, -2, -3), point(5, 3, 3), point(-1, 3, -3),
                               point(5, 8, 3));
         }},
        {"bvh_test.go:TestSplitZWideBoundingBox",
         [] {
             return split_case(box(-1, -2, -3, 5, 3, 7), point(-1, -2, -3), point(5, 3, 2), point(-1, -2, 2),
                               point(5, 3, 7));
         }},
        {"bvh_test.go:TestPartitionChildrenOfGroup",
         [] {
             Arena A;
             Shape* s1 = sphere_at(A, translate(-2, 0, 0));
             Shape* s2 = sphere_at(A, translate(2, 0, 0));
             Shape* s3 = A.sphere();
             Shape* g = A.group();
             g->add_child(s1);
             g->add_child(s2);
             g->add_child(s3);
             g->bounds();
             Shape *l, *r;
             partition_children(A, g, l, r);
             return check(l->children.size() == 1 && l->children[0] == s1, "left") &&
                    check(r->children.size() == 1 && r->children[0] == s2, "right") &&
                    check(g->children.size() == 1 && g->children[0] == s3, "remaining");
         }},
        {"bvh_test.go:TestCreateSubGroupFromListOfChildren",
         [] {
             Arena A;
             Shape* s1 = A.sphere();
             Shape* s2 = A.sphere();
             Shape* g = A.group();
             make_sub_group(A, g, {s1, s2});
             return check(g->children.size() == 1 && g->children[0]->kind == GROUP, "one subgroup") &&
                    check(g->children[0]->children.size() == 2 && g->children[0]->children[0] == s1 &&
                              g->children[0]->children[1] == s2,
                          "subgroup children");
         }},
        {"bvh_test.go:TestDividePrimitiveDoesNothing",
         [] {
             Arena A;
             Shape* s = A.sphere();
             divide(A, s, 1);
             return check(s->kind == SPHERE && s->children.empty(), "still a sphere");
         }},
        {"bvh_test.go:TestSubdivideGroupPartitionsItsChildren",
         [] {
             Arena A;
             Shape* s1 = sphere_at(A, translate(-2, -2, 0));
             Shape* s2 = sphere_at(A, translate(-2, 2, 0));
             Shape* s3 = sphere_at(A, scale(4, 4, 4));
             Shape* g = A.group();
             g->add_child(s1);
             g->add_child(s2);
             g->add_child(s3);
             divide(A, g, 1);
             if (!check(g->children.size() == 2 && g->children[0] == s3, "g[0] = s3")) return false;
             Shape* sub = g->children[1];
             return check(sub->kind == GROUP && sub->children.size() == 2, "subgroup of 2") &&
                    check(sub->children[0]->kind == GROUP && sub->children[0]->children.size() == 1 &&
                              sub->children[0]->children[0] == s1,
                          "subgroup[0] = [s1]") &&
                    check(sub->children[1]->kind == GROUP && sub->children[1]->children.size() == 1 &&
                              sub->children[1]->children[0] == s2,
                          "subgroup[1] = [s2]");
         }},
        {"bvh_test.go:TestName",
         [] {
             Arena A;
             Shape* s1 = sphere_at(A, translate(-2, 0, 0));
             Shape* s2 = sphere_at(A, translate(2, 1, 0));
             Shape* s3 = sphere_at(A, translate(2, -1, 0));
             Shape* subgr = A.group();
             subgr->add_children({s1, s2, s3});
             Shape* s4 = A.sphere();
             Shape* g = A.group();
             g->add_children({subgr, s4});
             divide(A, g, 3);
             if (!check(g->children.size() == 2 && g->children[0] == subgr && g->children[1] == s4, "g = [subgr, s4]"))
                 return false;
             Shape* c1 = g->children[0];
             return check(c1->children.size() == 2, "child1 has 2") &&
                    check(c1->children[0]->children.size() == 1 && c1->children[0]->children[0] == s1, "[s1]") &&
                    check(c1->children[1]->children.size() == 2 && c1->children[1]->children[0] == s2 &&
                              c1->children[1]->children[1] == s3,
                          "[s2, s3]");
         }},
        {"objparser_test.go:TestParseGibberish",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A,
                                          "There was a young lady named Bright\nwho traveled much faster than light.\n"
                                          "She set out one day\nin a relative way,\nand came back the previous night.",
                                          ".");
             return check(m.ignored_lines == 5, "ignored " + std::to_string(m.ignored_lines));
         }},
        {"objparser_test.go:TestParseVerticies",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A, "\nv -1 1 0\nv -1.0000 0.5000 0.0000\nv 1 0 0\nv 1 1 0\n", ".");
             return check(m.vertices.size() == 5 && tup_eq(m.vertices[1], point(-1, 1, 0)) &&
                              tup_eq(m.vertices[2], point(-1, 0.5, 0)) && tup_eq(m.vertices[3], point(1, 0, 0)) &&
                              tup_eq(m.vertices[4], point(1, 1, 0)),
                          "vertices");
         }},
        {"objparser_test.go:TestParseTriangleFaces",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A, std::string(kObj3) + "f 1 2 3\nf 1 3 4\n", ".");
             const Shape* g = m.groups[0].second;
             if (!check(m.groups[0].first == "DefaultGroup" && g->children.size() == 2, "default group of 2"))
                 return false;
             const Shape *t1 = g->children[0], *t2 = g->children[1];
             return check(tup_eq(t1->p1, m.vertices[1]) && tup_eq(t1->p2, m.vertices[2]) &&
                              tup_eq(t1->p3, m.vertices[3]) && tup_eq(t2->p1, m.vertices[1]) &&
                              tup_eq(t2->p2, m.vertices[3]) && tup_eq(t2->p3, m.vertices[4]),
                          "faces");
         }},
        {"objparser_test.go:TestTriangulatePolygon",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A, "\nv -1 1 0\nv -1 0 0\nv 1 0 0\nv 1 1 0\nv 0 2 0\nf 1 2 3 4 5", ".");
             const Shape* g = m.groups[0].second;
             if (!check(g->children.size() == 3, "3 triangles")) return false;
             const int want[3][3] = {{1, 2, 3}, {1, 3, 4}, {1, 4, 5}};
             bool ok = true;
             for (int k = 0; k < 3; k++) {
                 const Shape* t = g->children[k];
                 ok = ok && tup_eq(t->p1, m.vertices[want[k][0]]) && tup_eq(t->p2, m.vertices[want[k][1]]) &&
                      tup_eq(t->p3, m.vertices[want[k][2]]);
             }
             return check(ok, "fan");
         }},
        {"objparser_test.go:TestTrianglesInGroups",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A, std::string(kObj3) + "g FirstGroup\nf 1 2 3\ng SecondGroup\nf 1 3 4", ".");
             const Shape *g1 = nullptr, *g2 = nullptr;
             for (const auto& kv : m.groups) {
                 if (kv.first == "FirstGroup") g1 = kv.second;
                 if (kv.first == "SecondGroup") g2 = kv.second;
             }
             if (!check(g1 && g2 && g1->children.size() == 1 && g2->children.size() == 1, "groups")) return false;
             const Shape *t1 = g1->children[0], *t2 = g2->children[0];
             return check(tup_eq(t1->p1, m.vertices[1]) && tup_eq(t1->p2, m.vertices[2]) &&
                              tup_eq(t1->p3, m.vertices[3]) && tup_eq(t2->p1, m.vertices[1]) &&
                              tup_eq(t2->p2, m.vertices[3]) && tup_eq(t2->p3, m.vertices[4]),
                          "faces");
         }},
        {"objparser_test.go:TestNormalData",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A, "\nvn 0 0 1\nvn 0.707 0 -0.707\nvn 1 2 3", ".");
             return check(m.normals.size() == 4 && tup_eq(m.normals[1], vector(0, 0, 1)) &&
                              tup_eq(m.normals[2], vector(0.707, 0, -0.707)) && tup_eq(m.normals[3], vector(1, 2, 3)),
                          "normals");
         }},
        {"objparser_test.go:TestFacesWithNormals",
         [] {
             Arena A;
             const ObjModel m = parse_obj(A,
                                          "\nv 0 1 0\nv -1 0 0\nv 1 0 0\nvn -1 0 0\nvn 1 0 0\nvn 0 1 0\n"
                                          "f 1//3 2//1 3//2\nf 1/0/3 2/102/1 3/14/2",
                                          ".");
             const Shape* g = m.groups[0].second;
             if (!check(g->children.size() == 2, "2 triangles")) return false;
             const Shape *t1 = g->children[0], *t2 = g->children[1];
             const bool first = tup_eq(t1->p1, m.vertices[1]) && tup_eq(t1->p2, m.vertices[2]) &&
                                tup_eq(t1->p3, m.vertices[3]) && tup_eq(t1->n1, m.normals[3]) &&
                                tup_eq(t1->n2, m.normals[1]) && tup_eq(t1->n3, m.normals[2]);
             // reflect.DeepEqual(*t1, *t2): every geometric field equal
             const bool same = tup_eq(t1->p1, t2->p1) && tup_eq(t1->p2, t2->p2) && tup_eq(t1->p3, t2->p3) &&
                               tup_eq(t1->e1, t2->e1) && tup_eq(t1->e2, t2->e2) && tup_eq(t1->n, t2->n) &&
                               tup_eq(t1->n1, t2->n1) && tup_eq(t1->n2, t2->n2) && tup_eq(t1->n3, t2->n3);
             return check(first, "t1 points / normals") && check(same, "t1 == t2");
         }},
    };
    for (auto& c : cases) {
        g_detail.clear();
        bool ok = false;
        try {
            ok = c.second();
        } catch (const std::exception& e) {
            g_detail = e.what();
        }
        std::printf("%s %s%s%s\n", ok ? "PASS" : "FAIL", c.first.c_str(), ok ? "" : ": ", ok ? "" : g_detail.c_str());
        failures += ok ? 0 : 1;
    }
    return failures;
}

// shapes.cpp -- scene graph, bounding boxes, BVH Divide and the OBJ/MTL reader
// (see shapes.h for the reference files restated).
#include "shapes.h"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace ptmi_host {

Shape* Arena::make(Kind k) {
    shapes.emplace_back();
    Shape* s = &shapes.back();
    s->kind = k;
    return s;
}
Shape* Arena::plane() {
    Shape* s = make(PLANE);
    s->material = new_material(tuple3(0, .5, 1), tuple3(0, 0, 0), 0.0);
    return s;
}
Shape* Arena::sphere() {
    Shape* s = make(SPHERE);
    s->material = new_material(tuple3(1, .5, .5), tuple3(0, 0, 0), 1.0);
    return s;
}
Shape* Arena::cylinder(double min_y, double max_y, bool closed) {  // cylinder.go:10-41
    Shape* s = make(CYLINDER);
    s->material = new_default_material();
    s->min_y = min_y, s->max_y = max_y, s->closed = closed;
    return s;
}
Shape* Arena::cube() {  // cube.go:9-23
    Shape* s = make(CUBE);
    s->material = new_default_material();
    return s;
}
Shape* Arena::group() {
    Shape* s = make(GROUP);
    s->material = new_material(tuple3(0, 0, 0), tuple3(0, 0, 0), 0.0);
    return s;
}
// triangle.go: e1 = p2 - p1, e2 = p3 - p1, n = Normalize(Cross(e2, e1)); vertex
// normals default to n.
Shape* Arena::triangle(const Tup& p1, const Tup& p2, const Tup& p3, const Tup* n1, const Tup* n2, const Tup* n3) {
    Shape* s = make(TRIANGLE);
    s->p1 = p1, s->p2 = p2, s->p3 = p3;
    s->e1 = sub(p2, p1);
    s->e2 = sub(p3, p1);
    s->n = normalize(cross(s->e2, s->e1));
    s->n1 = n1 ? *n1 : s->n;
    s->n2 = n2 ? *n2 : s->n;
    s->n3 = n3 ? *n3 : s->n;
    s->material = new_default_material();
    return s;
}

void Shape::add_child(Shape* s) {  // AddChild: append + BoundingBox.MergeWith(BoundsOf(s))
    children.push_back(s);
    bbox.merge(bounds_of(s));
}
void Shape::bounds() { bbox = bounds_of(this); }

// TransformBoundingBox (boundingbox.go:72-94): the 8 corners in this order,
// each through MultiplyByTuple, added to an empty box.
static Box transform_box(const Box& b, const Mat& m) {
    const Tup& mn = b.mn;
    const Tup& mx = b.mx;
    const Tup corners[8] = {mn,
                            point(mn[0], mn[1], mx[2]),
                            point(mn[0], mx[1], mn[2]),
                            point(mn[0], mx[1], mx[2]),
                            point(mx[0], mn[1], mn[2]),
                            point(mx[0], mn[1], mx[2]),
                            point(mx[0], mx[1], mn[2]),
                            mx};
    Box out;
    for (const Tup& c : corners) out.add(multiply_by_tuple(m, c));
    return out;
}

Box parent_space_bounds(const Shape* s) {  // boundingbox.go:67-70
    return transform_box(bounds_of(s), s->kind == TRIANGLE ? identity() : s->transform);
}

Box bounds_of(const Shape* s) {  // BoundsOf (boundingbox.go:96-116)
    Box b;
    if (s->kind == GROUP) {
        for (const Shape* c : s->children) b.merge(parent_space_bounds(c));
        return b;
    }
    if (s->kind == TRIANGLE) {
        b.add(s->p1);
        b.add(s->p2);
        b.add(s->p3);
        return b;
    }
    b.mn = point(-1, -1, -1);
    b.mx = point(1, 1, 1);
    return b;
}

// SplitBounds (bvh.go:8-44)
void split_bounds(const Box& b, Box& left, Box& right) {
    const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    double greatest = dx;  // shapes.max (basic.go): strict '>' scan
    if (dy > greatest) greatest = dy;
    if (dz > greatest) greatest = dz;
    double x0 = b.mn[0], y0 = b.mn[1], z0 = b.mn[2];
    double x1 = b.mx[0], y1 = b.mx[1], z1 = b.mx[2];
    if (greatest == dx) {
        x0 = x0 + dx / 2.0;
        x1 = x0;
    } else if (greatest == dy) {
        y0 = y0 + dy / 2.0;
        y1 = y0;
    } else {
        z0 = z0 + dz / 2.0;
        z1 = z0;
    }
    left.mn = b.mn;
    left.mx = point(x1, y1, z1);
    right.mn = point(x0, y0, z0);
    right.mx = b.mx;
}

static bool contains_point(const Box& b, const Tup& p) {
    return b.mn[0] <= p[0] && b.mn[1] <= p[1] && b.mn[2] <= p[2] && b.mx[0] >= p[0] && b.mx[1] >= p[1] &&
           b.mx[2] >= p[2];
}
static bool contains_box(const Box& b, const Box& c) { return contains_point(b, c.mn) && contains_point(b, c.mx); }

// PartitionChildren (bvh.go:46-70)
void partition_children(Arena& A, Shape* g, Shape*& left, Shape*& right) {
    left = A.group();
    right = A.group();
    Box lb, rb;
    split_bounds(bounds_of(g), lb, rb);
    std::vector<Shape*> ll, rl, remain;
    for (Shape* c : g->children) {
        const Box cb = parent_space_bounds(c);
        if (contains_box(lb, cb))
            ll.push_back(c);
        else if (contains_box(rb, cb))
            rl.push_back(c);
        else
            remain.push_back(c);
    }
    left->add_children(ll);
    right->add_children(rl);
    g->children = remain;
    g->bounds();
    left->bounds();
    right->bounds();
}

// MakeSubGroup (bvh.go:74-84)
void make_sub_group(Arena& A, Shape* g, const std::vector<Shape*>& v) {
    A.subgroup_counter++;
    Shape* sg = A.group();
    sg->material = g->material;
    sg->label = "Subgroup " + std::to_string(A.subgroup_counter);
    sg->add_children(v);
    g->add_child(sg);
}

void divide(Arena& A, Shape* s, size_t threshold) {  // Divide (bvh.go:86-119)
    if (s->kind != GROUP) return;
    if (threshold <= s->children.size()) {
        Shape *left, *right;
        partition_children(A, s, left, right);
        if (!left->children.empty()) make_sub_group(A, s, left->children);
        if (!right->children.empty()) make_sub_group(A, s, right->children);
    }
    const std::vector<Shape*> kids = s->children;
    for (Shape* c : kids) divide(A, c, threshold);
}

// ---- OBJ / MTL --------------------------------------------------------------

static std::vector<std::string> fields(const std::string& row) {
    std::istringstream is(row);
    std::vector<std::string> out;
    std::string w;
    while (is >> w) out.push_back(w);
    return out;
}
// strconv.ParseFloat / Atoi with the error ignored (-> 0).
static double pf(const std::string& s) {
    if (s.empty()) return 0.0;
    char* end = nullptr;
    errno = 0;
    const double v = std::strtod(s.c_str(), &end);
    return (end && *end == '\0') ? v : 0.0;
}
static long atoi0(const std::string& s) {
    if (s.empty()) return 0;
    char* end = nullptr;
    const long v = std::strtol(s.c_str(), &end, 10);
    return (end && *end == '\0') ? v : 0;
}
static std::vector<std::string> split_slash(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    while (true) {
        const size_t b = s.find('/', a);
        out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
    }
    return out;
}
static std::string trim(const std::string& s) {
    const size_t a = s.find_first_not_of(" \t\r\n\v\f");
    if (a == std::string::npos) return "";
    const size_t b = s.find_last_not_of(" \t\r\n\v\f");
    return s.substr(a, b - a + 1);
}

struct Mtl {  // material.Mtl (material/mtl.go)
    Tup ambient{}, diffuse{}, specular{};
    double shininess = 0, transparency = 0, refractive_index = 0;
};

static std::map<std::string, Mtl> parse_mtl(const std::string& data) {  // ParseMtl (objparser.go:225-273)
    std::map<std::string, Mtl> out;
    std::string current;
    std::istringstream is(data);
    std::string row;
    while (std::getline(is, row)) {
        if (trim(row).empty()) continue;
        const auto p = fields(row);
        const std::string& k = p[0];
        if (k == "newmtl") {
            current = p.at(1);
            out[current] = Mtl();
        } else if (k == "Ns") {
            out.at(current).shininess = pf(p.at(1));
        } else if (k == "Ka" || k == "Kd" || k == "Ks") {
            const Tup c = color(pf(p.at(1)), pf(p.at(2)), pf(p.at(3)));
            Mtl& m = out.at(current);
            (k == "Ka" ? m.ambient : k == "Kd" ? m.diffuse : m.specular) = c;
        } else if (k == "Ni") {
            out.at(current).refractive_index = pf(p.at(1));
        } else if (k == "d") {
            out.at(current).transparency = 1 - pf(p.at(1));
        }
    }
    return out;
}

static Material to_material(const Mtl& m) {  // toMaterial (objparser.go:180-190)
    Material out = new_material(tuple3(0, 0, 0), tuple3(0, 0, 0), 0.0);
    const double r = m.ambient[0] + m.diffuse[0] + m.specular[0];
    const double g = m.ambient[1] + m.diffuse[1] + m.specular[1];
    const double b = m.ambient[2] + m.diffuse[2] + m.specular[2];
    out.color = color(r, g, b);
    out.refractive_index = m.refractive_index;
    return out;
}

Shape* ObjModel::to_group(Arena& A) const {  // Obj.ToGroup (objparser.go:206-215), file order
    Shape* g = A.group();
    g->label = "ROOT";
    for (const auto& kv : groups) g->add_child(kv.second);
    return g;
}

ObjModel parse_obj(Arena& A, const std::string& data, const std::string& base_dir) {  // ParseObj (objparser.go:13-135)
    ObjModel out;
    std::map<std::string, Mtl> mats;
    std::map<std::string, Shape*> by_name;
    auto get_group = [&](const std::string& name) {
        auto it = by_name.find(name);
        if (it != by_name.end()) return it->second;
        Shape* g = A.group();
        g->label = name;
        by_name[name] = g;
        out.groups.push_back({name, g});
        return g;
    };
    std::string current = "DefaultGroup";
    Material current_material = new_default_material();
    get_group(current);
    auto vtx = [&](long i) -> const Tup& {
        if (i < 0 || (size_t)i >= out.vertices.size()) throw std::out_of_range("OBJ vertex index out of range");
        return out.vertices[(size_t)i];
    };
    auto nrm = [&](long i) -> const Tup& {
        if (i < 0 || (size_t)i >= out.normals.size()) throw std::out_of_range("OBJ normal index out of range");
        return out.normals[(size_t)i];
    };
    std::istringstream is(data);
    std::string row;
    while (std::getline(is, row)) {
        if (trim(row).empty()) {
            out.ignored_lines++;
            continue;
        }
        const auto p = fields(row);
        const std::string& k = p[0];
        if (k == "mtllib") {
            std::ifstream f(base_dir + "/" + p.at(1));
            if (!f) throw std::runtime_error("cannot read mtllib " + p.at(1));
            std::stringstream ss;
            ss << f.rdbuf();
            mats = parse_mtl(ss.str());
        } else if (k == "usemtl") {
            current_material = to_material(mats.at(p.at(1)));
            get_group(current)->set_material(current_material);
        } else if (k == "v") {
            out.vertices.push_back(point(pf(p.at(1)), pf(p.at(2)), pf(p.at(3))));
        } else if (k == "vn") {
            out.normals.push_back(vector(pf(p.at(1)), pf(p.at(2)), pf(p.at(3))));
        } else if (k == "f") {
            Shape* g = get_group(current);
            if (row.find('/') == std::string::npos) {
                for (size_t i = 2; i + 1 < p.size(); i++)
                    g->add_child(A.triangle(vtx(atoi0(p[1])), vtx(atoi0(p[i])), vtx(atoi0(p[i + 1]))));
            } else {
                for (size_t i = 2; i + 1 < p.size(); i++) {
                    const auto s1 = split_slash(p[1]), s2 = split_slash(p[i]), s3 = split_slash(p[i + 1]);
                    long n1 = 0, n2 = 0, n3 = 0;
                    if (s1.size() == 3) n1 = atoi0(s1[2]), n2 = atoi0(s2[2]), n3 = atoi0(s3[2]);
                    Shape* t = A.triangle(vtx(atoi0(s1[0])), vtx(atoi0(s2[0])), vtx(atoi0(s3[0])), &nrm(n1),
                                          &nrm(n2), &nrm(n3));
                    t->material = current_material;
                    g->add_child(t);
                }
            }
        } else if (k == "g" || k == "o") {
            current = p.at(1);
            get_group(current);
        } else {
            out.ignored_lines++;
        }
    }
    // strings.Split(data, "\n") also yields the empty row after a final newline
    if (data.empty() || data.back() == '\n') out.ignored_lines++;
    return out;
}

// ComputeVertexNormals (objparser.go:137-178): for every vertex of every
// triangle, its face normal plus the face normals of all OTHER triangles with a
// vertex TupleEquals-close (0.01) to it, in triangle order, then Normalize.
// Candidates come from a 0.01-grid hash (cells within +-2 cover the fuzzy match
// even when the cell division rounds); the sum still runs over matching
// triangles in increasing index.
void compute_vertex_normals(const std::vector<Shape*>& tris) {
    const size_t n = tris.size();
    std::vector<Tup> face(n);
    for (size_t i = 0; i < n; i++) face[i] = tris[i]->n;
    auto key = [](const Tup& p) {
        return std::array<long long, 3>{(long long)std::floor(p[0] / 0.01), (long long)std::floor(p[1] / 0.01),
                                        (long long)std::floor(p[2] / 0.01)};
    };
    std::map<std::array<long long, 3>, std::vector<uint32_t>> grid;
    bool hashable = true;
    for (size_t i = 0; i < n && hashable; i++)
        for (const Tup* p : {&tris[i]->p1, &tris[i]->p2, &tris[i]->p3}) {
            if (!std::isfinite((*p)[0]) || !std::isfinite((*p)[1]) || !std::isfinite((*p)[2]) ||
                std::fabs((*p)[0]) > 1e12 || std::fabs((*p)[1]) > 1e12 || std::fabs((*p)[2]) > 1e12) {
                hashable = false;
                break;
            }
            auto& v = grid[key(*p)];
            if (v.empty() || v.back() != i) v.push_back((uint32_t)i);
        }
    std::vector<std::array<Tup, 3>> res(n);
    std::vector<uint32_t> cand;
    for (size_t i = 0; i < n; i++) {
        const Tup* pts[3] = {&tris[i]->p1, &tris[i]->p2, &tris[i]->p3};
        for (int k = 0; k < 3; k++) {
            const Tup& p = *pts[k];
            cand.clear();
            if (hashable) {
                const auto c = key(p);
                for (long long dx = -2; dx <= 2; dx++)
                    for (long long dy = -2; dy <= 2; dy++)
                        for (long long dz = -2; dz <= 2; dz++) {
                            auto it = grid.find({c[0] + dx, c[1] + dy, c[2] + dz});
                            if (it != grid.end()) cand.insert(cand.end(), it->second.begin(), it->second.end());
                        }
                std::sort(cand.begin(), cand.end());
                cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
            } else {
                for (size_t j = 0; j < n; j++) cand.push_back((uint32_t)j);
            }
            Tup acc = face[i];
            for (uint32_t j : cand) {
                if (j == i) continue;
                const Shape* t = tris[j];
                if (tuple_equals(p, t->p1) || tuple_equals(p, t->p2) || tuple_equals(p, t->p3))
                    acc = add(acc, face[j]);
            }
            res[i][k] = normalize(acc);
        }
    }
    for (size_t i = 0; i < n; i++) {
        tris[i]->n1 = res[i][0];
        tris[i]->n2 = res[i][1];
        tris[i]->n3 = res[i][2];
    }
}

}  // namespace ptmi_host

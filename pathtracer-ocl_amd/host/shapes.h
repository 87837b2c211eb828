// shapes.h -- the reference's scene graph (internal/app/shapes, material, obj)
// as far as it feeds the kernel's input records: transforms (SetTransform
// post-multiplies then inverts, sphere.go:60-64), materials (material.go),
// bounding boxes with Go's sequential BoundingBox.Add (boundingbox.go), the BVH
// Divide / PartitionChildren / MakeSubGroup / SplitBounds (bvh.go:8-119), the
// OBJ/MTL reader (objparser.go) and ComputeVertexNormals (objparser.go:137-178).
#pragma once
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "geom.h"

namespace ptmi_host {

constexpr double kInf = HUGE_VAL;

struct Material {  // material.Material (material/material.go:7-21)
    Tup color = tuple3(1, 1, 1);
    Tup emission = tuple3(0, 0, 0);
    double refractive_index = 1.0;
    double reflectivity = 0.0;
    bool textured = false, textured_nm = false, is_env_map = false;
    uint8_t texture_id = 0, texture_id_nm = 0;
    double texture_scale_x = 0.0, texture_scale_y = 0.0, texture_scale_x_nm = 0.0, texture_scale_y_nm = 0.0;
};
inline Material new_material(Tup c, Tup e, double ri, double refl = 0.0) {
    Material m;
    m.color = c, m.emission = e, m.refractive_index = ri, m.reflectivity = refl;
    return m;
}
inline Material new_default_material() { return new_material(tuple3(1, 1, 1), tuple3(0, 0, 0), 1.0); }
inline Material new_diffuse(double r, double g, double b) { return new_material(tuple3(r, g, b), tuple3(0, 0, 0), 1.0); }
inline Material new_glass() { return new_material(tuple3(1, 1, 1), tuple3(0, 0, 0), 1.52, 0.05); }
inline Material new_mirror() { return new_material(tuple3(1, 1, 1), tuple3(0, 0, 0), 1.0, 1.0); }
inline Material new_light_bulb() { return new_material(tuple3(1, 1, 1), tuple3(8, 8, 8), 1.0); }

struct Box {  // BoundingBox: Min/Max points (w = 1)
    Tup mn{kInf, kInf, kInf, 1.0};
    Tup mx{-kInf, -kInf, -kInf, 1.0};
    // Add (boundingbox.go): strict compares, so NaN never enters and on a tie the
    // first value seen stays.
    void add(const Tup& p) {
        for (int k = 0; k < 3; k++) {
            if (mn[k] > p[k]) mn[k] = p[k];
            if (mx[k] < p[k]) mx[k] = p[k];
        }
    }
    void merge(const Box& b) {  // MergeWith: Add(b.Min), Add(b.Max)
        add(b.mn);
        add(b.mx);
    }
};

enum Kind { PLANE = 0, SPHERE = 1, CYLINDER = 2, CUBE = 3, GROUP = 4, TRIANGLE = 5 };

struct Shape {
    Kind kind;
    std::string label;
    Mat transform = identity(), inverse = identity(), inverse_transpose = identity();
    Material material;
    double min_y = -kInf, max_y = kInf;  // cylinder
    bool closed = false;
    Tup p1{}, p2{}, p3{}, e1{}, e2{}, n{}, n1{}, n2{}, n3{};  // triangle
    std::vector<Shape*> children;                              // group
    Box bbox;                                                  // group

    void set_transform(const Mat& m) {
        transform = multiply(transform, m);
        inverse = ptmi_host::inverse(transform);
        inverse_transpose = transpose(inverse);
    }
    void set_material(const Material& m) { material = m; }  // groups do not propagate (group.go:80-85)
    void add_child(Shape* s);
    void add_children(const std::vector<Shape*>& v) {
        for (Shape* s : v) add_child(s);
    }
    void bounds();  // Group.Bounds(): BoundingBox = BoundsOf(g)
};

// Owns every shape of a scene build.
struct Arena {
    std::deque<Shape> shapes;
    int subgroup_counter = 0;  // MakeSubGroup's process-global label counter (bvh.go:74-84)
    Shape* make(Kind k);
    Shape* plane();     // plane.go:12-29: RefractiveIndex 0 until SetMaterial
    Shape* sphere();    // sphere.go:15-31
    Shape* cylinder(double min_y, double max_y, bool closed);
    Shape* cube();
    Shape* group();     // zero Material{}
    Shape* triangle(const Tup& p1, const Tup& p2, const Tup& p3, const Tup* n1 = nullptr, const Tup* n2 = nullptr,
                    const Tup* n3 = nullptr);
};

Box bounds_of(const Shape* s);
Box parent_space_bounds(const Shape* s);
void divide(Arena& A, Shape* s, size_t threshold);
// Divide's steps (bvh.go:8-84), exported for the reference's own known-answer tests
// (tests/host_kat/host_kat.cpp).
void split_bounds(const Box& b, Box& left, Box& right);
void partition_children(Arena& A, Shape* g, Shape*& left, Shape*& right);
void make_sub_group(Arena& A, Shape* g, const std::vector<Shape*>& v);

// OBJ model (obj/objparser.go): groups attached to the root in FILE order (the
// Go code iterates a map, objparser.go:208-214); mtllib resolved next to the OBJ.
struct ObjModel {
    std::vector<Tup> vertices{point(0, 0, 0)};
    std::vector<Tup> normals{vector(0, 0, 0)};
    std::vector<std::pair<std::string, Shape*>> groups;
    size_t ignored_lines = 0;  // Obj.IgnoredLines: blank rows and unknown keywords
    Shape* to_group(Arena& A) const;
};
ObjModel parse_obj(Arena& A, const std::string& data, const std::string& base_dir);
void compute_vertex_normals(const std::vector<Shape*>& tris);

}  // namespace ptmi_host

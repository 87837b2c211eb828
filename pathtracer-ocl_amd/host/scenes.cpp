// scenes.cpp -- the cmd/pt scene factories (internal/app/scenes), the
// camera (camera/camera.go) and BuildSceneBufferCL / BuildCLGroup
// (internal/ocl/scene.go:14-155), behind the C ABI of include/ptmi_host.h.
// The records are byte-identical to the Python restatement (ptmi/scenes.py,
// ptmi/layout.py), which the reference-kernel goldens pin (tests/test_host.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>
#include <stdexcept>

#include "../../include/ptmi.h"
#include "../../include/ptmi_host.h"
#include "shapes.h"

namespace ptmi_host {
namespace {

// Go untyped constants are rounded once to float64.
constexpr double PI_OVER_2 = 1.5707963267948966;
constexpr double PI_OVER_3 = 1.0471975511965979;
constexpr double PI_OVER_4 = 0.7853981633974483;
constexpr double PI_OVER_12 = 0.26179938779914946;
constexpr double PI = 3.141592653589793;  // math.Pi

struct Camera {  // camera.Camera (camera.go:8-19)
    int width = 0, height = 0;
    double fov = 0, pixel_size = 0, half_width = 0, half_height = 0, aperture = 0, focal_length = 0;
    Mat transform = identity(), inverse = identity();
};

Mat view_transform(const Tup& frm, const Tup& to, const Tup& up) {  // camera.go:50-81
    Mat vt = identity();
    const Tup forward = normalize(sub(to, frm));
    const Tup up_n = normalize(up);
    const Tup left = cross(forward, up_n);
    const Tup true_up = cross(left, forward);
    vt[0] = left[0], vt[1] = left[1], vt[2] = left[2];
    vt[4] = true_up[0], vt[5] = true_up[1], vt[6] = true_up[2];
    vt[8] = -forward[0], vt[9] = -forward[1], vt[10] = -forward[2];
    return multiply(vt, translate(-frm[0], -frm[1], -frm[2]));
}

Camera new_camera(int width, int height, double fov, const Tup& frm, const Tup& to) {  // camera.go:21-48
    Camera c;
    const double half_view = gomath::Tan(fov / 2);
    const double aspect = (double)width / (double)height;
    if (aspect >= 1.0) {
        c.half_width = half_view;
        c.half_height = half_view / aspect;
    } else {
        c.half_width = half_view * aspect;
        c.half_height = half_view;
    }
    c.width = width, c.height = height, c.fov = fov;
    c.pixel_size = (c.half_width * 2) / (double)width;
    c.transform = view_transform(frm, to, vector(0, 1, 0));
    c.inverse = ptmi_host::inverse(c.transform);
    return c;
}

struct Scene {
    Camera cam;
    std::vector<Shape*> objects;
};

struct Ctx {
    Arena A;
    std::string assets;
    Camera std_camera(int w, int h, double ap, double fl) {
        Camera c = new_camera(w, h, PI_OVER_3, point(0, 0.1, -1.5), point(0, 0.05, 0));
        c.focal_length = fl;
        c.aperture = ap;
        return c;
    }
    // left, right, floor, ceil, back, front (the walls of the Cornell scenes)
    std::array<Shape*, 6> walls(double back_z = .4) {
        Shape* left = A.plane();
        left->set_transform(translate(-.6, 0, 0));
        left->set_transform(rotate_z(PI_OVER_2));
        left->set_material(new_diffuse(0.75, 0.25, 0.25));
        Shape* right = A.plane();
        right->set_transform(translate(.6, 0, 0));
        right->set_transform(rotate_z(PI_OVER_2));
        right->set_material(new_diffuse(0.25, 0.25, 0.75));
        Shape* floor = A.plane();
        floor->set_transform(translate(0, -.4, 0));
        floor->set_material(new_diffuse(0.9, 0.8, 0.7));
        Shape* ceil = A.plane();
        ceil->set_transform(translate(0, .4, 0));
        ceil->set_material(new_diffuse(0.9, 0.8, 0.7));
        Shape* back = A.plane();
        back->set_transform(translate(0, 0, back_z));
        back->set_transform(rotate_x(PI_OVER_2));
        back->set_material(new_diffuse(0.9, 0.8, 0.7));
        Shape* front = A.plane();
        front->set_transform(translate(0, 0, -2));
        front->set_transform(rotate_x(PI_OVER_2));
        front->set_material(new_diffuse(0.9, 0.8, 0.7));
        return {left, right, floor, ceil, back, front};
    }
    void label_walls(std::array<Shape*, 6>& w) {
        const char* l[6] = {"leftwall", "rghtwall", "floor   ", "ceiling ", "backwall", "frntwall"};
        for (int i = 0; i < 6; i++) w[i]->label = l[i];
    }
    Shape* sphere(double tx, double ty, double tz, double s, const Material& m) {
        Shape* sp = A.sphere();
        sp->set_transform(translate(tx, ty, tz));
        sp->set_transform(scale(s, s, s));
        sp->set_material(m);
        return sp;
    }
    Shape* light_sphere(const Tup& emission, const Tup* color = nullptr) {
        Shape* src = A.sphere();
        src->set_transform(translate(0, .399, 0));
        src->set_transform(scale(0.283, 0.01, 0.283));
        Material light = new_light_bulb();
        light.emission = emission;
        if (color) light.color = *color;
        src->set_material(light);
        return src;
    }
    Shape* cube_light(double tx, double ty, double tz, double sx, double sy, double sz, const Tup& emission) {
        Shape* c = A.cube();
        c->set_transform(translate(tx, ty, tz));
        c->set_transform(scale(sx, sy, sz));
        Material m = new_light_bulb();
        m.emission = emission;
        m.color = color(1, 1, 1);
        c->set_material(m);
        return c;
    }
    ObjModel load_obj(const std::string& name) {
        const std::string path = assets + "/" + name;
        std::ifstream f(path);
        if (!f) throw std::runtime_error("cannot read " + path);
        std::stringstream ss;
        ss << f.rdbuf();
        return parse_obj(A, ss.str(), assets);
    }
};

// ---- scenes ------------------------------------------------------------------

Scene reference_scene(Ctx& C, int w, int h, double ap, double fl) {  // scenes/reference.go:12-83
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls();
    Shape* ls = C.sphere(-0.35, -0.28, -0.15, 0.12, new_diffuse(0.9, 0.8, 0.7));
    Shape* rs = C.sphere(0, -0.24, -0.30, 0.16, new_diffuse(0.9, 0.8, 0.7));
    Shape* light = C.light_sphere(color(9, 9, 9));
    S.objects = {light, W[2], W[3], W[0], W[1], W[4], ls, rs};
    return S;
}

Scene ocl_scene(Ctx& C, int w, int h, double ap, double fl) {  // scenes/ocl.go (the CLI default)
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls();
    Shape* lsp = C.sphere(-0.25, -0.24, 0.1, 0.16, new_diffuse(0.9, 0.8, 0.7));
    Material half_mirror = new_mirror();
    half_mirror.reflectivity = 0.8;
    half_mirror.color = color(0.97, 0.97, 0.843);
    Shape* rsp = C.sphere(0.25, -0.24, 0.1, 0.16, half_mirror);
    Shape* cyl = C.A.cylinder(0, 0.4, true);
    cyl->set_transform(translate(0.45, -0.5, -0.2));
    cyl->set_transform(scale(0.075, 1, 0.075));
    cyl->set_material(new_diffuse(0.92, 0.4, 0.8));
    Shape* cube = C.A.cube();
    cube->set_transform(translate(-0.3, -0.375, -0.3));
    cube->set_transform(scale(0.1, 0.05, 0.04));
    cube->set_transform(rotate_y(PI_OVER_4));
    cube->set_transform(rotate_z(PI_OVER_2));
    cube->set_material(new_diffuse(0.25, 0.25, 0.75));
    Shape* light_src = C.A.sphere();
    light_src->set_transform(translate(0, 1.36, 0));
    Material light = new_light_bulb();
    light.emission = color(9, 8, 6);
    light_src->set_material(light);
    Shape* t1 = C.A.triangle(point(-0.2, -.4, 0), point(0.0, -.4, 0), point(0, -0.1, 0));
    Shape* t2 = C.A.triangle(point(0, -.4, 0), point(0.2, -.4, 0), point(0, -0.1, 0));
    Shape* t3 = C.A.triangle(point(0.1, -.4, -0.4), point(0, -0.1, 0), point(0, -.4, 0));
    Shape* grp = C.A.group();
    grp->set_material(new_diffuse(0.7, 0.4, 0.9));
    grp->set_transform(translate(0.15, 0, -0.25));
    grp->add_children({t1, t2, t3});
    grp->bounds();
    S.objects = {W[2], W[3], W[0], W[1], W[4], lsp, rsp, cyl, cube, grp, light_src};
    return S;
}

Shape* mesh_group(Ctx& C, const char* file, bool normals) {
    ObjModel model = C.load_obj(file);
    Shape* group = model.to_group(C.A);
    if (normals) compute_vertex_normals(group->children.at(0)->children);
    return group;
}

Scene teapot_scene(Ctx& C, int w, int h, double ap, double fl) {  // ModelScene (scenes/teapot.go:15-125)
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls();
    Shape* lsp = C.sphere(-0.35, -0.28, -0.15, 0.12, new_diffuse(0.9, 0.8, 0.7));
    Shape* group = mesh_group(C, "teapot.obj", true);
    group->bounds();
    group->set_transform(translate(0, -0.4, 0));
    group->set_transform(scale(0.07, 0.07, 0.07));
    Material silver = new_diffuse(0.75, 0.75, 0.75);
    silver.reflectivity = 0.2;
    group->set_material(silver);
    divide(C.A, group, 50);
    group->bounds();
    Shape* light_src = C.A.sphere();
    light_src->set_transform(translate(0, .4, 0));
    light_src->set_transform(scale(0.3, 0.03, 0.3));
    Material light = new_light_bulb();
    light.emission = color(9, 8, 6);
    light_src->set_material(light);
    S.objects = {light_src, W[2], W[3], W[0], W[1], W[4], group, lsp};
    return S;
}

Scene gopher_scene(Ctx& C, int w, int h, double ap, double fl) {  // GopherScene (scenes/gopher.go)
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(1.4);
    Material half_mirror = new_mirror();
    half_mirror.reflectivity = 0.8;
    half_mirror.color = color(0.97, 0.97, 0.843);
    Shape* rsp = C.sphere(0.28, -0.24, 0.15, 0.16, half_mirror);
    S.objects = {W[2], W[3], W[0], W[1], W[4], W[5], rsp};
    Shape* group = mesh_group(C, "gopher.obj", false);
    group->bounds();
    group->set_transform(translate(-.4, -0.15, 0.2));
    group->set_transform(rotate_z(-PI_OVER_2));
    group->set_transform(rotate_x(-PI_OVER_4));
    group->set_transform(scale(0.2, 0.2, 0.2));
    Material silver = new_diffuse(0.75, 0.75, 0.75);
    silver.reflectivity = 0.2;
    group->set_material(silver);
    divide(C.A, group, 60);
    group->bounds();
    S.objects.push_back(group);
    Shape* light_src = C.A.sphere();
    light_src->set_transform(translate(0, 1.36, 0));
    Material light = new_light_bulb();
    light.emission = color(9, 8, 6);
    light_src->set_material(light);
    S.objects.push_back(light_src);
    return S;
}

Scene reflection_scene(Ctx& C, int w, int h, double ap, double fl) {  // scenes/reflections.go:12-83
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.4);
    Shape* lsp = C.sphere(-0.35, -0.28, -0.15, 0.12, new_mirror());
    Shape* rsp = C.sphere(0, -0.24, -0.30, 0.16, new_diffuse(0.9, 0.8, 0.7));
    Shape* light = C.light_sphere(color(9, 9, 9));
    S.objects = {light, W[2], W[3], W[0], W[1], W[4], lsp, rsp};
    return S;
}

// Glass, diffuse with RI 1.57, mirror (scenes/transparency*.go:62-82)
std::array<Shape*, 3> transparency_spheres(Ctx& C, double lx, double ly, double lz, double ls, double rx, double ry,
                                           double rz, double rs) {
    Shape* lsp = C.sphere(lx, ly, lz, ls, new_glass());
    Shape* msp = C.sphere(0, -0.24, -0.30, 0.16, new_diffuse(0.9, 0.8, 0.7));
    msp->material.refractive_index = 1.57;
    Shape* rsp = C.sphere(rx, ry, rz, rs, new_mirror());
    lsp->label = "left_spr", msp->label = "mddl_spr", rsp->label = "right_spr";
    return {lsp, msp, rsp};
}

Scene transparency_scene(Ctx& C, int w, int h, double ap, double fl) {  // scenes/transparency.go:13-101
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.6);
    C.label_walls(W);
    auto sp = transparency_spheres(C, -0.25, -0.28, 0.25, 0.12, 0.25, -0.28, 0.25, 0.12);
    const Tup white = color(1, 1, 1);
    Shape* light = C.light_sphere(color(9, 9, 9), &white);
    light->label = "light   ";
    S.objects = {light, W[2], W[3], W[0], W[1], W[4], sp[0], sp[1], sp[2]};
    return S;
}

Scene transparency_f_light_scene(Ctx& C, int w, int h, double ap, double fl) {  // transparency_f_light.go:13-113
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.6);
    C.label_walls(W);
    auto sp = transparency_spheres(C, -0.25, -0.18, 0.25, 0.14, 0.35, -0.23, 0.2, 0.17);
    const Tup e = color(9, 9, 9);
    Shape* l1 = C.cube_light(-0.125, .3999, 0.05, 0.05, 0.01, 0.45, e);
    Shape* l2 = C.cube_light(-0.02, .3999, -0.35, 0.075, 0.01, 0.05, e);
    Shape* l3 = C.cube_light(-0.05, .3999, 0, 0.075, 0.01, 0.05, e);
    l1->label = "light 1", l2->label = "light top", l3->label = "light middle";
    S.objects = {W[2], W[3], W[0], W[1], W[4], sp[0], sp[1], sp[2], l1, l2, l3};
    return S;
}

Scene transparency_quad_lights_scene(Ctx& C, int w, int h, double ap, double fl) {  // transparency_quadlights.go
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.6);
    C.label_walls(W);
    auto sp = transparency_spheres(C, -0.25, -0.18, 0.25, 0.14, 0.35, -0.23, 0.2, 0.17);
    S.objects = {W[2], W[3], W[0], W[1], W[4], sp[0], sp[1], sp[2]};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) {
            Shape* l = C.cube_light(-0.25 + (double)i * 0.5, .399, -0.25 + (double)j * 0.5, 0.15, 0.01, 0.15,
                                    color(9, 9, 9));
            l->label = "light " + std::to_string(i) + "-" + std::to_string(j);
            S.objects.push_back(l);
        }
    return S;
}

Scene transparent_teapot_scene(Ctx& C, int w, int h, double ap, double fl) {  // transparent_teapot.go:14-128
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.6);
    C.label_walls(W);
    Shape* lsp = C.sphere(-0.25, -0.28, 0.25, 0.12, new_diffuse(0.9, 0.8, 0.7));
    Shape* rsp = C.sphere(0.25, -0.28, 0.25, 0.12, new_glass());
    lsp->label = "left_spr", rsp->label = "right_spr";
    Material mtrl = new_glass();
    mtrl.refractive_index = -1.0;
    mtrl.reflectivity = 0.2;
    Shape* group = mesh_group(C, "teapot.obj", true);
    group->bounds();
    group->set_transform(translate(0, -0.38, -0.2));
    group->set_transform(rotate_y(PI_OVER_12));
    group->set_transform(scale(0.1, 0.1, 0.1));
    group->set_material(mtrl);
    divide(C.A, group, 50);
    group->bounds();
    group->label = "teapot  ";
    Shape* light = C.light_sphere(color(9, 9, 9));
    light->label = "light   ";
    S.objects = {light, W[2], W[3], W[0], W[1], W[4], lsp, rsp, group};
    return S;
}

Material textured(Material m, uint8_t tid, double sx = 0.0, double sy = 0.0) {  // Material.Textured ...
    m.textured = true;
    m.texture_id = tid;
    m.texture_scale_x = sx;
    m.texture_scale_y = sy;
    return m;
}
Material with_nm(Material m, uint8_t tid, double sx, double sy) {  // Material.TexturedNM ...
    m.textured_nm = true;
    m.texture_id_nm = tid;
    m.texture_scale_x_nm = sx;
    m.texture_scale_y_nm = sy;
    return m;
}

Scene textured_planets_scene(Ctx& C, int w, int h, double ap, double fl) {  // texturedplanets.go:13-135
    Scene S{C.std_camera(w, h, ap, fl), {}};
    Shape* left = C.A.plane();
    left->set_transform(translate(-.6, 0, 0));
    left->set_transform(rotate_x(PI));
    left->set_transform(rotate_z(PI_OVER_2));
    left->set_transform(rotate_y(PI_OVER_2));
    left->set_material(with_nm(textured(new_diffuse(0.75, 0.25, 0.25), 0, 1.0, 1.0), 3, 1.0, 1.0));
    Shape* right = C.A.plane();
    right->set_transform(translate(.6, 0, 0));
    right->set_transform(rotate_z(PI_OVER_2));
    right->set_transform(rotate_y(PI_OVER_2));
    right->set_material(with_nm(textured(new_diffuse(0.25, 0.25, 0.75), 0, 1.0, 1.0), 3, 1.0, 1.0));
    Shape* floor = C.A.plane();
    floor->set_transform(translate(0, -.4, 0));
    floor->set_material(textured(new_diffuse(0.9, 0.8, 0.7), 1, 0.25, 0.25));
    Shape* ceil = C.A.plane();
    ceil->set_transform(translate(0, .4, 0));
    ceil->set_material(textured(new_diffuse(0.9, 0.8, 0.7), 2, 1.0, 1.0));
    Shape* back = C.A.plane();
    back->set_transform(translate(0, 0, .4));
    back->set_transform(rotate_x(PI_OVER_2));
    back->set_material(with_nm(textured(new_diffuse(0.9, 0.8, 0.7), 0, 1.0, 1.0), 3, 1.0, 1.0));
    Shape* lsp = C.sphere(-0.3, -0.1, -0.25, 0.2, textured(new_diffuse(0.9, 0.8, 0.7), 1));
    Shape* rsp = C.A.sphere();
    rsp->set_transform(translate(0.2, 0, -0.3));
    rsp->set_transform(rotate_y(PI));
    rsp->set_transform(scale(0.25, 0.25, 0.25));
    rsp->set_material(textured(new_diffuse(0.9, 0.8, 0.7), 0));
    Material light = new_light_bulb();
    light.emission = color(10, 10, 10);
    Shape* l1 = C.A.sphere();
    l1->set_transform(translate(0, .395, -.9));
    l1->set_transform(scale(0.283, 0.01, 0.283));
    l1->set_material(light);
    Shape* l2 = C.A.sphere();
    l2->set_transform(translate(0, 0, -1.7));
    l2->set_transform(scale(0.283, 0.283, 0.01));
    l2->set_material(light);
    S.objects = {l1, l2, floor, ceil, left, right, back, lsp, rsp};
    return S;
}

Material sky_material(bool env_map) {  // envmap.go:55-61, cubemap.go:60-66
    Material m = textured(new_default_material(), 0, 1.0, 1.0);
    m.emission = color(1, 1, 1);
    m.is_env_map = env_map;
    return m;
}

Scene envmap_scene(Ctx& C, int w, int h, double ap, double fl) {  // EnvironmentMap (envmap.go:13-72)
    Camera cam = new_camera(w, h, PI_OVER_3, point(0, 0.1, -1.5), point(0, 0.15, 0));
    cam.focal_length = fl, cam.aperture = ap;
    Scene S{cam, {}};
    Shape* rsp = C.sphere(0, -0.14, -0.30, 0.16, new_mirror());
    Shape* sky = C.A.sphere();
    sky->set_transform(scale(5, 5, 5));
    sky->set_material(sky_material(false));
    S.objects = {rsp, sky};
    return S;
}

Scene cubemap_scene(Ctx& C, int w, int h, double ap, double fl) {  // EnvironmentCubeMap (cubemap.go:15-94)
    C.A.subgroup_counter = 0;
    Camera cam = new_camera(w, h, PI_OVER_3, point(0, 0.3, -2.7), point(0, 0.45, 0));
    cam.focal_length = fl, cam.aperture = ap;
    Scene S{cam, {}};
    Shape* rsp = C.sphere(.2, 1, 2, 0.26, new_mirror());
    Material light = new_light_bulb();
    light.emission = color(19.5, 19.5, 19.5);
    Shape* lsrc = C.sphere(1.1, 1, -4, 0.7, light);
    Shape* sky = C.A.cube();
    sky->set_transform(translate(0, 0, 0));
    sky->set_transform(scale(5, 5, 5));
    sky->set_material(sky_material(true));
    Shape* group = mesh_group(C, "gopher.obj", false);
    group->bounds();
    group->set_transform(translate(-.7, -0.15, 0.2));
    group->set_transform(rotate_z(-PI_OVER_2));
    group->set_transform(rotate_x(-PI_OVER_4));
    group->set_transform(scale(0.4, 0.4, 0.4));
    Material silver = new_diffuse(0.75, 0.75, 0.75);
    silver.reflectivity = 0.0;
    group->set_material(silver);
    divide(C.A, group, 60);
    group->bounds();
    S.objects = {lsrc, rsp, sky, group};
    return S;
}

Shape* cube_at(Ctx& C, double tx, double ty, double tz, std::initializer_list<Mat> rots, double sx, double sy,
               double sz, const Material& m) {
    Shape* c = C.A.cube();
    c->set_transform(translate(tx, ty, tz));
    for (const Mat& r : rots) c->set_transform(r);
    c->set_transform(scale(sx, sy, sz));
    c->set_material(m);
    return c;
}

Scene gopher_window_scene(Ctx& C, int w, int h, double ap, double fl) {  // gopher-with-window.go:15-140
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(1.4);
    Material window = new_diffuse(0.75, 0.75, 1);
    window.emission = color(24, 24, 24);
    const Mat ry = rotate_y(PI_OVER_2), rx = rotate_x(PI_OVER_2);
    const Material border = new_diffuse(0.95, 0.95, 1);
    Shape* cube = cube_at(C, 0.6, .1, 0, {ry}, 0.1, 0.16, 0.002, window);
    Shape* rb = cube_at(C, 0.6, .1, -0.1, {ry}, 0.01, 0.16, 0.02, border);
    Shape* lb = cube_at(C, 0.6, .1, 0.1, {ry}, 0.01, 0.16, 0.02, border);
    Shape* bb = cube_at(C, 0.6, -.06, 0.0, {rx, ry}, 0.01, 0.11, 0.04, border);
    Shape* tb = cube_at(C, 0.6, .26, 0.0, {rx, ry}, 0.01, 0.11, 0.03, border);
    Shape* csp = C.sphere(0, -0.28, -0.3, 0.12, new_diffuse(0.9, 0.8, 0.7));
    Material half_mirror = new_mirror();
    half_mirror.reflectivity = 0.8;
    half_mirror.color = color(0.97, 0.97, 0.843);
    Shape* rsp = C.sphere(0.28, -0.24, 0.15, 0.16, half_mirror);
    S.objects = {W[2], W[3], W[0], W[1], W[4], cube, lb, rb, bb, tb, W[5], csp, rsp};
    Shape* group = mesh_group(C, "gopher.obj", false);
    group->bounds();
    group->set_transform(translate(-.4, -0.15, 0.2));
    group->set_transform(rotate_z(-PI_OVER_2));
    group->set_transform(rotate_x(-PI_OVER_4));
    group->set_transform(scale(0.2, 0.2, 0.2));
    Material silver = new_diffuse(0.75, 0.75, 0.75);
    silver.reflectivity = 0.2;
    group->set_material(silver);
    divide(C.A, group, 60);
    group->bounds();
    S.objects.push_back(group);
    Shape* lsrc = C.A.sphere();
    lsrc->set_transform(translate(0, 1.36, 0));
    Material light = new_light_bulb();
    light.emission = color(9, 8, 6);
    lsrc->set_material(light);
    S.objects.push_back(lsrc);
    return S;
}

Scene christian_scene(Ctx& C, int w, int h, double ap, double fl) {  // christian.go:14-190
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls();
    Shape* lsp = C.sphere(-0.35, -0.28, -0.15, 0.12, new_diffuse(0.9, 0.9, 0.9));
    lsp->material.reflectivity = 0.99;
    Shape* group = mesh_group(C, "teapot.obj", true);
    group->bounds();
    group->set_transform(translate(0, -0.4, 0));
    group->set_transform(scale(0.07, 0.07, 0.07));
    Material silver = new_diffuse(0.75, 0.75, 0.75);
    silver.reflectivity = 0.2;
    group->set_material(silver);
    divide(C.A, group, 50);
    group->bounds();
    Material light = new_light_bulb();
    light.emission = color(90, 80, 60);
    Material cover_m = new_diffuse(0.8, 0.8, 0.8);
    cover_m.reflectivity = 0.95;
    auto lamp = [&](double x) { return C.sphere(x, .3, 0, 0.03, light); };
    auto cover = [&](double x) {
        Shape* c = C.A.cylinder(0, 1, false);
        c->set_transform(translate(x, .295, 0));
        c->set_transform(scale(0.06, 0.4, 0.06));
        c->set_material(cover_m);
        return c;
    };
    Shape* l2 = lamp(-0.3);
    Shape* l3 = lamp(-0.1);
    Shape* l4 = lamp(0.1);
    Shape* l5 = lamp(0.3);
    Shape* c2 = cover(-0.3);
    Shape* c3 = cover(-0.1);
    Shape* c4 = cover(0.1);
    Shape* c5 = cover(0.3);
    S.objects = {l2, l3, l4, l5, c2, c3, c4, c5, W[2], W[3], W[0], W[1], W[4], group, lsp};
    return S;
}

// GlassScene (transparent_glass.go:15-146).  Its mesh, assets/glass.obj, is not
// shipped with the reference: without it the build fails as Go's os.ReadFile panic.
Scene glass_scene(Ctx& C, int w, int h, double ap, double fl) {
    C.A.subgroup_counter = 0;
    Scene S{C.std_camera(w, h, ap, fl), {}};
    auto W = C.walls(.6);
    C.label_walls(W);
    Shape* lsp = C.sphere(-0.2, -0.28, 0.25, 0.12, new_mirror());
    Shape* rsp = C.sphere(0.25, -0.28, 0.25, 0.12, new_glass());
    lsp->label = "left_spr", rsp->label = "right_spr";
    Material mtrl = new_glass();
    mtrl.reflectivity = 0.0;
    ObjModel model = C.load_obj("glass.obj");
    Shape* group = model.to_group(C.A);
    std::vector<Shape*> tris = group->children.at(0)->children;  // glass(): children 0 and 1 (:128-134)
    const auto& t1 = group->children.at(1)->children;
    tris.insert(tris.end(), t1.begin(), t1.end());
    compute_vertex_normals(tris);
    group->bounds();
    group->set_transform(translate(-0.3, -0.395, -0.2));
    group->set_transform(scale(0.03, 0.03, 0.03));
    group->set_material(mtrl);
    divide(C.A, group, 50);
    group->bounds();
    group->label = "glass   ";
    S.objects = {W[2], W[3], W[0], W[1], W[4], W[5], lsp, rsp, group};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) {
            Shape* l = C.cube_light(-0.25 + (double)i * 0.5, .4, -0.25 + (double)j * 0.5, 0.15, 0.001, 0.15,
                                    color(10, 10, 10));
            l->label = "light " + std::to_string(i) + "-" + std::to_string(j);
            S.objects.push_back(l);
        }
    return S;
}

using Factory = std::function<Scene(Ctx&, int, int, double, double)>;
const std::vector<std::pair<const char*, Factory>>& factories() {
    static const std::vector<std::pair<const char*, Factory>> f = {
        {"reference", reference_scene},
        {"teapot", teapot_scene},
        {"gopher", gopher_scene},
        {"reflection", reflection_scene},
        {"transparency", transparency_scene},
        {"transparency_quad_lights", transparency_quad_lights_scene},
        {"transparency_f_light", transparency_f_light_scene},
        {"transparent_teapot", transparent_teapot_scene},
        {"default", ocl_scene},
        {"textures", textured_planets_scene},
        {"envmap", envmap_scene},
        {"cubemap", cubemap_scene},
        {"gopher-window", gopher_window_scene},
        {"christian", christian_scene},
        {"glass", glass_scene},
    };
    return f;
}

// ---- BuildSceneBufferCL (internal/ocl/scene.go:14-155) --------------------------

template <typename T>
void put(std::vector<uint8_t>& b, size_t off, const T& v) {
    std::memcpy(b.data() + off, &v, sizeof(T));
}
void put_tup(std::vector<uint8_t>& b, size_t off, const Tup& t) { std::memcpy(b.data() + off, t.data(), 32); }
void put_mat(std::vector<uint8_t>& b, size_t off, const Mat& m) { std::memcpy(b.data() + off, m.data(), 128); }

struct Records {
    std::vector<uint8_t> objs, tris, grps;
    uint32_t n_tri = 0, n_grp = 0;
};

// BuildCLGroup (scene.go:96-155): preorder numbering, the node's triangles
// contiguous at triOffset, children[] == 0 means "absent".
int32_t build_cl_group(Records& R, const Shape* g) {
    const int32_t gid = (int32_t)R.n_grp++;
    R.grps.resize(R.grps.size() + PTMI_GROUP_BYTES, 0);
    const size_t base = (size_t)gid * PTMI_GROUP_BYTES;
    put_tup(R.grps, base + 0, g->bbox.mn);
    put_tup(R.grps, base + 32, g->bbox.mx);
    if (g->label.size() > 108) throw std::runtime_error("group label longer than the 108-byte pad (scene.go:108)");
    std::memcpy(R.grps.data() + base + 148, g->label.data(), g->label.size());
    put(R.grps, base + 128, (int32_t)R.n_tri);
    int32_t n = 0;
    for (const Shape* c : g->children) {
        if (c->kind != TRIANGLE) continue;
        const size_t tb = R.tris.size();
        R.tris.resize(tb + PTMI_TRIANGLE_BYTES, 0);
        put_tup(R.tris, tb + 0, c->p1);
        put_tup(R.tris, tb + 32, c->p2);
        put_tup(R.tris, tb + 64, c->p3);
        put_tup(R.tris, tb + 96, c->e1);
        put_tup(R.tris, tb + 128, c->e2);
        put_tup(R.tris, tb + 160, c->n1);
        put_tup(R.tris, tb + 192, c->n2);
        put_tup(R.tris, tb + 224, c->n3);
        put_tup(R.tris, tb + 256, c->material.color);
        R.n_tri++;
        n++;
    }
    put(R.grps, base + 132, n);
    int32_t k = 0;
    for (const Shape* c : g->children) {
        if (c->kind != GROUP) continue;
        if (k >= 2) throw std::runtime_error("BuildCLGroup: more than 2 sub-groups (scene.go:143 index out of range)");
        const int32_t child = build_cl_group(R, c);  // may grow R.grps: write by index afterwards
        put(R.grps, base + 140 + 4 * (size_t)k, child);
        k++;
    }
    put(R.grps, base + 136, (int32_t)(k > 0 ? k : -1));
    return gid;
}

Records build_scene_buffer_cl(const std::vector<Shape*>& objects) {
    Records R;
    R.objs.assign(objects.size() * PTMI_OBJECT_BYTES, 0);
    for (size_t i = 0; i < objects.size(); i++) {
        const Shape* s = objects[i];
        const size_t b = i * PTMI_OBJECT_BYTES;
        std::memcpy(R.objs.data() + b + 849, s->label.data(), std::min<size_t>(8, s->label.size()));
        put_mat(R.objs, b + 0, s->transform);
        put_mat(R.objs, b + 128, s->inverse);
        put_mat(R.objs, b + 256, s->inverse_transpose);
        put_tup(R.objs, b + 384, s->material.color);
        put_tup(R.objs, b + 416, s->material.emission);
        put(R.objs, b + 448, s->material.refractive_index);
        const Material& m = s->material;  // texture fields (scene.go:31-43)
        if (m.textured) {
            R.objs[b + 844] = 1;
            R.objs[b + 845] = m.texture_id;
            put(R.objs, b + 488, m.texture_scale_x);
            put(R.objs, b + 496, m.texture_scale_y);
        }
        if (m.textured_nm) {
            R.objs[b + 846] = 1;
            R.objs[b + 847] = m.texture_id_nm;
            put(R.objs, b + 504, m.texture_scale_x_nm);
            put(R.objs, b + 512, m.texture_scale_y_nm);
        }
        R.objs[b + 848] = m.is_env_map ? 1 : 0;
        for (int c = 0; c < 64; c++) put(R.objs, b + 588 + 4 * (size_t)c, (int32_t)-1);
        int64_t type = 999;
        if (s->kind == GROUP) {
            type = 4;
            put_tup(R.objs, b + 520, s->bbox.mn);
            put_tup(R.objs, b + 552, s->bbox.mx);
            int32_t idx = 0;
            for (const Shape* c : s->children) {
                if (c->kind != GROUP) continue;
                if (idx >= 64) throw std::runtime_error("object with more than 64 root groups");
                const int32_t gid = build_cl_group(R, c);
                put(R.objs, b + 588 + 4 * (size_t)idx, gid);
                idx++;
            }
            put(R.objs, b + 584, idx);
        } else if (s->kind != TRIANGLE) {
            type = (int64_t)s->kind;
            if (s->kind == CYLINDER) {
                put(R.objs, b + 464, s->min_y);
                put(R.objs, b + 472, s->max_y);
            }
        }
        put(R.objs, b + 456, type);
        put(R.objs, b + 480, s->material.reflectivity);
    }
    return R;
}

void camera_record(const Camera& c, uint8_t* out) {  // renderer.go:44-56
    std::memset(out, 0, PTMI_CAMERA_BYTES);
    std::memcpy(out + 0, &c.width, 4);
    std::memcpy(out + 4, &c.height, 4);
    std::memcpy(out + 8, &c.fov, 8);
    std::memcpy(out + 16, &c.pixel_size, 8);
    std::memcpy(out + 24, &c.half_width, 8);
    std::memcpy(out + 32, &c.half_height, 8);
    std::memcpy(out + 40, &c.aperture, 8);
    std::memcpy(out + 48, &c.focal_length, 8);
    std::memcpy(out + 56, c.inverse.data(), 128);
}

void set_err(char* err, size_t len, const std::string& msg) {
    if (err && len) std::snprintf(err, len, "%s", msg.c_str());
}

uint8_t* dup(const std::vector<uint8_t>& v) {
    if (v.empty()) return nullptr;
    uint8_t* p = (uint8_t*)std::malloc(v.size());
    if (p) std::memcpy(p, v.data(), v.size());
    return p;
}

}  // namespace
}  // namespace ptmi_host

using namespace ptmi_host;

extern "C" int ptmi_host_build_scene(const char* name, int width, int height, double aperture, double focal_length,
                                     const char* assets_dir, ptmi_records* out, char* err, size_t err_len) {
    if (!name || !out || width <= 0 || height <= 0) {
        set_err(err, err_len, "ptmi_host_build_scene: bad arguments");
        return PTMI_ERR_ARG;
    }
    std::memset(out, 0, sizeof(*out));
    const Factory* f = nullptr;
    for (const auto& kv : factories())
        if (std::strcmp(kv.first, name) == 0) f = &kv.second;
    if (!f) {
        set_err(err, err_len, std::string("unknown scene '") + name + "' (see ptmi_host_scene_names)");
        return PTMI_ERR_UNSUPPORTED;
    }
    try {
        Ctx C;
        C.assets = assets_dir ? assets_dir : "assets";
        Scene S = (*f)(C, width, height, aperture, focal_length);
        if (S.objects.size() > PTMI_MAX_OBJECTS) {
            set_err(err, err_len, "scene has more than 16 objects (tracer.cl:846)");
            return PTMI_ERR_UNSUPPORTED;
        }
        Records R = build_scene_buffer_cl(S.objects);
        out->objects = dup(R.objs);
        out->n_obj = (uint32_t)S.objects.size();
        out->triangles = dup(R.tris);
        out->n_tri = R.n_tri;
        out->groups = dup(R.grps);
        out->n_grp = R.n_grp;
        camera_record(S.cam, out->camera);
        if ((R.objs.size() && !out->objects) || (R.tris.size() && !out->triangles) ||
            (R.grps.size() && !out->groups)) {
            ptmi_host_free_records(out);
            set_err(err, err_len, "out of host memory");
            return PTMI_ERR_NOMEM;
        }
    } catch (const std::exception& e) {
        set_err(err, err_len, std::string("scene '") + name + "': " + e.what());
        return PTMI_ERR_ARG;
    }
    return PTMI_OK;
}

extern "C" void ptmi_host_free_records(ptmi_records* r) {
    if (!r) return;
    std::free(r->objects);
    std::free(r->triangles);
    std::free(r->groups);
    r->objects = r->triangles = r->groups = nullptr;
    r->n_obj = r->n_tri = r->n_grp = 0;
}

extern "C" const char* ptmi_host_scene_names(void) {
    static const std::string names = [] {
        std::string s;
        for (const auto& kv : factories()) s += std::string(kv.first) + "\n";
        return s;
    }();
    return names.c_str();
}

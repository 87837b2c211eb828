"""Restatement of the reference's camera (internal/app/camera/camera.go) and of the
scene factories the benchmark configs use:

* ``reference``  scenes/reference.go:12-83   (configs C1-C3)
* ``teapot``     scenes/teapot.go:15-125     (config C4, ModelScene)
* ``gopher``     scenes/gopher.go            (config C5)
* ``default``    scenes/ocl.go               (OCLScene: every primitive type, glass, mirror)

Go untyped constants (``math.Pi/3`` ...) are rounded ONCE to float64, unlike
Python's ``math.pi/3`` which rounds twice; they are spelled out below.
"""
import math
import os

from . import geom, objparser, shapes
from .gomath import Tan

PI_OVER_2 = 1.5707963267948966    # float64(math.Pi / 2)
PI_OVER_3 = 1.0471975511965979    # float64(math.Pi / 3)  (!= math.pi / 3)
PI_OVER_4 = 0.7853981633974483    # float64(math.Pi / 4)
PI_OVER_12 = 0.26179938779914946  # float64(math.Pi / 12)  (Go: exact constant, then rounded; != math.pi / 12)

# The OBJ/MTL assets are read from the reference checkout (this container only);
# the GPU box uses the scene records pre-built from them (tests/golden/scene_*.npz,
# made by tests/golden/make_scenes.py).
ASSETS = os.environ.get("PTMI_ASSETS", "/root/reference/assets")


class Camera:
    """camera.Camera (camera.go:8-19)."""

    def __init__(self, width, height, fov, frm, to):
        half_view = Tan(fov / 2)
        aspect = float(width) / float(height)
        if aspect >= 1.0:
            half_width = half_view
            half_height = half_view / aspect
        else:
            half_width = half_view * aspect
            half_height = half_view
        self.width = int(width)
        self.height = int(height)
        self.fov = fov
        self.pixel_size = (half_width * 2) / float(width)
        self.transform = view_transform(frm, to, geom.vector(0, 1, 0))
        self.inverse = geom.inverse(self.transform)
        self.half_width = half_width
        self.half_height = half_height
        self.aperture = 0.0
        self.focal_length = 0.0


def view_transform(frm, to, up):
    """camera.ViewTransform (camera.go:50-81)."""
    vt = geom.identity()
    forward = geom.normalize(geom.sub(to, frm))
    up_n = geom.normalize(up)
    left = geom.cross(forward, up_n)
    true_up = geom.cross(left, forward)
    vt[0], vt[1], vt[2] = left[0], left[1], left[2]
    vt[4], vt[5], vt[6] = true_up[0], true_up[1], true_up[2]
    vt[8], vt[9], vt[10] = -forward[0], -forward[1], -forward[2]
    return geom.multiply(vt, geom.translate(-frm[0], -frm[1], -frm[2]))


class Scene:
    def __init__(self, camera, objects):
        self.camera = camera
        self.objects = objects


def _std_camera(width, height, aperture, focal_length):
    cam = Camera(width, height, PI_OVER_3, geom.point(0, 0.1, -1.5), geom.point(0, 0.05, 0))
    cam.focal_length = float(focal_length)
    cam.aperture = float(aperture)
    return cam


def _walls(back_z=.4):
    left = shapes.Plane()
    left.set_transform(geom.translate(-.6, 0, 0))
    left.set_transform(geom.rotate_z(PI_OVER_2))
    left.set_material(shapes.new_diffuse(0.75, 0.25, 0.25))
    right = shapes.Plane()
    right.set_transform(geom.translate(.6, 0, 0))
    right.set_transform(geom.rotate_z(PI_OVER_2))
    right.set_material(shapes.new_diffuse(0.25, 0.25, 0.75))
    floor = shapes.Plane()
    floor.set_transform(geom.translate(0, -.4, 0))
    floor.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    ceil = shapes.Plane()
    ceil.set_transform(geom.translate(0, .4, 0))
    ceil.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    back = shapes.Plane()
    back.set_transform(geom.translate(0, 0, back_z))
    back.set_transform(geom.rotate_x(PI_OVER_2))
    back.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    front = shapes.Plane()
    front.set_transform(geom.translate(0, 0, -2))
    front.set_transform(geom.rotate_x(PI_OVER_2))
    front.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    return left, right, floor, ceil, back, front


def reference_scene(width, height, aperture=0.0, focal_length=0.0):
    """ReferenceScene (scenes/reference.go:12-83): the Cornell box with two diffuse
    spheres; the front wall is built but not added (reference.go:76)."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _walls()
    ls = shapes.Sphere()
    ls.set_transform(geom.translate(-0.35, -0.28, -0.15))
    ls.set_transform(geom.scale(0.12, 0.12, 0.12))
    ls.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    rs = shapes.Sphere()
    rs.set_transform(geom.translate(0, -0.24, -0.30))
    rs.set_transform(geom.scale(0.16, 0.16, 0.16))
    rs.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    light_src = shapes.Sphere()
    light_src.set_transform(geom.translate(0, .399, 0))
    light_src.set_transform(geom.scale(0.283, 0.01, 0.283))
    light = shapes.new_light_bulb()
    light.emission = geom.color(9, 9, 9)
    light_src.set_material(light)
    return Scene(cam, [light_src, floor, ceil, left, right, back, ls, rs])


def ocl_scene(width, height, aperture=0.0, focal_length=0.0):
    """OCLScene (scenes/ocl.go), the CLI default: planes, diffuse / glass / mirror
    spheres, cylinder, cube and a 3-triangle group (which has no sub-groups, so
    BuildSceneBufferCL gives it childCount 0 and the kernel never tests it)."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _walls()
    lsp = shapes.Sphere()
    lsp.set_transform(geom.translate(-0.25, -0.24, 0.1))
    lsp.set_transform(geom.scale(0.16, 0.16, 0.16))
    lsp.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    msp = shapes.Sphere()
    msp.set_transform(geom.translate(0, -0.24, -0.30))
    msp.set_transform(geom.scale(0.16, 0.16, 0.16))
    msp.set_material(shapes.new_glass())
    rsp = shapes.Sphere()
    rsp.set_transform(geom.translate(0.25, -0.24, 0.1))
    rsp.set_transform(geom.scale(0.16, 0.16, 0.16))
    half_mirror = shapes.new_mirror()
    half_mirror.reflectivity = 0.8
    half_mirror.color = geom.color(0.97, 0.97, 0.843)
    rsp.set_material(half_mirror)
    cyl = shapes.Cylinder(0, 0.4, True)
    cyl.set_transform(geom.translate(0.45, -0.5, -0.2))
    cyl.set_transform(geom.scale(0.075, 1, 0.075))
    cyl.set_material(shapes.new_diffuse(0.92, 0.4, 0.8))
    cube = shapes.Cube()
    cube.set_transform(geom.translate(-0.3, -0.375, -0.3))
    cube.set_transform(geom.scale(0.1, 0.05, 0.04))
    cube.set_transform(geom.rotate_y(PI_OVER_4))
    cube.set_transform(geom.rotate_z(PI_OVER_2))
    cube.set_material(shapes.new_diffuse(0.25, 0.25, 0.75))
    light_src = shapes.Sphere()
    light_src.set_transform(geom.translate(0, 1.36, 0))
    light = shapes.new_light_bulb()
    light.emission = geom.color(9, 8, 6)
    light_src.set_material(light)
    t1 = shapes.new_triangle_n(geom.point(-0.2, -.4, 0), geom.point(0.0, -.4, 0), geom.point(0, -0.1, 0))
    t2 = shapes.new_triangle_n(geom.point(0, -.4, 0), geom.point(0.2, -.4, 0), geom.point(0, -0.1, 0))
    t3 = shapes.new_triangle_n(geom.point(0.1, -.4, -0.4), geom.point(0, -0.1, 0), geom.point(0, -.4, 0))
    grp = shapes.Group()
    grp.set_material(shapes.new_diffuse(0.7, 0.4, 0.9))
    grp.set_transform(geom.translate(0.15, 0, -0.25))
    grp.add_children([t1, t2, t3])
    grp.bounds()
    return Scene(cam, [floor, ceil, left, right, back, lsp, rsp, cyl, cube, grp, light_src])


def _load_obj(name):
    path = os.path.join(ASSETS, name)
    with open(path) as f:
        return objparser.parse_obj(f.read(), base_dir=os.path.dirname(path))


def teapot_scene(width, height, aperture=0.0, focal_length=0.0, obj_path=None):
    """ModelScene (scenes/teapot.go:15-125): Cornell box + BVH teapot (Divide 50)."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _walls()
    lsp = shapes.Sphere()
    lsp.set_transform(geom.translate(-0.35, -0.28, -0.15))
    lsp.set_transform(geom.scale(0.12, 0.12, 0.12))
    lsp.set_material(shapes.new_diffuse(0.9, 0.8, 0.7))
    model = _load_obj("teapot.obj") if obj_path is None else objparser.parse_obj(open(obj_path).read())
    group = model.to_group()
    tris = list(group.children[0].children)
    objparser.compute_vertex_normals(tris)
    group.bounds()
    group.set_transform(geom.translate(0, -0.4, 0))
    group.set_transform(geom.scale(0.07, 0.07, 0.07))
    silver = shapes.new_diffuse(0.75, 0.75, 0.75)
    silver.reflectivity = 0.2
    group.set_material(silver)
    shapes.divide(group, 50)
    group.bounds()
    light_src = shapes.Sphere()
    light_src.set_transform(geom.translate(0, .4, 0))
    light_src.set_transform(geom.scale(0.3, 0.03, 0.3))
    light = shapes.new_light_bulb()
    light.emission = geom.color(9, 8, 6)
    light_src.set_material(light)
    return Scene(cam, [light_src, floor, ceil, left, right, back, group, lsp])


def gopher_scene(width, height, aperture=0.0, focal_length=0.0):
    """GopherScene (scenes/gopher.go): Cornell box + BVH gopher (Divide 60)."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, front = _walls(back_z=1.4)
    rsp = shapes.Sphere()
    rsp.set_transform(geom.translate(0.28, -0.24, 0.15))
    rsp.set_transform(geom.scale(0.16, 0.16, 0.16))
    half_mirror = shapes.new_mirror()
    half_mirror.reflectivity = 0.8
    half_mirror.color = geom.color(0.97, 0.97, 0.843)
    rsp.set_material(half_mirror)
    objects = [floor, ceil, left, right, back, front, rsp]
    group = _load_obj("gopher.obj").to_group()
    group.bounds()
    group.set_transform(geom.translate(-.4, -0.15, 0.2))
    group.set_transform(geom.rotate_z(-PI_OVER_2))
    group.set_transform(geom.rotate_x(-PI_OVER_4))
    group.set_transform(geom.scale(0.2, 0.2, 0.2))
    silver = shapes.new_diffuse(0.75, 0.75, 0.75)
    silver.reflectivity = 0.2
    group.set_material(silver)
    shapes.divide(group, 60)
    group.bounds()
    objects.append(group)
    light_src = shapes.Sphere()
    light_src.set_transform(geom.translate(0, 1.36, 0))
    light = shapes.new_light_bulb()
    light.emission = geom.color(9, 8, 6)
    light_src.set_material(light)
    objects.append(light_src)
    return Scene(cam, objects)


def _labelled(objs, labels):
    """Shape labels as the Go scene sets them (copied into CLObject.Label, scene.go:18-22)."""
    for o, lbl in zip(objs, labels):
        o.label = lbl
    return objs


_WALL_LABELS = ("leftwall", "rghtwall", "floor   ", "ceiling ", "backwall", "frntwall")


def _light_sphere(emission, color=None):
    """The flattened ceiling light sphere of the Cornell scenes (translate (0,.399,0),
    scale (0.283, 0.01, 0.283)) with a LightBulb material."""
    src = shapes.Sphere()
    src.set_transform(geom.translate(0, .399, 0))
    src.set_transform(geom.scale(0.283, 0.01, 0.283))
    light = shapes.new_light_bulb()
    light.emission = emission
    if color is not None:
        light.color = color
    src.set_material(light)
    return src


def _sphere(t, s, material):
    sp = shapes.Sphere()
    sp.set_transform(geom.translate(*t))
    sp.set_transform(geom.scale(s, s, s))
    sp.set_material(material)
    return sp


def reflection_scene(width, height, aperture=0.0, focal_length=0.0):
    """ReflectionsScene (scenes/reflections.go:12-83): mirror + diffuse sphere."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _walls(.4)
    lsp = _sphere((-0.35, -0.28, -0.15), 0.12, shapes.new_mirror())
    rsp = _sphere((0, -0.24, -0.30), 0.16, shapes.new_diffuse(0.9, 0.8, 0.7))
    light = _light_sphere(geom.color(9, 9, 9))
    return Scene(cam, [light, floor, ceil, left, right, back, lsp, rsp])


def _transparency_spheres(left_t, left_s, right_t, right_s):
    """Glass (RI 1.52, reflectivity 0.05), diffuse with RI 1.57, mirror
    (scenes/transparency*.go:62-82)."""
    lsp = _sphere(left_t, left_s, shapes.new_glass())
    mmat = shapes.new_diffuse(0.9, 0.8, 0.7)
    msp = _sphere((0, -0.24, -0.30), 0.16, mmat)
    msp.material.refractive_index = 1.57
    rsp = _sphere(right_t, right_s, shapes.new_mirror())
    return lsp, msp, rsp


def transparency_scene(width, height, aperture=0.0, focal_length=0.0):
    """TransparencyScene (scenes/transparency.go:13-101)."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _labelled(_walls(.6), _WALL_LABELS)
    lsp, msp, rsp = _labelled(_transparency_spheres((-0.25, -0.28, 0.25), 0.12, (0.25, -0.28, 0.25), 0.12),
                              ("left_spr", "mddl_spr", "right_spr"))
    light = _light_sphere(geom.color(9, 9, 9), geom.color(1, 1, 1))
    light.label = "light   "
    return Scene(cam, [light, floor, ceil, left, right, back, lsp, msp, rsp])


def _cube_light(t, s, emission):
    c = shapes.Cube()
    c.set_transform(geom.translate(*t))
    c.set_transform(geom.scale(*s))
    m = shapes.new_light_bulb()
    m.emission = emission
    m.color = geom.color(1, 1, 1)
    c.set_material(m)
    return c


def transparency_f_light_scene(width, height, aperture=0.0, focal_length=0.0):
    """TransparencyFLightScene (scenes/transparency_f_light.go:13-113): three cube
    lights forming an F."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _labelled(_walls(.6), _WALL_LABELS)
    lsp, msp, rsp = _labelled(_transparency_spheres((-0.25, -0.18, 0.25), 0.14, (0.35, -0.23, 0.2), 0.17),
                              ("left_spr", "mddl_spr", "right_spr"))
    e = geom.color(9, 9, 9)
    l1 = _cube_light((-0.125, .3999, 0.05), (0.05, 0.01, 0.45), e)
    l2 = _cube_light((-0.02, .3999, -0.35), (0.075, 0.01, 0.05), e)
    l3 = _cube_light((-0.05, .3999, 0), (0.075, 0.01, 0.05), e)
    _labelled((l1, l2, l3), ("light 1", "light top", "light middle"))
    return Scene(cam, [floor, ceil, left, right, back, lsp, msp, rsp, l1, l2, l3])


def transparency_quad_lights_scene(width, height, aperture=0.0, focal_length=0.0):
    """TransparencyQuadLightsScene (scenes/transparency_quadlights.go:13-106)."""
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _labelled(_walls(.6), _WALL_LABELS)
    lsp, msp, rsp = _labelled(_transparency_spheres((-0.25, -0.18, 0.25), 0.14, (0.35, -0.23, 0.2), 0.17),
                              ("left_spr", "mddl_spr", "right_spr"))
    lights = [_cube_light((-0.25 + float(i) * 0.5, .399, -0.25 + float(j) * 0.5), (0.15, 0.01, 0.15),
                          geom.color(9, 9, 9)) for i in range(2) for j in range(2)]
    _labelled(lights, ["light %d-%d" % (i, j) for i in range(2) for j in range(2)])
    return Scene(cam, [floor, ceil, left, right, back, lsp, msp, rsp] + lights)


def transparent_teapot_scene(width, height, aperture=0.0, focal_length=0.0, obj_path=None):
    """TransparentTeapotScene (scenes/transparent_teapot.go:14-128): a thin-glass
    (refractive index -1, reflectivity 0.2) BVH teapot and a glass sphere."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _labelled(_walls(.6), _WALL_LABELS)
    lsp = _sphere((-0.25, -0.28, 0.25), 0.12, shapes.new_diffuse(0.9, 0.8, 0.7))
    rsp = _sphere((0.25, -0.28, 0.25), 0.12, shapes.new_glass())
    _labelled((lsp, rsp), ("left_spr", "right_spr"))
    mtrl = shapes.new_glass()
    mtrl.refractive_index = -1.0
    mtrl.reflectivity = 0.2
    model = _load_obj("teapot.obj") if obj_path is None else objparser.parse_obj(open(obj_path).read())
    group = model.to_group()
    tris = list(group.children[0].children)
    objparser.compute_vertex_normals(tris)
    group.bounds()
    group.set_transform(geom.translate(0, -0.38, -0.2))
    group.set_transform(geom.rotate_y(PI_OVER_12))
    group.set_transform(geom.scale(0.1, 0.1, 0.1))
    group.set_material(mtrl)
    shapes.divide(group, 50)
    group.bounds()
    group.label = "teapot  "
    light = _light_sphere(geom.color(9, 9, 9))
    light.label = "light   "
    return Scene(cam, [light, floor, ceil, left, right, back, lsp, rsp, group])


def _textured(m, tid, sx=0.0, sy=0.0, nm=None):
    """Material.Textured / TextureID / TextureScaleX/Y (+ the NM set when nm = (id, sx, sy))."""
    m.textured = True
    m.texture_id = tid
    m.texture_scale_x = float(sx)
    m.texture_scale_y = float(sy)
    if nm is not None:
        m.textured_nm = True
        m.texture_id_nm, m.texture_scale_x_nm, m.texture_scale_y_nm = nm[0], float(nm[1]), float(nm[2])
    return m


# Texture lists of the textured scenes: (name, width, height) of each image the Go
# scene loads with LoadImage (scene.go:30-56); the files are not in the reference
# checkout, so callers supply pixels of these shapes (tests/textures_synth.py).
TEXTURE_ASSETS = {
    "textures": {"textures": ["concrete_squares.png", "seamless-cobblestone-texture.jpg", "floor_boards.png",
                              "concrete_squares_nm2.png"],
                 "sphereTextures": ["planet.png", "jupiter2_6k_contrast.png"]},
    "envmap": {"sphereTextures": ["alps_field_8k.png"]},
    "cubemap": {"cubeTextures": ["shrine_cubemap.jpeg"]},
}


def textured_planets_scene(width, height, aperture=0.0, focal_length=0.0):
    """TexturedPlanetsScene (scenes/texturedplanets.go:13-135): textured walls (three
    with the normal map, texture 3), floor, ceiling and two sphere-mapped planets."""
    cam = _std_camera(width, height, aperture, focal_length)
    left = shapes.Plane()
    left.set_transform(geom.translate(-.6, 0, 0))
    left.set_transform(geom.rotate_x(math.pi))
    left.set_transform(geom.rotate_z(PI_OVER_2))
    left.set_transform(geom.rotate_y(PI_OVER_2))
    left.set_material(_textured(shapes.new_diffuse(0.75, 0.25, 0.25), 0, 1.0, 1.0, nm=(3, 1.0, 1.0)))
    right = shapes.Plane()
    right.set_transform(geom.translate(.6, 0, 0))
    right.set_transform(geom.rotate_z(PI_OVER_2))
    right.set_transform(geom.rotate_y(PI_OVER_2))
    right.set_material(_textured(shapes.new_diffuse(0.25, 0.25, 0.75), 0, 1.0, 1.0, nm=(3, 1.0, 1.0)))
    floor = shapes.Plane()
    floor.set_transform(geom.translate(0, -.4, 0))
    floor.set_material(_textured(shapes.new_diffuse(0.9, 0.8, 0.7), 1, 0.25, 0.25))
    ceil = shapes.Plane()
    ceil.set_transform(geom.translate(0, .4, 0))
    ceil.set_material(_textured(shapes.new_diffuse(0.9, 0.8, 0.7), 2, 1.0, 1.0))
    back = shapes.Plane()
    back.set_transform(geom.translate(0, 0, .4))
    back.set_transform(geom.rotate_x(PI_OVER_2))
    back.set_material(_textured(shapes.new_diffuse(0.9, 0.8, 0.7), 0, 1.0, 1.0, nm=(3, 1.0, 1.0)))
    lsp = shapes.Sphere()
    lsp.set_transform(geom.translate(-0.3, -0.1, -0.25))
    lsp.set_transform(geom.scale(0.2, 0.2, 0.2))
    lsp.set_material(_textured(shapes.new_diffuse(0.9, 0.8, 0.7), 1))
    rsp = shapes.Sphere()
    rsp.set_transform(geom.translate(0.2, 0, -0.3))
    rsp.set_transform(geom.rotate_y(math.pi))
    rsp.set_transform(geom.scale(0.25, 0.25, 0.25))
    rsp.set_material(_textured(shapes.new_diffuse(0.9, 0.8, 0.7), 0))
    light = shapes.new_light_bulb()
    light.emission = geom.color(10, 10, 10)
    l1 = shapes.Sphere()
    l1.set_transform(geom.translate(0, .395, -.9))
    l1.set_transform(geom.scale(0.283, 0.01, 0.283))
    l1.set_material(light)
    l2 = shapes.Sphere()
    l2.set_transform(geom.translate(0, 0, -1.7))
    l2.set_transform(geom.scale(0.283, 0.283, 0.01))
    l2.set_material(light)
    return Scene(cam, [l1, l2, floor, ceil, left, right, back, lsp, rsp])


def _sky_material(env_map=False):
    m = _textured(shapes.new_default_material(), 0, 1.0, 1.0)
    m.emission = geom.color(1, 1, 1)
    m.is_env_map = env_map
    return m


def envmap_scene(width, height, aperture=0.0, focal_length=0.0):
    """EnvironmentMap (scenes/envmap.go:13-72): a mirror sphere inside an emissive,
    sphere-mapped sky sphere (the scene list holds only those two)."""
    cam = Camera(width, height, PI_OVER_3, geom.point(0, 0.1, -1.5), geom.point(0, 0.15, 0))
    cam.focal_length, cam.aperture = float(focal_length), float(aperture)
    rsp = _sphere((0, -0.14, -0.30), 0.16, shapes.new_mirror())
    sky = shapes.Sphere()
    sky.set_transform(geom.scale(5, 5, 5))
    sky.set_material(_sky_material())
    return Scene(cam, [rsp, sky])


def _cubemap_camera(width, height, aperture, focal_length):
    cam = Camera(width, height, PI_OVER_3, geom.point(0, 0.3, -2.7), geom.point(0, 0.45, 0))
    cam.focal_length, cam.aperture = float(focal_length), float(aperture)
    return cam


def cubemap_scene(width, height, aperture=0.0, focal_length=0.0):
    """EnvironmentCubeMap (scenes/cubemap.go:15-94): light, mirror sphere, an
    emissive cube-mapped sky cube and the BVH gopher (Divide 60)."""
    shapes.reset_subgroup_counter()
    cam = _cubemap_camera(width, height, aperture, focal_length)
    rsp = _sphere((.2, 1, 2), 0.26, shapes.new_mirror())
    light = shapes.new_light_bulb()
    light.emission = geom.color(19.5, 19.5, 19.5)
    lsrc = _sphere((1.1, 1, -4), 0.7, light)
    sky = shapes.Cube()
    sky.set_transform(geom.translate(0, 0, 0))
    sky.set_transform(geom.scale(5, 5, 5))
    sky.set_material(_sky_material(env_map=True))
    group = _load_obj("gopher.obj").to_group()
    group.bounds()
    group.set_transform(geom.translate(-.7, -0.15, 0.2))
    group.set_transform(geom.rotate_z(-PI_OVER_2))
    group.set_transform(geom.rotate_x(-PI_OVER_4))
    group.set_transform(geom.scale(0.4, 0.4, 0.4))
    silver = shapes.new_diffuse(0.75, 0.75, 0.75)
    silver.reflectivity = 0.0
    group.set_material(silver)
    shapes.divide(group, 60)
    group.bounds()
    return Scene(cam, [lsrc, rsp, sky, group])


def _cube(t, s, material, rots=()):
    c = shapes.Cube()
    c.set_transform(geom.translate(*t))
    for r in rots:
        c.set_transform(r)
    c.set_transform(geom.scale(*s))
    c.set_material(material)
    return c


def gopher_window_scene(width, height, aperture=0.0, focal_length=0.0):
    """GopherWindowScene (scenes/gopher-with-window.go:15-140): the gopher box lit
    through an emissive window cube with four border cubes."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, front = _walls(back_z=1.4)
    window = shapes.new_diffuse(0.75, 0.75, 1)
    window.emission = geom.color(24, 24, 24)
    ry, rx = geom.rotate_y(PI_OVER_2), geom.rotate_x(PI_OVER_2)
    cube = _cube((0.6, .1, 0), (0.1, 0.16, 0.002), window, (ry,))
    rb = _cube((0.6, .1, -0.1), (0.01, 0.16, 0.02), shapes.new_diffuse(0.95, 0.95, 1), (ry,))
    lb = _cube((0.6, .1, 0.1), (0.01, 0.16, 0.02), shapes.new_diffuse(0.95, 0.95, 1), (ry,))
    bb = _cube((0.6, -.06, 0.0), (0.01, 0.11, 0.04), shapes.new_diffuse(0.95, 0.95, 1), (rx, ry))
    tb = _cube((0.6, .26, 0.0), (0.01, 0.11, 0.03), shapes.new_diffuse(0.95, 0.95, 1), (rx, ry))
    csp = _sphere((0, -0.28, -0.3), 0.12, shapes.new_diffuse(0.9, 0.8, 0.7))
    half_mirror = shapes.new_mirror()
    half_mirror.reflectivity = 0.8
    half_mirror.color = geom.color(0.97, 0.97, 0.843)
    rsp = _sphere((0.28, -0.24, 0.15), 0.16, half_mirror)
    objects = [floor, ceil, left, right, back, cube, lb, rb, bb, tb, front, csp, rsp]
    group = _load_obj("gopher.obj").to_group()
    group.bounds()
    group.set_transform(geom.translate(-.4, -0.15, 0.2))
    group.set_transform(geom.rotate_z(-PI_OVER_2))
    group.set_transform(geom.rotate_x(-PI_OVER_4))
    group.set_transform(geom.scale(0.2, 0.2, 0.2))
    silver = shapes.new_diffuse(0.75, 0.75, 0.75)
    silver.reflectivity = 0.2
    group.set_material(silver)
    shapes.divide(group, 60)
    group.bounds()
    objects.append(group)
    light = shapes.new_light_bulb()
    light.emission = geom.color(9, 8, 6)
    lsrc = shapes.Sphere()
    lsrc.set_transform(geom.translate(0, 1.36, 0))
    lsrc.set_material(light)
    objects.append(lsrc)
    return Scene(cam, objects)


def christian_scene(width, height, aperture=0.0, focal_length=0.0, obj_path=None):
    """ChristianScene (scenes/christian.go:14-190): the teapot box with four small
    lights under open reflective cylinder covers and a mirror-like sphere."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, _front = _walls()
    lsp = _sphere((-0.35, -0.28, -0.15), 0.12, shapes.new_diffuse(0.9, 0.9, 0.9))
    lsp.material.reflectivity = 0.99
    model = _load_obj("teapot.obj") if obj_path is None else objparser.parse_obj(open(obj_path).read())
    group = model.to_group()
    objparser.compute_vertex_normals(list(group.children[0].children))
    group.bounds()
    group.set_transform(geom.translate(0, -0.4, 0))
    group.set_transform(geom.scale(0.07, 0.07, 0.07))
    silver = shapes.new_diffuse(0.75, 0.75, 0.75)
    silver.reflectivity = 0.2
    group.set_material(silver)
    shapes.divide(group, 50)
    group.bounds()
    light = shapes.new_light_bulb()
    light.emission = geom.color(90, 80, 60)
    cover_m = shapes.new_diffuse(0.8, 0.8, 0.8)
    cover_m.reflectivity = 0.95

    def lamp(x):
        return _sphere((x, .3, 0), 0.03, light)

    def cover(x):
        c = shapes.Cylinder(0, 1, False)
        c.set_transform(geom.translate(x, .295, 0))
        c.set_transform(geom.scale(0.06, 0.4, 0.06))
        c.set_material(cover_m)
        return c

    return Scene(cam, [lamp(-0.3), lamp(-0.1), lamp(0.1), lamp(0.3), cover(-0.3), cover(-0.1), cover(0.1),
                       cover(0.3), floor, ceil, left, right, back, group, lsp])


def glass_scene(width, height, aperture=0.0, focal_length=0.0, obj_path=None):
    """GlassScene (scenes/transparent_glass.go:15-146).  Its mesh, assets/glass.obj,
    is not shipped with the reference (its own objparser test fails on it), so
    without ``obj_path`` this raises as the Go os.ReadFile panic does."""
    shapes.reset_subgroup_counter()
    cam = _std_camera(width, height, aperture, focal_length)
    left, right, floor, ceil, back, front = _labelled(_walls(.6), _WALL_LABELS)
    lsp = _sphere((-0.2, -0.28, 0.25), 0.12, shapes.new_mirror())
    rsp = _sphere((0.25, -0.28, 0.25), 0.12, shapes.new_glass())
    _labelled((lsp, rsp), ("left_spr", "right_spr"))
    mtrl = shapes.new_glass()
    mtrl.reflectivity = 0.0
    model = _load_obj("glass.obj") if obj_path is None else objparser.parse_obj(open(obj_path).read())
    group = model.to_group()
    objparser.compute_vertex_normals(list(group.children[0].children) + list(group.children[1].children))
    group.bounds()
    group.set_transform(geom.translate(-0.3, -0.395, -0.2))
    group.set_transform(geom.scale(0.03, 0.03, 0.03))
    group.set_material(mtrl)
    shapes.divide(group, 50)
    group.bounds()
    group.label = "glass   "
    lights = [_cube_light((-0.25 + float(i) * 0.5, .4, -0.25 + float(j) * 0.5), (0.15, 0.001, 0.15),
                          geom.color(10, 10, 10)) for i in range(2) for j in range(2)]
    _labelled(lights, ["light %d-%d" % (i, j) for i in range(2) for j in range(2)])
    return Scene(cam, [floor, ceil, left, right, back, front, lsp, rsp, group] + lights)


# Scene cameras other than _std_camera (records of mesh scenes are pre-built; only
# the camera is rebuilt per W/H).
CAMERAS = {"cubemap": _cubemap_camera}


SCENES = {
    "reference": reference_scene,
    "reflection": reflection_scene,
    "transparency": transparency_scene,
    "transparency_f_light": transparency_f_light_scene,
    "transparency_quad_lights": transparency_quad_lights_scene,
    "transparent_teapot": transparent_teapot_scene,
    "teapot": teapot_scene,
    "gopher": gopher_scene,
    "default": ocl_scene,
    "textures": textured_planets_scene,
    "envmap": envmap_scene,
    "cubemap": cubemap_scene,
    "gopher-window": gopher_window_scene,
    "christian": christian_scene,
    "glass": glass_scene,
}

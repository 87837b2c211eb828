"""Textures on CPU: the oracle's restated sampler and UV maps, and the host-side
texture packing.  PARITY UNPINNED for the sampler: the reference samples with
read_imagef, which gfx950 cannot execute (no image instructions; DESIGN.md
"Textures"), so there is no reference output to pin it to.  What is pinned:

* the sampler against hand-computed values of the OpenCL 1.2 s8.2 formulas
  (CLK_NORMALIZED_COORDS_TRUE | CLK_ADDRESS_REPEAT | CLK_FILTER_LINEAR, tracer.cl:829);
* sphericalMap against the reference's own known answers for its Go twin
  (internal/app/shapes/sphericalmap_test.go:13-21) -- within 1e-7, because the
  kernel's PI is the FLOAT literal 3.14159265359f (tracer.cl:1) where Go uses math.Pi;
* cubeUV's face choice against FaceFromPoint's known answers
  (internal/app/shapes/cubemap_test.go:17-24: 0 right, 1 left, 2 up, 3 down,
  4 front, 5 back -- the branch order of tracer.cl:153-172).
"""
import math

import numpy as np
import pytest

import pyoracle
from ptmi import layout
from ptmi.textures import TextureSet
from tests import textures_synth
from tests.scene_inputs import scene_inputs

PI_F = float(np.float32(3.14159265359))


def _img(rgb_rows):
    a = np.array(rgb_rows, dtype=np.uint8)
    out = np.full(a.shape[:2] + (4,), 255, np.uint8)
    out[..., :3] = a
    return out


RED, GREEN, BLUE, WHITE = (255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 255)
TEX2 = _img([[RED, GREEN], [BLUE, WHITE]])


@pytest.mark.parametrize("s,t,layer,want", [
    (0.25, 0.25, 0, (1.0, 0.0, 0.0)),      # texel centre (0,0): weight 1
    (0.75, 0.25, 0, (0.0, 1.0, 0.0)),      # texel (1,0)
    (0.25, 0.75, 0, (0.0, 0.0, 1.0)),      # texel (0,1): row 1 = second Pix row
    (0.5, 0.5, 0, (0.5, 0.5, 0.5)),        # the four-texel average
    (0.0, 0.0, 0, (0.5, 0.5, 0.5)),        # REPEAT: i0 = -1 wraps to 1
    (1.25, -0.75, 0, (1.0, 0.0, 0.0)),     # REPEAT of (0.25, 0.25)
    (0.25, 0.25, 7, (1.0, 0.0, 0.0)),      # layer clamp(rint(7), 0, n-1)
    (0.5, 0.25, 0, (0.5, 0.5, 0.0)),       # horizontal half
])
def test_sampler_known_answers(s, t, layer, want):
    got = pyoracle.tex_sample([TEX2], s, t, layer)
    assert np.allclose(got, want, rtol=0, atol=1e-7), got


def test_sampler_layers_and_unorm():
    a = _img([[(10, 20, 30)]])
    b = _img([[(200, 100, 50)]])
    assert np.allclose(pyoracle.tex_sample([a, b], 0.3, 0.9, 1.4), np.array([200, 100, 50]) / 255.0, atol=1e-7)
    assert np.allclose(pyoracle.tex_sample([a, b], 0.3, 0.9, 0.49), np.array([10, 20, 30]) / 255.0, atol=1e-7)
    # rint rounds half to even: 0.5 -> layer 0, 1.5 -> layer 2 -> clamped to 1
    assert np.allclose(pyoracle.tex_sample([a, b], 0.3, 0.9, 0.5), np.array([10, 20, 30]) / 255.0, atol=1e-7)
    assert pyoracle.tex_sample([], 0.3, 0.3, 0) == (0.0, 0.0, 0.0)  # the all-zero fake image


def test_sampler_bilinear_weights():
    """A 4x1 ramp: linear interpolation between texel centres, wrapping at 0/1."""
    ramp = _img([[(0, 0, 0), (85, 0, 0), (170, 0, 0), (255, 0, 0)]])
    for s in np.linspace(0.125, 0.875, 13):
        u = s * 4 - 0.5
        i0 = math.floor(u)
        a = u - i0
        want = ((1 - a) * ramp[0, i0, 0] + a * ramp[0, min(i0 + 1, 3), 0]) / 255.0
        assert abs(pyoracle.tex_sample([ramp], float(s), 0.5, 0)[0] - want) < 1e-6
    # between the last and the first texel centre the filter wraps around
    got = pyoracle.tex_sample([ramp], 0.0, 0.5, 0)[0]
    assert abs(got - 0.5 * (255 + 0) / 255.0) < 1e-6


@pytest.mark.parametrize("p,u,v", [
    ((0, 0, -1), 0.0, 0.5), ((1, 0, 0), 0.25, 0.5), ((0, 0, 1), 0.5, 0.5), ((-1, 0, 0), 0.75, 0.5),
    ((0, 1, 0), 0.5, 1.0), ((0, -1, 0), 0.5, 0.0), ((math.sqrt(2.0) / 2.0, math.sqrt(2.0) / 2.0, 0), 0.25, 0.75),
])
def test_spherical_map_known_answers(p, u, v):
    gu, gv = pyoracle.spherical_map(*p)
    assert abs(gu - u) < 1e-7 and abs(gv - v) < 1e-7, (gu, gv)
    # ... and exactly the kernel formula with the float PI (tracer.cl:178-213)
    theta = math.atan2(p[0], p[2])
    phi = math.acos(p[1] / math.sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]))
    assert gu == 1 - (theta / (2.0 * PI_F) + 0.5) and gv == 1 - phi / PI_F


@pytest.mark.parametrize("p,face", [((-1, 0.5, -0.25), 1), ((1.1, -0.75, 0.8), 0), ((0.1, 0.6, 0.9), 4),
                                    ((-0.7, 0, -2), 5), ((0.5, 1, 0.9), 2), ((-0.2, -1.3, 1.1), 3)])
def test_cube_uv_faces(p, face):
    """FaceFromPoint known answers -> the cross cell the kernel's uv lands in."""
    u, v = pyoracle.cube_uv(*p)
    cell = {0: (2, 1), 1: (0, 1), 2: (1, 2), 3: (1, 0), 4: (1, 1), 5: (3, 1)}[face]
    assert cell[0] * 0.25 <= u <= (cell[0] + 1) * 0.25 + 1e-12, (u, v)
    assert cell[1] / 3.0 - 1e-6 <= v <= (cell[1] + 1) / 3.0 + 1e-6, (u, v)


def test_cube_uv_formula():
    """cubeUVRightCross etc. (tracer.cl:113-148) literally, for a point per face."""
    x, y, z = 1.0, 0.3, -0.4
    u, v = pyoracle.cube_uv(x, y, z)
    assert u == 0.5 + math.fmod(1.0 - z, 2) / 2.0 * 0.25
    assert v == 0.6666666 - math.fmod(y + 1.0, 2) / 2.0 * 0.333333
    x, y, z = 0.2, -0.1, -1.0  # back
    u, v = pyoracle.cube_uv(x, y, z)
    assert u == 0.75 + math.fmod(1.0 - x, 2) / 2.0 * 0.25


def test_texture_set_packing():
    a = textures_synth.checker(8, 6, 2, (0, 0, 0), (255, 255, 255))
    ts = TextureSet([a, a], None, [a])
    assert list(ts.struct.count) == [2, 0, 1] and list(ts.struct.width) == [8, 0, 8]
    assert list(ts.struct.height) == [6, 0, 6] and ts.pointer() is not None
    assert TextureSet().pointer() is None
    with pytest.raises(ValueError):
        TextureSet([a, textures_synth.checker(6, 6, 2, (0, 0, 0), (1, 1, 1))])
    with pytest.raises(TypeError):
        TextureSet([a[..., :3]])


def test_textured_scene_records():
    """TexturedPlanetsScene records (texturedplanets.go:13-135): flags, indices, scales."""
    objs, _, _, _ = scene_inputs("textures", 16, 12)
    assert list(objs["is_textured"]) == [0, 0, 1, 1, 1, 1, 1, 1, 1]
    assert list(objs["texture_index"]) == [0, 0, 1, 2, 0, 0, 0, 1, 0]
    assert list(objs["is_textured_nm"]) == [0, 0, 0, 0, 1, 1, 1, 0, 0]
    assert list(objs["texture_index_nm"][4:7]) == [3, 3, 3]
    assert objs["texture_scale_x"][2] == 0.25 and objs["texture_scale_y_nm"][4] == 1.0
    o, _, _, _ = scene_inputs("cubemap", 16, 12)
    assert o["type"][2] == 3 and o["is_textured"][2] == 1 and o["is_env_map"][2] == 1


def _uniform(rgb, w=5, h=3, n=1):
    return [np.tile(np.array(list(rgb) + [255], np.uint8), (h, w, 1)) for _ in range(n)]


@pytest.mark.parametrize("scene", ["textures", "envmap"])
def test_oracle_uniform_texture_equals_object_colour(scene):
    """A texture of one colour c renders like the untextured object with colour
    float(c/255): colour textures never change a path (no RNG draw, no direction),
    only the bounce colour -- up to the filter weights' FP32 rounding."""
    w, h, spp = 24, 16, 2
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    seeds = layout.seeds_go_float64(w * h, 3)
    c = (51, 153, 204)
    tex = [_uniform(c, n=4), _uniform(c, 7, 4, n=2), None]
    plain = objs.copy()
    col = np.float32(np.array(c) / 255.0).astype(np.float64)
    for i in range(len(plain)):
        if plain["is_textured"][i] and plain["type"][i] in (0, 1, 3):
            plain["color"][i][:3] = col
            plain["color"][i][3] = 1.0
            plain["is_textured"][i] = 0
    plain["is_textured_nm"] = 0
    objs_nonm = objs.copy()
    objs_nonm["is_textured_nm"] = 0
    t2, g2 = layout.pad_empty(tris, grps)
    a = pyoracle.cpu_trace(objs_nonm, t2, g2, cam, spp, seeds, textures=tex)
    b = pyoracle.cpu_trace(plain, t2, g2, cam, spp, seeds)
    assert np.abs(a - b).max() < 1e-5
    assert np.abs(a - pyoracle.cpu_trace(objs_nonm, t2, g2, cam, spp, seeds)).max() > 1e-3  # textures matter


def test_oracle_textured_scene_deterministic_and_finite():
    w, h, spp = 24, 16, 2
    objs, tris, grps, cam = scene_inputs("textures", w, h)
    seeds = layout.seeds_go_float64(w * h, 4)
    tex = textures_synth.scene_textures("textures")
    t2, g2 = layout.pad_empty(tris, grps)
    a = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, textures=tex)
    b = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, textures=tex)
    assert np.array_equal(a, b) and np.isfinite(a).all()

"""GPU parity: the HIP path (libptmi.so, via its C ABI) against
  1. the golden vectors made by the reference kernel itself (tests/golden),
  2. the reference kernel run live on the same GPU (oracle/_ref, HSA launch),
  3. the CPU oracle restatement (oracle/pt_oracle.c),
plus invariances the multi-GPU splits rely on (sample split, tile split,
chunking) and the boundary's error behaviour.

Tolerance: the north_star bar, L-inf < 1e-4 per channel.  The kernel uses the
same device-library math as the reference build, so the observed error is
expected to be ~0 (reported in the assertion messages).
"""
import numpy as np
import pytest

import pyoracle
from ptmi import api, layout
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _render(scene, w, h, spp, seeds, ap=0.0, fl=0.0):
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    return api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)


GOLDEN = ["ref_64x48_s4", "ref_64x48_s16", "ref_40x30_s3", "ref_dof_64x48_s8", "ocl_64x48_s8", "ocl_dof_48x32_s5",
          "teapot_32x24_s4", "gopher_32x24_s4", "ref_160x120_s4", "transp_48x32_s6", "transp_quad_48x32_s4",
          "transp_f_dof_48x32_s5", "reflect_48x32_s6", "glassteapot_32x24_s4"]


@pytest.mark.parametrize("name", GOLDEN)
def test_hip_matches_reference_golden(golden_cases, name):
    if name not in golden_cases:
        pytest.skip("golden %s not generated" % name)
    z = golden_cases[name]
    out = _render(str(z["scene"]), int(z["width"]), int(z["height"]), int(z["samples"]), z["seeds"],
                  float(z["aperture"]), float(z["focal_length"]))
    err = np.abs(out - z["rgba"]).max()
    assert err < TOL, "%s: L-inf %.3e vs reference kernel" % (name, err)
    # Same device-library math as the reference build: agreement is at the level
    # of FP64 rounding (any semantic slip moves a pixel by ~1/spp).
    assert err < 1e-12, "%s: L-inf %.3e (expected rounding-level agreement)" % (name, err)


@pytest.mark.parametrize("scene,w,h,spp,ap,fl,seed", [
    ("reference", 96, 64, 6, 0.0, 0.0, 101),
    ("reference", 72, 40, 5, 0.15, 1.6, 102),
    ("default", 64, 64, 6, 0.0, 0.0, 103),
    ("teapot", 48, 32, 3, 0.0, 0.0, 104),
    ("gopher", 48, 32, 2, 0.0, 0.0, 105),
    ("teapot", 128, 96, 4, 0.0, 0.0, 106),
    ("gopher", 128, 96, 3, 0.0, 0.0, 107),
    ("teapot", 96, 64, 3, 0.15, 1.6, 108),
    ("reflection", 96, 64, 6, 0.0, 0.0, 109),
    ("transparency", 96, 64, 6, 0.0, 0.0, 110),
    ("transparency", 72, 48, 5, 0.15, 1.6, 111),
    ("transparency_f_light", 96, 64, 4, 0.0, 0.0, 112),
    ("transparency_quad_lights", 96, 64, 4, 0.0, 0.0, 113),
    ("transparent_teapot", 96, 64, 4, 0.0, 0.0, 114),
    ("transparent_teapot", 64, 48, 3, 0.15, 1.6, 115),
    ("gopher-window", 96, 64, 3, 0.0, 0.0, 116),
    ("christian", 96, 64, 3, 0.0, 0.0, 117),
    ("christian", 64, 48, 3, 0.15, 1.6, 118),
])
def test_hip_matches_live_reference(scene, w, h, spp, ap, fl, seed):
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    seeds = layout.seeds_go_float64(w * h, seed)
    t2, g2 = layout.pad_empty(tris, grps)
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ref).max()
    assert err < TOL, "%s: L-inf %.3e vs live reference" % (scene, err)
    assert err < 1e-12, "%s: L-inf %.3e (expected rounding-level agreement)" % (scene, err)


def _paths(objs, tris, grps, cam, spp, seeds, force=None):
    """Every (pixel, sample) path's colour: one-sample renders [n, n + 1) of the spp-sample
    frame, so no sum is formed.  The affine mesh kernels add a pixel's paths in completion
    order (the path pool, ptmi_kernels.hip trace_groups_pool) and the generic ones in sample
    order, so their frames differ in FP64 summation order; the paths must not differ at all."""
    import contextlib
    import torch
    c = np.asarray(cam).reshape(())
    w, h = int(c["width"]), int(c["height"])
    with (api.force_flags(force) if force is not None else contextlib.nullcontext()):
        sc = api.Scene(0, objs, tris, grps, cam)
    sd = torch.tensor(seeds, dtype=torch.float64, device="cuda")
    out = torch.empty((spp, w * h * 4), dtype=torch.float64, device="cuda")
    for n in range(spp):
        sc.render(spp, n, n + 1, sd.data_ptr(), out[n].data_ptr())
    torch.cuda.synchronize()
    sc.close()
    return out.cpu().numpy()


@pytest.mark.parametrize("force", ["15", "31"])
@pytest.mark.parametrize("scene,ap", [("reference", 0.0), ("default", 0.15), ("teapot", 0.0), ("gopher", 0.0)])
def test_generic_instantiation_matches(scene, ap, force):
    """The feature-specialised kernel instantiation and the generic ones give
    identical images: 15 = all features compiled in (affine), 31 = all features
    with the literal double4 w-lane arithmetic (the path for non-affine scenes).
    Mesh scenes against 31 compare every path (_paths): identical bit for bit."""
    w, h, spp = 40, 24, 3
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, 1.6 if ap else 0.0)
    seeds = layout.seeds_go_float64(w * h, 77)
    spec = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    with api.force_flags(int(force)):  # ptmi_diag_force_flags
        gen = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    if len(grps) and force == "31":
        assert np.abs(spec - gen).max() < 1e-15
        assert np.array_equal(_paths(objs, tris, grps, cam, spp, seeds), _paths(objs, tris, grps, cam, spp, seeds, 31))
    else:
        assert np.array_equal(spec, gen)


@pytest.mark.parametrize("scene,ap", [("reference", 0.0), ("reference", 0.15), ("teapot", 0.0)])
def test_affine_cores_match_generic_large(scene, ap):
    """The affine instantiations' divide / sqrt / rsqrt cores (csrc/ptmi_fp64core.h)
    against the generic instantiation's full compiler expansions over a larger
    frame: 160x120 at 24 spp (~1.8 M paths), images bit-identical (the teapot: every
    path bit-identical, the frames up to the path pool's summation order)."""
    w, h, spp = 160, 120, 24
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, 1.6 if ap else 0.0)
    seeds = layout.seeds_go_float64(w * h, 91)
    spec = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    with api.force_flags(31):
        gen = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    if len(grps):
        assert np.abs(spec - gen).max() < 1e-14
        assert np.array_equal(_paths(objs, tris, grps, cam, spp, seeds), _paths(objs, tris, grps, cam, spp, seeds, 31))
    else:
        assert np.array_equal(spec, gen)


@pytest.mark.parametrize("scene,w,h,spp,ap,fl,seed", [
    ("reference", 24, 16, 1300, 0.0, 0.0, 201),
    ("reference", 16, 16, 1200, 0.15, 1.6, 202),
    ("teapot", 16, 12, 1100, 0.0, 0.0, 203),
    ("gopher", 16, 12, 900, 0.0, 0.0, 204),
    # glass: noise3D(fgi, n*n, b) puts arguments far above 2^19 -> ocml's own sin (out of line)
    ("transparency", 16, 12, 400, 0.0, 0.0, 205),
    ("transparent_teapot", 16, 12, 300, 0.0, 0.0, 206),
])
def test_hip_matches_live_reference_high_sample_indices(scene, w, h, spp, ap, fl, seed):
    """Sample indices past ~550 put the noise's sin arguments above 2^17, onto the
    large-argument reduction (csrc/ptmi_sinf.h); short frames never reach it.  Small
    images at ~1000 spp against the live reference kernel: any noise bit off moves a
    pixel by ~1/spp, far above the 1e-12 asserted."""
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    seeds = layout.seeds_go_float64(w * h, seed)
    t2, g2 = layout.pad_empty(tris, grps)
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ref).max()
    assert err < 1e-12, "%s: L-inf %.3e vs live reference at %d spp" % (scene, err, spp)


def test_untame_scene_matches_cpu_oracle():
    """A sphere scaled by 2^-70 (inverse entries 2^70, outside the tame-scene bound of
    ptmi_api.cpp) sends the scene to the generic instantiation with the compiler's full
    divide / sqrt / normalize expansions; the image still matches the oracle."""
    from ptmi import geom, layout as lay, scenes, shapes
    w, h, spp = 40, 32, 4
    sc = scenes.reference_scene(w, h)
    tiny = shapes.Sphere()
    tiny.set_transform(geom.translate(0.1, 0.1, -0.2))
    tiny.set_transform(geom.scale(2.0 ** -70, 2.0 ** -70, 2.0 ** -70))
    tiny.set_material(shapes.new_diffuse(0.5, 0.5, 0.5))
    objs, tris, grps = lay.build_scene_buffer_cl(sc.objects + [tiny])
    cam = lay.camera_record(sc.camera)
    seeds = layout.seeds_go_float64(w * h, 5)
    t2, g2 = layout.pad_empty(tris, grps)
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(out - ora).max() < TOL


def test_hip_matches_cpu_oracle_odd_size():
    w, h, spp = 37, 23, 7   # not a multiple of the 8x8 tile
    objs, tris, grps, cam = scene_inputs("default", w, h)
    seeds = layout.seeds_go_float64(w * h, 7)
    t2, g2 = layout.pad_empty(tris, grps)
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(out - ora).max() < TOL


def test_trace_generated_seeds_deterministic():
    objs, tris, grps, cam = scene_inputs("reference", 32, 24)
    a = api.Trace(objs, tris, grps, 0, 3, cam, seed_stream=42)
    b = api.Trace(objs, tris, grps, 0, 3, cam, seed_stream=42)
    c = api.Trace(objs, tris, grps, 0, 3, cam, seed_stream=43)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert np.all(a[3::4] == 1.0) and np.isfinite(a).all()


def _torch_scene(scene, w, h, ap=0.0, fl=0.0):
    import torch
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    sc = api.Scene(0, objs, tris, grps, cam)
    return torch, sc


def test_sample_split_and_chunking_invariance():
    torch, sc = _torch_scene("reference", 64, 48, 0.15, 1.6)
    S, n = 12, 64 * 48
    seeds = torch.tensor(layout.seeds_go_float64(n, 9), dtype=torch.float64, device="cuda")
    full = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    sc.render(S, 0, S, seeds.data_ptr(), full.data_ptr(), chunks=1)
    acc = torch.zeros_like(full)
    part = torch.empty_like(full)
    for a, b in ((0, 5), (5, 6), (6, 12)):
        sc.render(S, a, b, seeds.data_ptr(), part.data_ptr(), chunks=3)
        acc += part
    torch.cuda.synchronize()
    assert torch.all(acc[3::4] == S)
    assert (acc - full).abs().max().item() < 1e-12
    chunked = torch.empty_like(full)
    sc.render(S, 0, S, seeds.data_ptr(), chunked.data_ptr(), chunks=5)
    torch.cuda.synchronize()
    assert (chunked - full).abs().max().item() < 1e-12


def test_mesh_plan_short_last_round():
    """A mesh scene's automatic plan cuts its last chunk round into shorter chunks
    (KNOB_TAIL_SPLIT, ptmi_api.cpp render; here forced on a small frame through 128-sample
    chunks): the frame equals the uniform plan's up to FP64 summation order, with every
    pixel's sample count exact, and equals the whole-tile render likewise."""
    torch, sc = _torch_scene("teapot", 64, 48, 0.0, 0.0)
    S, n = 600, 64 * 48
    seeds = torch.tensor(layout.seeds_go_float64(n, 12), dtype=torch.float64, device="cuda")
    frames = []
    for ts in (1, 2, 3):
        assert sc.set_knob(api.KNOB_MIN_CHUNK, 128) == api.PTMI_OK
        assert sc.set_knob(api.KNOB_TAIL_SPLIT, ts) == api.PTMI_OK
        f = torch.empty(n * 4, dtype=torch.float64, device="cuda")
        sc.render(S, 0, S, seeds.data_ptr(), f.data_ptr())
        frames.append(f)
    whole = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    sc.render(S, 0, S, seeds.data_ptr(), whole.data_ptr(), chunks=1)
    torch.cuda.synchronize()
    sc.close()
    for f in frames:
        assert torch.all(f[3::4] == S)
        assert (f - whole).abs().max().item() < 1e-12 * S
    assert not torch.equal(frames[0], frames[1])  # the split plan sums other partials


@pytest.mark.parametrize("scene,stride", [("reference", 1), ("reference", 3), ("teapot", 1), ("teapot", 2)])
def test_whole_tiles_and_chunked_tail(scene, stride):
    """Automatic work plan (ptmi_device.h WorkPlan): whole-tile items first, the last
    tiles in sample chunks.  The TAIL_TILES knob shrinks the chunked tail so a small frame
    has both kinds; the frame equals the all-whole render (chunks=1) and each tile-split
    part is zero outside its tiles."""
    torch, sc = _torch_scene(scene, 72, 40)
    assert sc.set_knob(api.KNOB_TAIL_TILES, 5) == api.PTMI_OK
    S, n = 70, 72 * 40  # 45 tiles (the last column and row partial)
    seeds = torch.tensor(layout.seeds_go_float64(n, 11), dtype=torch.float64, device="cuda")
    whole = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    sc.render(S, 0, S, seeds.data_ptr(), whole.data_ptr(), chunks=1)
    acc = torch.zeros_like(whole)
    part = torch.empty_like(whole)
    for g in range(stride):
        sc.render(S, 0, S, seeds.data_ptr(), part.data_ptr(), tile_stride=stride, tile_offset=g)
        acc += part
    torch.cuda.synchronize()
    assert torch.all(acc[3::4] == S)
    assert (acc - whole).abs().max().item() < 1e-12
    assert torch.all(torch.isfinite(acc))


@pytest.mark.parametrize("scene", ["teapot", "gopher"])
def test_mesh_hemisphere_table_switch(scene):
    """The mesh kernels read the hemisphere table unless the scene switches it off
    (DevScene::hemi_mesh, PTMI_KNOB_HEMI_MESH: a traffic / time trade-off on large meshes).
    The table holds the bits the kernel computes, so either way the frame is the same, bit
    for bit."""
    torch, sc = _torch_scene(scene, 64, 48)
    S, n = 40, 64 * 48
    seeds = torch.tensor(layout.seeds_go_float64(n, 21), dtype=torch.float64, device="cuda")
    frames = []
    for v in (0, 1):
        assert sc.set_knob(api.KNOB_HEMI_MESH, v) == api.PTMI_OK
        f = torch.empty(n * 4, dtype=torch.float64, device="cuda")
        sc.render(S, 0, S, seeds.data_ptr(), f.data_ptr())
        frames.append(f)
    torch.cuda.synchronize()
    sc.close()
    assert torch.equal(frames[0], frames[1])


def test_tile_split_partitions_frame():
    torch, sc = _torch_scene("teapot", 40, 24)
    S, n = 3, 40 * 24
    seeds = torch.tensor(layout.seeds_go_float64(n, 10), dtype=torch.float64, device="cuda")
    full = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    sc.render(S, 0, S, seeds.data_ptr(), full.data_ptr())
    acc = torch.zeros_like(full)
    part = torch.empty_like(full)
    G = 3
    for g in range(G):
        sc.render(S, 0, S, seeds.data_ptr(), part.data_ptr(), tile_stride=G, tile_offset=g)
        acc += part
    torch.cuda.synchronize()
    assert torch.equal(acc, full)


@pytest.mark.parametrize("scene,stride", [("teapot", 4), ("gopher", 8), ("teapot", 3)])
def test_mesh_tile_split_ownership(scene, stride):
    """Tile split of an affine mesh scene (ptmi_api.cpp render): diagonal ownership through
    the F_TLIST kernels when the tile rows divide by the stride (16 tiles per row: 4 and 8),
    raster striding otherwise (3).  Each rank's frame holds exactly its tiles (A = S there,
    zeros elsewhere, as ptmi/dist.py's tile_owner_mask predicts) and the shards sum to the
    one-launch frame bit for bit (same chunks per tile in every launch; the mesh kernels' path
    pool runs an item the same way in the F_TLIST kernels and the one-GPU ones), and a second
    launch of a share is identical (the pool is deterministic)."""
    from ptmi import dist as pdist
    W, H, S = 128, 48, 24
    torch, sc = _torch_scene(scene, W, H)
    seeds = torch.tensor(layout.seeds_go_float64(W * H, 12), dtype=torch.float64, device="cuda")
    full = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
    sc.render(S, 0, S, seeds.data_ptr(), full.data_ptr(), chunks=3)
    acc = torch.zeros_like(full)
    part = torch.empty_like(full)
    diag = sc.tile_ownership(stride) == "diagonal"  # the library's decision (ptmi_diag_tile_ownership)
    assert diag == (stride != 3) == pdist.diagonal_ownership(W, stride, True)
    for g in range(stride):
        sc.render(S, 0, S, seeds.data_ptr(), part.data_ptr(), tile_stride=stride, tile_offset=g, chunks=3)
        torch.cuda.synchronize()
        mask = torch.tensor(pdist.tile_owner_mask(W, H, stride, g, diag).reshape(-1), device="cuda")
        p4 = part.view(-1, 4)
        assert torch.all(p4[mask, 3] == S) and torch.all(p4[~mask] == 0)
        acc += part
        if diag:
            again = torch.empty_like(part)
            sc.render(S, 0, S, seeds.data_ptr(), again.data_ptr(), tile_stride=stride, tile_offset=g, chunks=3)
            torch.cuda.synchronize()
            assert torch.equal(again, part)
    assert torch.equal(acc, full)  # same chunks per tile in every launch: bit for bit
    sc.close()


def test_errors_are_loud():
    objs, tris, grps, cam = scene_inputs("reference", 8, 8)
    with pytest.raises(api.PtmiError) as e:
        api.Trace(objs, tris, grps, 99, 1, cam)
    assert e.value.code == api.PTMI_ERR_DEVICE
    with pytest.raises(api.PtmiError):
        api.Trace(np.concatenate([objs, objs, objs]), tris, grps, 0, 1, cam)  # 24 > 16 objects
    # device index < 0 selects device 0 (ocltracer.go:138-140)
    out = api.Trace(objs, tris, grps, -1, 1, cam, seed_stream=1)
    assert out.shape == (8 * 8 * 4,)


@pytest.mark.parametrize("kind", ["flat", "stairs", "dupes", "far"])
@pytest.mark.parametrize("ap", [0.0, 0.15])
def test_hip_matches_live_reference_adversarial_bvh(kind, ap):
    """Meshes built to break the BVH exactness arguments (tests/adversarial.py):
    zero-thickness reference boxes, shared edges, exact t ties, traversal bounds past
    binary16's range."""
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    from tests import adversarial
    w, h, spp = 96, 64, 4
    objs, tris, grps, cam = adversarial.scene_inputs(kind, w, h, ap, 1.6 if ap else 0.0)
    seeds = layout.seeds_go_float64(w * h, 300 + len(tris))
    t2, g2 = layout.pad_empty(tris, grps)
    _assert_ref_defined(objs, t2, g2, cam, spp, seeds)
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ref).max()
    assert err < 1e-12, "%s: L-inf %.3e vs live reference" % (kind, err)


def _assert_ref_defined(objs, t2, g2, cam, spp, seeds):
    """A live-reference case must stay inside the reference kernel's 64-entry ctx arrays
    (tracer.cl:97-99): past them its behaviour is undefined (it faults the GPU).  Checked
    on the CPU before the reference kernel is launched."""
    n = pyoracle.max_candidates(objs, t2, g2, cam, spp, seeds)
    assert 0 < n <= 64, "%d candidates on one line: past the reference's ctx arrays" % n


def test_hip_matches_live_reference_wide_child_codes():
    """A mesh past 16-bit child codes (tests/adversarial.py "big", 34,848 triangles) takes
    the wide codes and the affine F_WIDE instantiation's 32-bit traversal stack (round 6; it
    had been sent to the generic instantiation; it takes the path pool too): still the
    reference's image, and every path the generic instantiation's bit for bit (_paths; the
    frames differ only in the pool's summation order)."""
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    from tests import adversarial
    w, h, spp = 64, 48, 2
    objs, tris, grps, cam = adversarial.scene_inputs("big", w, h)
    assert api.index_stats(objs, tris, grps, cam)["leaf_bit"] == 0x40000000
    sc = api.Scene(0, objs, tris, grps, cam)
    assert sc.kernel_flags() == 15 | 256  # F_ALL | F_WIDE: affine, 32-bit stack
    assert sc.tile_ownership(8) == "raster"  # no F_TLIST instantiation for wide codes
    sc.close()
    seeds = layout.seeds_go_float64(w * h, 404)
    t2, g2 = layout.pad_empty(tris, grps)
    _assert_ref_defined(objs, t2, g2, cam, spp, seeds)
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ref).max()
    assert err < 1e-12, "big: L-inf %.3e vs live reference" % err
    with api.force_flags(31):  # the generic instantiation (literal double4 arithmetic)
        gen = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(out - gen).max() < 1e-15
    assert np.array_equal(_paths(objs, tris, grps, cam, spp, seeds), _paths(objs, tris, grps, cam, spp, seeds, 31))


def test_wide_code_scene_statistical_rng():
    """The statistical RNG mode on a wide-code mesh scene (F_WIDE | F_XRNG): allowed since the
    scene stays on the affine kernels, deterministic, and back to the parity image when switched off."""
    import torch
    from tests import adversarial
    w, h, spp = 64, 48, 2
    objs, tris, grps, cam = adversarial.scene_inputs("big", w, h)
    sc = api.Scene(0, objs, tris, grps, cam)
    seeds = torch.tensor(layout.seeds_go_float64(w * h, 404), dtype=torch.float64, device="cuda")
    out = torch.empty(w * h * 4, dtype=torch.float64, device="cuda")

    def frame():
        sc.render(spp, 0, spp, seeds.data_ptr(), out.data_ptr())
        torch.cuda.synchronize()
        return out.clone()

    par = frame()
    sc.set_rng(api.RNG_XOSHIRO)
    assert sc.kernel_flags() == 15 | 256 | 64
    x1, x2 = frame(), frame()
    assert torch.equal(x1, x2) and not torch.equal(x1, par)
    sc.set_rng(api.RNG_NOISE3D)
    assert torch.equal(frame(), par)
    sc.close()


def test_hip_matches_oracle_past_reference_ctx():
    """The bumpy 34,848-triangle height field (tests/adversarial.py "bumpy"): lines along it
    meet up to ~200 triangles, past the reference's 64-entry ctx arrays, where the reference
    kernel is undefined (it faults).  ptmi streams the candidates, as the CPU oracle does:
    the two images agree."""
    from tests import adversarial
    w, h, spp = 64, 48, 2
    objs, tris, grps, cam = adversarial.scene_inputs("bumpy", w, h)
    seeds = layout.seeds_go_float64(w * h, 404)
    t2, g2 = layout.pad_empty(tris, grps)
    assert pyoracle.max_candidates(objs, t2, g2, cam, spp, seeds) > 64
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ora).max()
    assert err < 1e-12, "bumpy: L-inf %.3e vs the CPU oracle" % err


@pytest.mark.parametrize("offset,scale", [((1.0e4, 0.0, 0.0), 1.0), ((-3.0e4, 2.0e4, 7.5e3), 1.0),
                                          ((1.0e9, 0.0, -2.0e9), 3.0e5)])
def test_hip_matches_live_reference_moved_mesh(offset, scale):
    """The teapot moved in its object space far from the origin and / or scaled past
    binary16's range (tests/moved_mesh.py): the traversal index's per-root frame
    (ptmi_bvh.cpp RootRec ctr / sc) must stay conservative."""
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    from tests.moved_mesh import moved
    w, h, spp = 64, 48, 3
    objs, tris, grps, cam = scene_inputs("teapot", w, h)
    objs, tris, grps = moved(objs, tris, grps, offset=offset, scale=scale)
    seeds = layout.seeds_go_float64(w * h, 640)
    ref = pyoracle.ref_trace(objs, tris, grps, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    err = np.abs(out - ref).max()
    assert err < 1e-12, "offset %s scale %g: L-inf %.3e vs live reference" % (offset, scale, err)


@pytest.mark.parametrize("scene,ap", [("transparency", 0.0), ("transparency_quad_lights", 0.15),
                                      ("reflection", 0.0), ("transparent_teapot", 0.0)])
def test_cpu_oracle_matches_live_reference_materials(scene, ap):
    """The CPU oracle's material paths (refraction, thin glass, mirrors) against
    the reference kernel itself -- the goldens pin the rest of the oracle."""
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built")
    w, h, spp = 32, 24, 3
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, 1.6 if ap else 0.0)
    seeds = layout.seeds_go_float64(w * h, 500)
    t2, g2 = layout.pad_empty(tris, grps)
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds)
    assert np.abs(ora - ref).max() < 1e-12



@pytest.mark.parametrize("scene,w,h,spp,split,ndev", [("reference", 40, 24, 5, "tile", 2),
                                                       ("teapot", 40, 24, 5, "tile", 3),
                                                       ("reference", 40, 24, 5, "sample", 2),
                                                       ("transparency", 40, 24, 5, "sample", 3),
                                                       ("reference", 8, 8, 1500, "sample", 8),
                                                       ("gopher", 64, 48, 4, "tile", 8)])
def test_trace_multi_matches_single_device(scene, w, h, spp, split, ndev):
    """ptmi_trace_multi with device 0 repeated (this box has one GPU): host scene
    prepared once, device-side combine (peer copies into a gather buffer, ordered sum).
    The tile split is bit-identical to ptmi_trace, the sample split equal up to FP64
    summation order; 1500 spp over 8 devices crosses both cost knots of the split."""
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    seeds = layout.seeds_go_float64(w * h, 61)
    single = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    out, timing = api.TraceMulti(objs, tris, grps, [0] * ndev, split, spp, cam, seeds=seeds)
    if split == "tile":
        assert np.array_equal(out, single)
    else:
        assert np.abs(out - single).max() < 1e-12
    assert all(timing[k] >= 0 for k in timing) and timing["total_ms"] >= timing["render_ms"]


def test_combine_frames_sums_distinct_slots_in_slot_order():
    """ptmi_combine_frames (the combine of ptmi_trace_multi) over 8 slots with distinct
    contents whose sum depends on the order of addition: equal bit for bit to the sums
    taken left to right in slot order, x (1.0 / S), alpha 1 (tracer.cl:1184-1187)."""
    import torch
    npix, nparts, S = 4096 + 37, 8, 1000
    rng = np.random.default_rng(5)
    # magnitudes spread over many binades, so FP64 addition is far from associative here
    parts = rng.standard_normal((nparts, npix, 4)) * np.exp2(rng.integers(-30, 30, (nparts, npix, 4)))
    parts[:, :, 3] = rng.integers(0, 300, (nparts, npix))
    want = parts[0, :, :3].copy()
    for k in range(1, nparts):
        want = want + parts[k, :, :3]
    want = want * (1.0 / S)
    shuffled = parts[::-1].sum(axis=0)[:, :3] * (1.0 / S)
    assert not np.array_equal(want, shuffled)  # the test can see an ordering error
    d = torch.tensor(parts.reshape(-1), dtype=torch.float64, device="cuda")
    out = torch.empty(npix * 4, dtype=torch.float64, device="cuda")
    api.combine_frames(d.data_ptr(), nparts, npix, out.data_ptr(), S)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(npix, 4)
    assert np.array_equal(got[:, :3], want)
    assert np.all(got[:, 3] == 1.0)
    api.combine_frames(d.data_ptr(), nparts, npix, d.data_ptr(), S)  # in place into slot 0
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().reshape(nparts, npix, 4)[0], got)

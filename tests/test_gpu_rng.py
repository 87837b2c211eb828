"""The reference RNG's float sin (tracer.cl:314-317 -> ocml __ocml_sin_f32):
exhaustive bit-identity of the oracle's restatement (oracle/ocml_sinf.h) and of
the kernel's own sin (csrc/ptmi_sinf.h) with the GPU device library, and replay
of ocml values on the host CPU (same code the CPU oracle runs)."""
import ctypes
import os

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu
LIB = os.path.join(os.path.dirname(__file__), "gpu_probe", "build", "libsinfprobe.so")


def _lib():
    if not os.path.exists(LIB):
        pytest.fail("probe library not built: %s (run __graft_entry__.build())" % LIB)
    import torch  # noqa: F401  one HIP runtime per process (ptmi/_runtime.py)
    lib = ctypes.CDLL(LIB)
    lib.probe_sinf_all.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint)]
    lib.probe_ptmi_sinf_all.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint)]
    lib.probe_fp64core.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_ulonglong)]
    lib.probe_sincos_core_all.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint)]
    for name in ("probe_ptmi_noise_sinf2_all", "probe_fract_all"):
        getattr(lib, name).argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint)]
    lib.probe_ptmi_noise_sinf_all.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint),
                                              ctypes.POINTER(ctypes.c_ulonglong)]
    lib.probe_sinf_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    return lib


def test_restated_sinf_bit_identical_all_floats():
    lib = _lib()
    m, f = ctypes.c_ulonglong(), ctypes.c_uint()
    assert lib.probe_sinf_all(ctypes.byref(m), ctypes.byref(f)) == 0
    assert m.value == 0, "%d mismatches, first input bits 0x%08x" % (m.value, f.value)


def test_kernel_sinf_bit_identical_below_2p19():
    """The kernel's noise sin (pathtracer-ocl_amd/csrc/ptmi_sinf.h: ocml's sin_f32 with
    the large-argument reduction specialised to 2^17 <= |x| < 2^19 and its four lowest
    2/pi table words dropped) equals the device library for every float |x| < 2^19."""
    lib = _lib()
    m, f = ctypes.c_ulonglong(), ctypes.c_uint()
    assert lib.probe_ptmi_sinf_all(ctypes.byref(m), ctypes.byref(f)) == 0
    assert m.value == 0, "%d mismatches, first input bits 0x%08x" % (m.value, f.value)


def test_kernel_noise_sinf_bit_identical_all_floats():
    """The kernel's whole noise sin as noise3d composes it (ptmi_sinf.h noise_sinf):
    sinf_lt19 below 2^19, the four-part FP64 Cody-Waite sinf_cw30 on [2^19, 2^30)
    (the glass noise's n*n arguments, and every noise past sample ~2210) with ocml's
    own sin on the lanes it declines, ocml above -- equal to the device library for
    every one of the 2^32 floats.  The number of declined lanes equals the exhaustive
    host check's (tools/sinf_check.cpp: 1054 of the 1.8e8 floats, both signs)."""
    lib = _lib()
    m, f, fb = ctypes.c_ulonglong(), ctypes.c_uint(), ctypes.c_ulonglong()
    assert lib.probe_ptmi_noise_sinf_all(ctypes.byref(m), ctypes.byref(f), ctypes.byref(fb)) == 0
    assert m.value == 0, "%d mismatches, first input bits 0x%08x" % (m.value, f.value)
    n_range = 2 * (0x4E800000 - 0x49000000)  # floats with 2^19 <= |x| < 2^30, both signs
    assert fb.value == 1054, "cw30 declined %d of %d lanes (host check: 1054)" % (fb.value, n_range)


def test_kernel_noise_sinf_pair_bit_identical_all_floats():
    """The paired noise sin the kernels evaluate a noise3D pair with (ptmi_sinf.h noise_sinf2,
    round 6): both outputs equal noise_sinf's (itself equal to the device library for every float,
    above) for every float in the first slot, each paired with another float drawn from the whole bit
    space -- every combination of reduction paths (small / Cody-Waite / Payne-Hanek band / >= 2^19)
    of the two draws occurs."""
    lib = _lib()
    m, f = ctypes.c_ulonglong(), ctypes.c_uint()
    assert lib.probe_ptmi_noise_sinf2_all(ctypes.byref(m), ctypes.byref(f)) == 0
    assert m.value == 0, "%d mismatches, first input bits 0x%08x" % (m.value, f.value)


def test_fract_instruction_matches_ocml_fract_all_floats():
    """v_fract_f32 against ocml's fract (min(x - floor(x), 0x1.fffffep-1f)) on every finite float:
    reported, and required only if the kernels use it (PTMI_R6_FRACT)."""
    lib = _lib()
    m, f = ctypes.c_ulonglong(), ctypes.c_uint()
    assert lib.probe_fract_all(ctypes.byref(m), ctypes.byref(f)) == 0
    print("v_fract_f32 vs ocml fract: %d mismatches (first 0x%08x)" % (m.value, f.value))
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "pathtracer-ocl_amd", "csrc", "ptmi_kernels.hip")).read()
    if re.search(r"#define PTMI_R6_FRACT 1", src):
        assert m.value == 0, "the kernels use v_fract_f32 but it differs from ocml's fract"


def test_fp64_cores_match_compiler_operators():
    """csrc/ptmi_fp64core.h: the divide / sqrt / rsqrt cores the affine kernels use
    return the bits of the compiler's x / y, sqrt and rsqrt on their ranges (2^28
    random operands per operation, uniform exponents, random mantissas)."""
    lib = _lib()
    m = (ctypes.c_ulonglong * 3)()
    assert lib.probe_fp64core(12345, 1 << 28, m) == 0
    assert list(m) == [0, 0, 0], "mismatches (div, sqrt, rsqrt): %s" % list(m)


def test_sincos_core_bit_identical_every_hemisphere_angle():
    """csrc/ptmi_fp64core.h sincos_core (ocml's sincos_f64 without its range steps)
    equals ocml's sincos for rand1 = 2 pi v at every float noise value v in [0, 1)."""
    lib = _lib()
    m, f = ctypes.c_ulonglong(), ctypes.c_uint()
    assert lib.probe_sincos_core_all(ctypes.byref(m), ctypes.byref(f)) == 0
    assert m.value == 0, "%d mismatches, first noise bits 0x%08x" % (m.value, f.value)


@pytest.mark.parametrize("scene", ["reference", "teapot"])
def test_hemisphere_table_generic_sequences_agree(scene):
    """The scene's hemisphere table (ptmi_kernels.hip hemi_table_kernel) holds the affine
    sequences' (sin, cos)(2 pi u), sqrt(u), sqrt(1 - u); the generic instantiations compute
    them with the full operators.  Every one of the 2^16 records must agree bit for bit
    (ptmi_diag_hemi_mismatch): the runtime tripwire for the affine specialisation."""
    from ptmi import api
    from tests.scene_inputs import scene_inputs
    objs, tris, grps, cam = scene_inputs(scene, 32, 24)
    sc = api.Scene(0, objs, tris, grps, cam)
    try:
        assert sc.hemi_mismatch() == 0
    finally:
        sc.close()


def test_cpu_restatement_replays_gpu_ocml():
    lib = _lib()
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-1e9, 1e9, 50000), rng.uniform(-200, 200, 50000),
                        rng.uniform(0, 8e8, 50000)]).astype(np.float32)
    gpu = np.empty_like(x)
    assert lib.probe_sinf_eval(x.ctypes.data, gpu.ctypes.data, x.size) == 0
    cpu = np.array([pyoracle.sinf(float(v)) for v in x[:20000]], dtype=np.float32)
    assert np.array_equal(cpu.view(np.uint32), gpu[:20000].view(np.uint32))

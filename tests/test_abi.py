"""The drop-in boundary on CPU (no GPU calls): libptmi.so loads, exports every
entry point include/ptmi.h declares with C linkage, carries gfx950 code, and the
record sizes the header promises are the reference's (ocltracer.go:25-96)."""
import os
import re
import subprocess

import pytest

from ptmi import api, layout

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "ptmi.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ptmi_[a-z_]+)\s*\(", src)))


def _lib_path():
    if not os.path.exists(api.LIB_PATH):
        pytest.fail("libptmi.so not built: run __graft_entry__.build() / make -C pathtracer-ocl_amd")
    return api.LIB_PATH


def test_header_declares_the_python_exports():
    assert _declared() == sorted(api.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in _declared() if s not in exported]
    assert not missing, "not exported with C linkage: %s" % missing


def test_library_exports_every_diagnostic_symbol():
    """include/ptmi_diag.h (diagnostics beside the boundary) is exported too."""
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "ptmi_diag.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(ptmi_diag_[a-z_]+)\s*\(", src)))
    assert len(declared) >= 7
    out = subprocess.run(["nm", "-D", "--defined-only", _lib_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in declared if s not in exported]
    assert not missing, "not exported with C linkage: %s" % missing


def test_product_library_holds_only_product_kernels():
    """The study kernels (standalone walks, the split form, the measured tile order) are in
    build/libptmi_study.so only: the product's kernels are trace_kernel<FL> and its helpers."""
    out = subprocess.run(["nm", "-D", "--defined-only", "-C", _lib_path()], capture_output=True, text=True,
                         check=True).stdout
    kernels = {k.replace("__device_stub__", "") for k in re.findall(r"ptmi::(\w+_kernel)\b", out)}
    assert "trace_kernel" in kernels
    assert kernels <= {"trace_kernel", "reduce_chunks_kernel", "finalize_kernel", "combine_kernel", "seeds_kernel",
                       "sunflower_kernel", "plane_normals_kernel", "hemi_table_kernel"}, sorted(kernels)


def test_product_library_reads_no_tuning_environment():
    """Plan and kernel choices come from the scene and the diag calls, never the environment:
    the only PTMI_* variable name in the product library is PTMI_VERBOSE."""
    names = set(re.findall(rb"PTMI_[A-Z0-9_]+", open(_lib_path(), "rb").read()))
    assert names <= {b"PTMI_VERBOSE"}, sorted(names)


def test_library_loads_and_identifies_gfx950():
    lib = api.load_library()
    for s in _declared():
        assert hasattr(lib, s)
    info = lib.ptmi_build_info().decode()
    assert "gfx950" in info, info
    blob = open(_lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded code object targets gfx950


def test_host_library_exports_every_declared_symbol():
    """include/ptmi_host.h <-> libptmi_host.so (the native scene side + writers)."""
    host_h = os.path.join(ROOT, "include", "ptmi_host.h")
    lib = os.path.join(ROOT, "pathtracer-ocl_amd", "build", "libptmi_host.so")
    if not os.path.exists(lib):
        pytest.fail("libptmi_host.so not built")
    src = re.sub(r"/\*.*?\*/", "", open(host_h).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(ptmi_host_[a-z_]+)\s*\(", src)))
    assert len(declared) >= 5
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert not [s for s in declared if s not in exported]


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(FileNotFoundError):
        api.load_library(str(tmp_path / "libptmi.so"))


def test_record_sizes_match_reference_layout():
    hdr = open(HEADER).read()
    sizes = dict(re.findall(r"#define (PTMI_\w+_BYTES) (\d+)", hdr))
    assert int(sizes["PTMI_OBJECT_BYTES"]) == layout.OBJECT_DTYPE.itemsize == 1024
    assert int(sizes["PTMI_TRIANGLE_BYTES"]) == layout.TRIANGLE_DTYPE.itemsize == 512
    assert int(sizes["PTMI_GROUP_BYTES"]) == layout.GROUP_DTYPE.itemsize == 256
    assert int(sizes["PTMI_CAMERA_BYTES"]) == layout.CAMERA_DTYPE.itemsize == 256

"""One HIP runtime per process.

PyTorch-ROCm bundles its own libamdhip64 / libhsa-runtime64 (SONAMEs
libamdhip64.so.7 / libhsa-runtime64.so.1) and loads them by their UNVERSIONED
file names, so if libptmi.so (linked against /opt/rocm) is loaded first, torch
later maps a second HIP runtime into the process and fails to initialise
("No HIP GPUs are available").  Loading torch first makes every later
DT_NEEDED libamdhip64.so.7 / libhsa-runtime64.so.1 resolve, by SONAME, to the
copy torch already mapped: one runtime, shared device pointers and streams.
A process without torch (e.g. a cgo caller) simply uses /opt/rocm's runtime.
"""
_done = False


def preload():
    global _done
    if _done:
        return
    _done = True
    try:
        import torch  # noqa: F401  (maps torch's HIP runtime)
    except ImportError:
        pass

"""ptmi: host-side mirror of the reference's ``internal/ocl`` boundary for the
MI355X HIP path tracer.  The compute path lives in
``pathtracer-ocl_amd/csrc`` (HIP, C-ABI ``libptmi.so``); this package holds the
scene-record restatement that produces the kernel's input bytes and the
``Trace`` binding (ocltracer.go:98-100)."""

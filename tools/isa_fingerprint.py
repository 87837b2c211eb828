"""DIAGNOSTIC: a fingerprint of each trace_kernel<FL>'s gfx950 ISA, to show that a change
elsewhere in the library (another kernel, host code) leaves a product kernel's code as it
was.
    python tools/isa_fingerprint.py [extra hipcc flags ...]
Compiles csrc/ptmi_kernels.hip to device assembly and prints, per trace_kernel<FL>, the
instruction count, VGPRs, scratch bytes and a hash of the instruction stream with labels
renumbered in order of appearance (function numbering changes when other kernels come or
go)."""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "pathtracer-ocl_amd", "csrc", "ptmi_kernels.hip")


def device_asm(extra):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-fno-fast-math", "-Wno-unused-result", "--cuda-device-only", "-S", "-o", out, SRC] + list(extra)
        subprocess.run(cmd, check=True)
        return open(out).read()


def fingerprints(asm):
    res = {}
    for m in re.finditer(r"^(_ZN4ptmi12trace_kernelILi(\d+)EEEv\w*):[^\n]*\n(.*?)\n\s*s_endpgm", asm, re.S | re.M):
        fl = int(m.group(2))
        body = m.group(3).split("\n")
        names, ins = {}, []
        for l in body:
            t = l.split(";")[0].strip()
            if not t or t.startswith("."):
                if t.endswith(":") and t.startswith(".LBB"):
                    names.setdefault(t[:-1], "L%d" % len(names))
                continue
            if t.endswith(":"):
                continue
            ins.append(t)
        # (labels past the first s_endpgm are not in `names`: drop the function number)
        norm = [re.sub(r"\.LBB\d+_(\d+)", lambda x: names.get(x.group(0), ".LBB_" + x.group(1)), t) for t in ins]
        h = hashlib.sha256("\n".join(norm).encode()).hexdigest()[:16]
        # the same with kernel-argument offsets masked (a field appended to a by-value argument
        # struct moves the later arguments' offsets and nothing else)
        ka = [re.sub(r"(s\[0:1\]), 0x[0-9a-f]+", r"\1, KA", t) for t in norm]
        hk = hashlib.sha256("\n".join(ka).encode()).hexdigest()[:16]
        res[fl] = (len(ins), h, hk)
    # resource usage from the metadata block (one entry per kernel, in .amdgpu_metadata)
    meta = {}
    for mm in re.finditer(r"\.name:\s+(_ZN4ptmi12trace_kernelILi(\d+)EEEv\w*)", asm):
        fl = int(mm.group(2))
        blk = asm[mm.end():].split("- .agpr_count", 1)[0]  # the rest of this kernel's entry
        vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        meta[fl] = (vg.group(1) if vg else "?", sc.group(1) if sc else "?")
    return res, meta


if __name__ == "__main__":
    res, meta = fingerprints(device_asm(sys.argv[1:]))
    for fl in sorted(res):
        n, h, hk = res[fl]
        vg, sc = meta.get(fl, ("?", "?"))
        print("trace_kernel<%-3d> insts %6d  vgpr %-4s scratch %-4s isa %s  isa-ka %s" % (fl, n, vg, sc, h, hk))

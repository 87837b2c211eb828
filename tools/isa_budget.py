"""DIAGNOSTIC: the instruction budget of one trace_kernel<FL> by phase, from its gfx950 ISA.
    python tools/isa_budget.py [FL] [extra hipcc flags ...]       (FL default 0: the C2 kernel)
Compiles csrc/ptmi_kernels.hip to device assembly with line info (-g does not change the code:
tools/isa_fingerprint.py gives the same hash) and attributes every instruction to a phase by
its inlining chain (the `.loc` comments: file:line @[ caller:line ] ...):
  noise3d/camera   noise3D draws of the anti-aliasing offsets (camera_offsets)
  noise3d/shading  noise3D draws of the bounce (hemisphere pair, materials)
  camera           the camera block and path start (ray_for_pixel, sunflower table, LDS buffer)
  planes, spheres  find_closest_prims' plane loops / sphere loops and deferred roots
  hull culls       (mesh kernels) group_needs_walk: the group objects' hull tests
  walks            (mesh kernels) the walk phases: group_walks, walk_index, triangle tests
  hemisphere       random_hemisphere (table lookup or sincos / sqrt chain, basis, direction)
  shading          the rest of bounce_shade (hit point, normal, material, mask / accumColor)
  loop             the bounce loop's own control (ballots, refill decision, LDS colour sums)
  outside          prologue (work item, seeds) and epilogue (sums) outside the main loop
and prints, per phase, VALU (vector ALU, of which FP64), SALU, SMEM, VMEM, LDS and branch
instruction counts.  Counts are static (instructions in the code); in the C2 kernel each
plane / sphere loop body and the shading run once per bounce, the camera block once per
sample, and the sin fallbacks rarely (see profiles/r5/SUMMARY.md)."""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pathtracer-ocl_amd", "csrc")
SRC = os.path.join(CSRC, "ptmi_kernels.hip")


def device_asm_g(extra):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-fno-fast-math", "-Wno-unused-result", "--cuda-device-only", "-S", "-g", "-o", out, SRC] + list(extra)
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        return open(out).read()


def function_ranges(path):
    """{name: (first line, last line)} of the device functions defined in a source file
    (1-based lines; brace matching from the definition's opening brace)."""
    lines = open(path).read().split("\n")
    res = {}
    i = 0
    pat = re.compile(r"^(?:template\s*<.*>\s*)?(?:__device__|__global__|static)[^;{]*?\b(\w+)\s*\(")
    while i < len(lines):
        m = pat.match(lines[i])
        if m and "__device__" in lines[i] or (m and "__global__" in lines[i]):
            name = m.group(1)
            depth, j, opened = 0, i, False
            while j < len(lines):
                for ch in lines[j]:
                    if ch == "{":
                        depth += 1
                        opened = True
                    elif ch == "}":
                        depth -= 1
                if opened and depth == 0:
                    break
                if not opened and lines[j].rstrip().endswith(";"):
                    break
                j += 1
            if opened:
                res.setdefault(name, (i + 1, j + 1))
            i = j + 1 if opened else i + 1
        else:
            i += 1
    return res


def main():
    args = sys.argv[1:]
    dump = None
    if "--dump" in args:  # --dump <phase>: list that phase's main-loop instructions with their source line
        i = args.index("--dump")
        dump = args[i + 1]
        del args[i:i + 2]
    fl = int(args[0]) if args and args[0].isdigit() else 0
    extra = [a for a in args if not a.isdigit()]
    asm = device_asm_g(extra)
    files = {int(m.group(1)): m.group(3) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', asm, re.M)}
    fr = function_ranges(SRC)
    fp = os.path.basename(SRC)
    # the sphere section of find_closest_prims begins at its sphere-record count
    fcp = fr["find_closest_prims"]
    src = open(SRC).read().split("\n")
    sph0 = next(i + 1 for i in range(fcp[0], fcp[1]) if "n_spheres_st" in src[i])

    def in_fn(chain, name):
        a, b = fr[name]
        return any(f == fp and a <= ln <= b for f, ln in chain)

    def phase(chain):
        if not chain:
            return "loop"
        if any(f == "ptmi_sinf.h" for f, _ in chain) or in_fn(chain, "noise3d"):
            return "noise3d/camera" if in_fn(chain, "camera_offsets") else "noise3d/shading"
        if in_fn(chain, "camera_offsets") or in_fn(chain, "ray_for_pixel") or in_fn(chain, "start_path") or \
                in_fn(chain, "camera_ptr") or in_fn(chain, "sunflower"):
            return "camera"
        if in_fn(chain, "group_walks") or in_fn(chain, "group_walks_impl") or in_fn(chain, "walk_index"):
            return "walks"
        if in_fn(chain, "group_needs_walk"):
            return "hull culls"
        for f, ln in chain:
            if f == fp and fcp[0] <= ln <= fcp[1]:
                return "planes" if ln < sph0 else "spheres"
        if in_fn(chain, "random_hemisphere") or in_fn(chain, "hemi_sincos") or in_fn(chain, "hemi_sqrt"):
            return "hemisphere"
        if in_fn(chain, "bounce_shade"):
            return "shading"
        return "loop"

    m = re.search(r"^(_ZN4ptmi12trace_kernelILi%dEEEv\w*):[^\n]*\n(.*?)\n\s*\.Lfunc_end" % fl, asm, re.S | re.M)
    body = m.group(2).split("\n")
    ins, labels, chain = [], {}, []
    for l in body:
        t = l.strip()
        if t.startswith(".loc"):
            c = t.split(";", 1)[1].strip() if ";" in t else ""
            chain = []
            for part in re.findall(r"([\w./-]+):(\d+):\d+", c):
                chain.append((os.path.basename(part[0]), int(part[1])))
            continue
        code = t.split(";")[0].strip()
        if not code:
            continue
        if code.endswith(":"):
            labels[code[:-1]] = len(ins)
            continue
        if code.startswith("."):
            continue
        ins.append((code, list(chain)))
    # the main loop: the outermost [label, backward branch] span
    loops = []
    for i, (code, _) in enumerate(ins):
        mm = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", code)
        if mm and mm.group(2) in labels and labels[mm.group(2)] <= i:
            loops.append((labels[mm.group(2)], i))
    main_lo, main_hi = max(loops, key=lambda x: x[1] - x[0]) if loops else (0, len(ins) - 1)

    def kind(op):
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            return "VALU"
        if op.startswith("v_"):
            return "VALU"
        if op.startswith(("s_load", "s_buffer_load", "s_store")):
            return "SMEM"
        if op.startswith(("s_cbranch", "s_branch")):
            return "branch"
        if op.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_setprio", "s_barrier")):
            return "wait"
        if op.startswith("s_"):
            return "SALU"
        if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
            return "VMEM"
        if op.startswith("ds_"):
            return "LDS"
        return "other"

    tab = defaultdict(Counter)
    for i, (code, ch) in enumerate(ins):
        op = code.split()[0]
        ph = phase(ch) if main_lo <= i <= main_hi else "outside"
        if dump and ph == dump:
            print("%5d  %-60s %s" % (i, code, " <- ".join("%s:%d" % c for c in ch[:3])))
        k = kind(op)
        tab[ph][k] += 1
        if k == "VALU" and "_f64" in op:
            tab[ph]["FP64"] += 1
        if k == "VALU" and op.startswith(("v_readlane", "v_writelane")):
            tab[ph]["lane_spill"] += 1
    order = ["camera", "noise3d/camera", "planes", "spheres", "hull culls", "walks", "shading", "hemisphere",
             "noise3d/shading", "loop", "outside"]
    cols = ["VALU", "FP64", "lane_spill", "SALU", "SMEM", "VMEM", "LDS", "branch"]
    print("trace_kernel<%d>: %d instructions, main loop [%d, %d]" % (fl, len(ins), main_lo, main_hi))
    print("| phase | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * len(cols))
    tot = Counter()
    for ph in order + sorted(set(tab) - set(order)):
        if ph not in tab:
            continue
        tot.update(tab[ph])
        print("| %s | " % ph + " | ".join(str(tab[ph][c]) for c in cols) + " |")
    print("| total | " + " | ".join(str(tot[c]) for c in cols) + " |")


if __name__ == "__main__":
    main()

"""DIAGNOSTIC: the dynamic instruction budget of a trace_kernel<FL> launch, by phase and op class.

    python tools/dyn_budget.py collect <out.json> [--config c2] [--samples S]     (GPU box, stats library)
    python tools/dyn_budget.py table [counts.json] [--fl 0] [-D... extra hipcc flags]  (here, CPU)

`collect` renders the bench workload with the stats library (PTMI_STATS=1, build/libptmi_stats.so:
the product's code plus per-wave counters; same images) and stores the wave-level execution count of
every block the counters mark (ptmi_kernels.hip ptmi_stats[32..46]: camera refills, sphere roots,
hemisphere fallbacks, noise paths, shading branches, prims, active lanes) and the loop iterations.

`table` compiles the product's device code (tools/isa_budget.py's parse), attributes every main-loop
instruction to a sub-phase by its inlining chain (noise: small-argument / Cody-Waite / Payne-Hanek /
>= 2^19 paths and their common part; sphere quadratics / deferred roots / in-place roots; hemisphere
table part / sincos fallback / sqrt fallback; shading common / plane normal / other normal / emission)
and to an op class (FP64 arithmetic, FP64 transcendental, FP32, select / compare, move / lane, integer,
conversion), and weights each sub-phase's static counts by its wave-level execution count.  The sum is
checked against the measured SQ_INSTS_VALU of the same launch when given (--measured).  Counts are
per wave execution of a block: a block costs its whole instruction stream whenever any lane of the
wave runs it, which is what SQ_INSTS_VALU counts.
"""
import json
import os
import re
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd"), os.path.join(ROOT, "tools")]

CLASSES = ["fp64", "fp64_trans", "fp32", "select_cmp", "move_lane", "int", "cvt"]


def op_class(op):
    if not op.startswith("v_"):
        return None
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane", "v_mov")):
        return "move_lane"
    if op.startswith(("v_cndmask", "v_cmp")):
        return "select_cmp"
    if op.startswith("v_cvt"):
        return "cvt"
    if re.match(r"v_(rcp|rsq|sqrt|sin|cos|exp|log)_f64", op):
        return "fp64_trans"
    if "_f64" in op:
        return "fp64"
    if "_f32" in op or "_f16" in op:
        return "fp32"
    return "int"


def counts_collect(out, config, samples):
    import ctypes
    os.environ.setdefault("PTMI_LIB", os.path.join(ROOT, "pathtracer-ocl_amd", "build", "libptmi_stats.so"))
    import torch  # noqa: F401
    from ptmi import api, layout
    from tests.scene_inputs import scene_inputs
    import bench
    scene, W, H, S, aper, focal = bench.CONFIGS[config][:6]
    spp = samples or S
    lib = api.load_library()
    buf = (ctypes.c_ulonglong * 80)()
    lib.ptmi_stats_read(buf, 1)
    objs, tris, grps, cam = scene_inputs(scene, W, H, aper, focal)
    api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 3))
    lib.ptmi_stats_read(buf, 1)
    v = list(buf)
    json.dump({"config": config, "scene": scene, "width": W, "height": H, "spp": spp, "stats": v}, open(out, "w"),
              indent=1)
    print("iterations", v[10], "refills", v[32], "prims", v[45], "lane util (prims)",
          v[46] / max(1, 64 * v[45]), "noise draws", v[40])


def subphase(chain, fr, src_lines, fp):
    """(phase, sub-phase) of one instruction from its inlining chain (file, line) innermost first."""
    import isa_budget as ib  # noqa: F401

    def in_fn(name, file=fp):
        if name not in fr:
            return False
        a, b = fr[name]
        return any(f == file and a <= ln <= b for f, ln in chain)

    def line_in(file, a, b):
        return any(f == file and a <= ln <= b for f, ln in chain)

    if not chain:
        return "loop", "loop"
    noise = any(f == "ptmi_sinf.h" for f, _ in chain) or in_fn("noise3d")
    if noise:
        site = "camera" if in_fn("camera_offsets") else "shading"
        sr = sinf_ranges()
        if line_in("ptmi_sinf.h", *sr["small"]):
            sub = "small"
        elif line_in("ptmi_sinf.h", *sr["cw64"]) or line_in("ptmi_sinf.h", *sr["cw64_fn"]):
            sub = "cw64"
        elif line_in("ptmi_sinf.h", *sr["payne_hanek"]):
            sub = "payne_hanek"
        elif line_in("ptmi_sinf.h", *sr["cw30"]):
            sub = "ge_2^19"
        else:
            sub = "common"
        return "noise3d/" + site, sub
    if in_fn("camera_offsets") or in_fn("ray_for_pixel") or in_fn("start_path") or in_fn("camera_ptr"):
        return "camera", "camera"
    fcp = fr["find_closest_prims"]
    site = [l2 for f2, l2 in chain if f2 == fp and fcp[0] <= l2 <= fcp[1]]
    if site:
        if in_fn("sphere_roots"):
            # the call site: the defer lambda (in place, a lane's second sphere) or the deferred one
            inplace = any("sphere_roots<A>(h, a, b, disc, pk)" in src_lines[l2 - 1] for l2 in site)
            return "spheres", "roots_inplace" if inplace else "roots_deferred"
        outer = site[-1]  # the line in find_closest_prims' own body (lambdas are inlined from it)
        for name, (x0, x1) in prims_blocks(src_lines, fcp).items():
            if x0 <= outer <= x1:
                return ("planes" if name.startswith("plane") else "spheres"), name
        sph0 = next(i + 1 for i in range(fcp[0], fcp[1]) if "n_spheres_st" in src_lines[i])
        return ("planes", "plane_other") if outer < sph0 else ("spheres", "sphere_other")
    if in_fn("random_hemisphere") or in_fn("hemi_sincos") or in_fn("hemi_sqrt"):
        if in_fn("hemi_sincos"):
            return "hemisphere", "sincos_fallback"
        if in_fn("hemi_sqrt"):
            return "hemisphere", "sqrt_fallback"
        return "hemisphere", "table_basis"
    if in_fn("bounce_shade"):
        a, b = fr["bounce_shade"]
        for f, ln in chain:
            if f == fp and a <= ln <= b:
                txt = src_lines[ln - 1]
                blk = shade_blocks(src_lines, a, b)
                for name, (x0, x1) in sorted(blk.items(), key=lambda kv: kv[1][1] - kv[1][0]):
                    if x0 <= ln <= x1:  # innermost (smallest) block first
                        return "shading", name
        return "shading", "common"
    return "loop", "loop"


_blk_cache = {}


def sinf_ranges():
    """Line ranges in ptmi_sinf.h of the noise sin's paths: the small-argument reduction, the FP64
    Cody-Waite block of sf_redux_large_17_19 (and sf_cw64), its Payne-Hanek rest, sinf_cw30."""
    if "sinf" in _blk_cache:
        return _blk_cache["sinf"]
    import isa_budget as ib
    path = os.path.join(ib.CSRC, "ptmi_sinf.h")
    lines = open(path).read().split("\n")
    fr = {}
    for i, l in enumerate(lines):
        m = re.match(r"^PTMI_SINF_FN\s.*?\b(\w+)\s*\(", l)
        if m:
            fr[m.group(1)] = (i + 1, _close(lines, i, len(lines)))
    a, b = fr["sf_redux_large_17_19"]
    cw_end = next(i + 1 for i in range(a, b) if lines[i].startswith("#endif"))
    res = {"small": fr["sf_redux_small"], "cw64": (a, cw_end), "payne_hanek": (cw_end + 1, b),
           "cw30": fr["sinf_cw30"], "cw64_fn": fr.get("sf_cw64", (0, -1))}
    _blk_cache["sinf"] = res
    return res


def _close(src_lines, start, limit):
    """1-based line of the brace closing the first '{' at or after line index start."""
    depth, opened = 0, False
    for i in range(start, limit):
        for ch in src_lines[i]:
            if ch == "{":
                depth += 1
                opened = True
            elif ch == "}":
                depth -= 1
                if opened and depth == 0:
                    return i + 1
    return limit


def prims_blocks(src_lines, fcp):
    """Line ranges of find_closest_prims' plane and sphere loop bodies (their execution counters:
    ptmi_stats[47..52])."""
    key = ("prims",) + tuple(fcp)
    if key in _blk_cache:
        return _blk_cache[key]
    marks = {"plane_ypair": "for (; p + 1 < npy; p += 2)", "plane_pair": "for (; p + 1 < np; p += 2)",
             "plane_single": "if (p < np) {", "sphere_first_pair": "if (PTMI_R6_SPH && nq >= 2) {",
             "sphere_pair": "for (; q + 1 < nq; q += 2)", "sphere_single": "if (q < nq) {",
             "sphere_roots_call": "if (pend) {", "sphere_general": "for (; j < S.run_end[1]; j++) {",
             "sphere_first_single": "if (PTMI_R6_SPH && nq == 1) {"}
    res = {}
    for i in range(fcp[0] - 1, fcp[1]):
        for name, m in marks.items():
            if m in src_lines[i] and name not in res:
                res[name] = (i + 1, _close(src_lines, i, fcp[1]))
    _blk_cache[key] = res
    return res


def shade_blocks(src_lines, a, b):
    """Line ranges of bounce_shade's plane-normal block, other-normal block and emission block."""
    key = (a, b)
    if key in _blk_cache:
        return _blk_cache[key]

    def block_from(start, col=0):
        """1-based line of the brace closing the first '{' at or after (line index start, column col)."""
        depth, opened = 0, False
        for i in range(start, b):
            for ch in src_lines[i][col if i == start else 0:]:
                if ch == "{":
                    depth += 1
                    opened = True
                elif ch == "}":
                    depth -= 1
                    if opened and depth == 0:
                        return i + 1
        return b

    res = {}
    for i in range(a, b):
        t = src_lines[i]
        if "type == 0 && !((FL & F_TEX)" in t and "plane_normal" not in res:
            e = block_from(i)  # the "} else {" line
            res["plane_normal"] = (i + 1, e - 1)
            res["other_normal"] = (e, block_from(e - 1, src_lines[e - 1].index("else")))
        if "if (er > 0.0) {" in t and "emission" not in res:
            res["emission"] = (i + 1, block_from(i))
        if "// group: interpolated vertex normal" in t and "normal_group" not in res:
            res["normal_group"] = (i + 1, block_from(i))
    _blk_cache[key] = res
    return res


def static_table(fl, extra):
    import isa_budget as ib
    asm = ib.device_asm_g(extra)
    fr = ib.function_ranges(ib.SRC)
    fr.update({k: v for k, v in ib.function_ranges(os.path.join(ib.CSRC, "ptmi_sinf.h")).items() if k not in fr})
    fp = os.path.basename(ib.SRC)
    src_lines = open(ib.SRC).read().split("\n")
    m = re.search(r"^(_ZN4ptmi12trace_kernelILi%dEEEv\w*):[^\n]*\n(.*?)\n\s*\.Lfunc_end" % fl, asm, re.S | re.M)
    body = m.group(2).split("\n")
    ins, labels, chain = [], {}, []
    for l in body:
        t = l.strip()
        if t.startswith(".loc"):
            c = t.split(";", 1)[1].strip() if ";" in t else ""
            chain = [(os.path.basename(p[0]), int(p[1])) for p in re.findall(r"([\w./-]+):(\d+):\d+", c)]
            continue
        code = t.split(";")[0].strip()
        if not code or code.startswith("."):
            if code.endswith(":"):
                labels[code[:-1]] = len(ins)
            continue
        if code.endswith(":"):
            labels[code[:-1]] = len(ins)
            continue
        ins.append((code, list(chain)))
    loops = []
    for i, (code, _) in enumerate(ins):
        mm = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", code)
        if mm and mm.group(2) in labels and labels[mm.group(2)] <= i:
            loops.append((labels[mm.group(2)], i))
    lo, hi = max(loops, key=lambda x: x[1] - x[0])
    class Tab(defaultdict):
        pass
    tab = Tab(Counter)
    sites = defaultdict(set)  # inlined copies of a sub-phase (the defer lambda's in-place roots: one per call)
    fcp = fr["find_closest_prims"]
    for i, (code, ch) in enumerate(ins):
        if not lo <= i <= hi:
            continue
        op = code.split()[0]
        c = op_class(op)
        if c is None:
            continue
        k = subphase(ch, fr, src_lines, fp)
        tab[k][c] += 1
        outer = [ln for f, ln in ch if f == fp and fcp[0] <= ln <= fcp[1]]
        if outer:
            sites[k].add(outer[-1])
    tab.copies = {k: len(v) for k, v in sites.items() if k == ("spheres", "roots_inplace")}
    return tab


# wave-level executions of each sub-phase from the stats counters (see the module docstring)
counts_fl_no_groups = True  # (table: set from --fl: kernels without F_GROUPS)


def executions(v):
    draws = max(v[40], 1)
    cam_draws = 2 * v[32]
    shade_draws = max(v[40] - cam_draws, 0)
    f_small, f_cw, f_hi = v[37] / draws, v[38] / draws, v[39] / draws
    e = {("loop", "loop"): v[10], ("camera", "camera"): v[32], ("planes", "plane_other"): v[45],
         ("planes", "plane_ypair"): v[47], ("planes", "plane_pair"): v[48], ("planes", "plane_single"): v[49],
         ("spheres", "sphere_other"): v[45], ("spheres", "sphere_first_pair"): v[50],
         ("spheres", "sphere_pair"): v[51], ("spheres", "sphere_single"): v[52],
         ("spheres", "sphere_roots_call"): v[33], ("spheres", "roots_deferred"): v[33],
         ("spheres", "sphere_general"): v[53],
         # the one-sphere peel runs only when the scene has exactly one such sphere
         ("spheres", "sphere_first_single"): v[45] if (v[50] == 0 and v[52] > 0) else 0,
         # the mesh triangle's normal: never in a kernel without groups (the C2 / C3 tables)
         ("shading", "normal_group"): 0 if counts_fl_no_groups else v[42],
         ("spheres", "roots_inplace"): v[34], ("hemisphere", "table_basis"): v[44],
         ("hemisphere", "sincos_fallback"): v[35], ("hemisphere", "sqrt_fallback"): v[36],
         ("shading", "common"): v[44], ("shading", "plane_normal"): v[41],
         ("shading", "other_normal"): v[42], ("shading", "emission"): v[43]}
    for site, n in (("camera", cam_draws), ("shading", shade_draws)):
        # the two draws of a site run back to back: a site's code holds both copies, so its
        # executions are pairs (n / 2)
        pairs = n / 2.0
        e[("noise3d/" + site, "common")] = pairs
        e[("noise3d/" + site, "small")] = pairs * f_small
        e[("noise3d/" + site, "cw64")] = pairs * f_cw
        e[("noise3d/" + site, "payne_hanek")] = pairs * 0.0
        e[("noise3d/" + site, "ge_2^19")] = pairs * f_hi
    return e


def main():
    args = sys.argv[1:]
    if args and args[0] == "collect":
        cfg, spp = "c2", 0
        if "--config" in args:
            cfg = args[args.index("--config") + 1]
        if "--samples" in args:
            spp = int(args[args.index("--samples") + 1])
        counts_collect(args[1], cfg, spp)
        return
    assert args and args[0] == "table", __doc__
    counts = None
    if len(args) > 1 and args[1].endswith(".json"):
        counts = json.load(open(args[1]))
    fl = int(args[args.index("--fl") + 1]) if "--fl" in args else 0
    global counts_fl_no_groups
    counts_fl_no_groups = (fl & 1) == 0
    measured = float(args[args.index("--measured") + 1]) if "--measured" in args else None
    extra = [a for a in args if a.startswith("-D")]
    tab = static_table(fl, extra)
    keys = sorted(tab)
    print("trace_kernel<%d>, main loop, static VALU by sub-phase and op class" % fl)
    print("| phase | sub-phase | " + " | ".join(CLASSES) + " | total |")
    print("|---|---|" + "---|" * (len(CLASSES) + 1))
    for k in keys:
        print("| %s | %s | " % k + " | ".join(str(tab[k][c]) for c in CLASSES) + " | %d |" % sum(tab[k].values()))
    if not counts:
        return
    v = counts["stats"]
    ex = executions(v)
    dyn = defaultdict(Counter)
    for k in keys:
        n = ex.get(k)
        if n is None:
            print("(no execution count for %s / %s: left out)" % k)
            continue
        copies = max(1, tab.copies.get(k, 1)) if hasattr(tab, "copies") else 1
        for c in CLASSES:
            dyn[k][c] += tab[k][c] * n / copies
    tot = Counter()
    for k in dyn:
        tot.update(dyn[k])
    T = sum(tot.values())
    print()
    print("dynamic VALU (wave instructions per launch) = static count x wave-level executions; %s, %d spp"
          % (counts["scene"], counts["spp"]))
    print("| phase | sub-phase | executions | " + " | ".join(CLASSES) + " | total | share |")
    print("|---|---|---|" + "---|" * (len(CLASSES) + 2))
    for k in sorted(dyn, key=lambda k: -sum(dyn[k].values())):
        s = sum(dyn[k].values())
        print("| %s | %s | %.3g | " % (k[0], k[1], ex[k]) + " | ".join("%.3g" % dyn[k][c] for c in CLASSES) +
              " | %.3g | %.3f |" % (s, s / T))
    print("| total | | | " + " | ".join("%.3g" % tot[c] for c in CLASSES) + " | %.3g | 1 |" % T)
    print("op-class shares: " + ", ".join("%s %.3f" % (c, tot[c] / T) for c in CLASSES))
    if measured:
        print("measured SQ_INSTS_VALU %.4g: estimate / measured = %.3f" % (measured, T / measured))
    print("loop iterations %d, prims executions %d, lane utilisation at prims %.3f"
          % (v[10], v[45], v[46] / max(1, 64 * v[45])))


if __name__ == "__main__":
    main()

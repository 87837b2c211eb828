#!/usr/bin/env python3
"""bench.py -- Msamples/s of the HIP path tracer on the 1280x960 reference Cornell
scene (BASELINE.json metric / configs[1]: 2048 spp, one frame per step).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

`--gpus N` with N > 1 and no torch.distributed environment starts the N ranks
itself (one child process per GPU, LOCAL_RANK 0..N-1, before this process touches
the GPU) and exits with their status; under torchrun WORLD_SIZE must equal N.

A step renders ONE complete frame (W*H*S primary samples) with the inputs (scene
records, per-pixel seeds) already resident in HBM: rank r renders its share of
the frame (sample split: a cost-balanced range of sample indices; tile split for
c5: the 8x8 tiles t with t % N == r), the per-GPU partial framebuffers are summed
onto rank 0 with one RCCL reduce over xGMI (torch.distributed "nccl" backend),
and rank 0 normalises the frame on device (colors * 1/S, alpha 1;
tracer.cl:1184-1187).  Total work per step is fixed ("scaling": "strong");
value = W*H*S*K / (max over ranks of the K-step wall time).

roofline: C2/C3 trace_kernel is FP64-VALU bound (the scene is 8 KB and HBM
traffic is ~0.02 B/sample): achieved = algorithmic FP64 flops per launch (frozen
model, profiles/alg_counts.json, ptmi/flops.py) / the kernel's average launch
time, measured with HIP events recorded on the launch stream around every launch
in the timed region; peak = MI355X FP64 vector peak (78.6 TFLOP/s).  C4/C5 (BVH
scenes) report the memory hierarchy of SURVEY.md 8d level by level: the bytes per
sample of the traversal the kernel runs (tools/traversal_bytes.py) are L2-served,
so they are priced against the L2 peak (34.5 TB/s), with the PMC-measured L2
requests and HBM bytes beside them; the bound is VALU issue / load latency (idle
lanes in the walk phases), which is what the counters show.  `traffic` = HBM bytes
per launch from rocprofv3 PMC passes of this build (they cannot run inside this
process; profiles/pmc_measured.json freezes them from profiles/<round>/).
cpu_baseline: the oracle's C restatement of the reference kernel (OpenMP) timed on
the host cores on a bounded sample of the same frame spread over its sample
indices, plus the whole C1 frame (rank 0, N=1 only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]

CONFIGS = {
    # name: (scene, W, H, spp, aperture, focal, split, alg_counts key, description)
    "c2": ("reference", 1280, 960, 2048, 0.0, 0.0, "sample", "c2_reference_1280x960",
           "reference Cornell scene 1280x960, 2048 spp (BASELINE configs[1])"),
    "c3": ("reference", 1280, 960, 2048, 0.15, 1.6, "sample", "c3_reference_dof_1280x960",
           "reference scene 1280x960, 2048 spp, DoF aperture 0.15 focal 1.6 (configs[2])"),
    "c4": ("teapot", 1280, 960, 2048, 0.0, 0.0, "sample", "c4_teapot_1280x960",
           "teapot BVH 1280x960, 2048 spp (configs[3])"),
    "c5": ("gopher", 1280, 960, 2048, 0.0, 0.0, "tile", "c5_gopher_1280x960",
           "gopher BVH 1280x960, 2048 spp, tile split (configs[4])"),
}
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (/opt/skills/guides/MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak
L2_PEAK_GBS = 34500.0    # MI355X aggregate L2 bandwidth, 8 XCDs x 4 MiB (MI355X_MICROARCH.md "L2 (per XCD)")
# rocprofv3 PMC measurements of the current build (HBM bytes and L2 requests per trace_kernel
# launch, per workload), frozen by tools/pmc_freeze.py from the profiles/<round>/ passes.
PMC_FROZEN = os.path.join(ROOT, "profiles", "pmc_measured.json")


def build_id():
    """A short hash of the kernel library's sources (pathtracer-ocl_amd/csrc, include/):
    frozen PMC counters (profiles/pmc_measured.json) are reported only for the build
    they were measured on."""
    import hashlib
    h = hashlib.sha256()
    for d in (os.path.join(ROOT, "pathtracer-ocl_amd", "csrc"), os.path.join(ROOT, "include")):
        for name in sorted(os.listdir(d)):
            with open(os.path.join(d, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:12]


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None):
    """Start n ranks of `script` (default: this file; RANK = LOCAL_RANK = 0..n-1) and
    wait for them.  Called before anything touches the GPU; the children inherit
    stdout, and only rank 0 prints the result line.  A failing rank stops the others.
    Returns the first non-zero exit status, else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script or __file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in procs:
                    q.terminate()
        time.sleep(0.2)
    return rc


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """(threads to use, details): the CPUs this process may run on -- its affinity
    mask, capped by a cgroup v2 CPU quota (cpu.max) when one is set and by the
    OpenMP thread count the environment grants.  The GPU box grants one GPU's job a
    16-CPU share of the host (its OMP_NUM_THREADS; jobs there must size worker pools
    to it), so the baseline runs on that share and reports the machine's nproc and
    CPU model beside it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    if omp:
        cores = min(cores, omp)
    return cores, {"nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp}


def cpu_baseline(layout, objs, tris, grps, cam, spp, seeds, budget_s=15.0):
    """The CPU restatement of the reference kernel on the host cores (rank 0, N=1):
    (1) the workload's frame at a bounded sample: every pixel, 8 windows of sample
    indices spread evenly over [0, S) (early indices are cheaper: small-argument
    noise sin), sized to about budget_s; (2) the whole C1 frame (reference scene
    640x480, 4 spp, BASELINE configs[0])."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from tests.scene_inputs import scene_inputs
    if not pyoracle.cpu_available():
        return None
    threads, cpus = host_cpus()
    w = int(np.asarray(cam).reshape(())["width"])
    h = int(np.asarray(cam).reshape(())["height"])
    t2, g2 = layout.pad_empty(tris, grps)
    windows = 8
    starts = [k * spp // windows for k in range(windows)]
    # calibrate: one sample at each window start over a centred band of rows
    band = max(1, h // 16)
    t0 = time.time()
    for s0 in starts:
        pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, row0=(h - band) // 2, rows=band, sample_begin=s0,
                           sample_end=s0 + 1, threads=threads)
    rate = band * w * windows / max(time.time() - t0, 1e-3)
    per_win = int(max(1, min(spp // windows, budget_s * rate / (w * h * windows))))
    for _ in range(3):  # re-size from the last measured run until it fills about half the budget
        t0 = time.time()
        for s0 in starts:
            pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, sample_begin=s0, sample_end=s0 + per_win,
                               threads=threads)
        el = time.time() - t0
        if el >= 0.5 * budget_s or per_win >= spp // windows:
            break
        per_win = int(max(1, min(spp // windows, per_win * budget_s / max(el, 1e-3))))
    out = {"value": round(w * h * per_win * windows / el / 1e6, 3), "unit": "Msamples/s", "cores": threads,
           "cpus": cpus, "cpu_model": _cpu_model(), "kind": "port",
           "sample": "all %dx%d pixels x samples [k*%d/8, k*%d/8 + %d) for k = 0..7 of the %d-spp frame (%.1f s)"
                     % (w, h, spp, spp, per_win, spp, el),
           "calibration_vs_reference_x86": None,
           "calibration_note": "the reference kernel cannot be built for x86 here without a stand-in OpenCL "
                               "builtin library (DESIGN.md s7); the port is pinned to the reference's own output "
                               "(goldens, live reference kernel on the GPU) instead"}
    o1, tr1, g1, c1 = scene_inputs("reference", 640, 480)
    s1 = layout.seeds_go_float64(640 * 480, 1234)
    tr1, g1 = layout.pad_empty(tr1, g1)
    t0 = time.time()
    pyoracle.cpu_trace(o1, tr1, g1, c1, 4, s1, threads=threads)
    e1 = time.time() - t0
    out["c1"] = {"workload": "reference Cornell scene 640x480, 4 spp (BASELINE configs[0]), whole frame",
                 "value": round(640 * 480 * 4 / e1 / 1e6, 3), "unit": "Msamples/s", "seconds": round(e1, 3)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--samples", type=int, default=0, help="override spp (0 = config)")
    ap.add_argument("--chunks", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-trace-call", action="store_true", help="skip the PCIe-inclusive ptmi_trace timing")
    ap.add_argument("--save-image", default="")
    ap.add_argument("--extra", default="auto",
                    help="other configs timed after the headline at the same GPU count: a comma list, none, or "
                         "auto (c3,c5 after a default c2 run at full spp)")
    ap.add_argument("--extra-steps", type=int, default=2)
    ap.add_argument("--rng", default="noise3d", choices=("noise3d", "xoshiro"),
                    help="xoshiro: the headline config in the opt-in statistical RNG mode (profiling; not `value`)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="DIAGNOSTIC: a work-plan knob of every scene (ptmi_diag_set_knob; names: tail_tiles, "
                         "tail_items, mesh_items, min_chunk, tile_order, split_chunk, split_slots, split_sync, "
                         "split_budget); tuning studies only")
    ap.add_argument("--split", action="store_true",
                    help="DIAGNOSTIC: mesh scenes in the split form (needs PTMI_LIB=<the study library>)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)

    import numpy as np
    import torch  # first: its HIP runtime is the process's (ptmi/_runtime.py)
    import torch.distributed as dist
    from ptmi import api, layout
    from ptmi import dist as pdist
    knobs = []  # --knob NAME=VALUE (DIAGNOSTIC)
    for kv in args.knob:
        k, v = kv.split("=", 1)
        knobs.append((getattr(api, "KNOB_" + k.strip().upper()), int(v)))
    from tests.scene_inputs import scene_inputs

    ndev = torch.cuda.device_count()
    # One GPU per rank.  With fewer devices than ranks (a rehearsal of the N-rank path on
    # a smaller box) ranks share devices and the reduce goes through gloo on the host;
    # the line says so ("shared_devices") and its numbers are not a scaling measurement.
    shared = world > ndev
    device = local % max(ndev, 1)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    torch.cuda.set_device(device)
    # Which GPU each rank landed on (a scaling run must show N distinct devices).
    props = torch.cuda.get_device_properties(device)
    me = {"rank": rank, "local_rank": local, "device": device, "name": props.name,
          "arch": getattr(props, "gcnArchName", None), "uuid": str(getattr(props, "uuid", "")),
          "pci": "%s:%s:%s" % (getattr(props, "pci_domain_id", "?"), getattr(props, "pci_bus_id", "?"),
                               getattr(props, "pci_device_id", "?")),
          "visible_devices": ndev}
    ranks_info = [me]
    if world > 1:
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, me)
    comm = {"backend": dist.get_backend() if world > 1 else "none", "world_size": world,
            "distinct_devices": len({r["uuid"] or r["pci"] for r in ranks_info}), "ranks": ranks_info}

    def run_config(cfg, steps, warmup, samples=0, chunks=0, save_image="", rng=0):
        """Render `steps` timed frames of config `cfg` on this rank's share (after
        `warmup` untimed ones): barrier + synchronize on both sides, max over ranks.
        Returns (per-config results on rank 0, the scene inputs)."""
        scene_name, W, H, S, aper, focal, split, alg_key, desc = CONFIGS[cfg]
        if samples:
            S = samples
        objs, tris, grps, cam = scene_inputs(scene_name, W, H, aper, focal)
        scene = api.Scene(device, objs, tris, grps, cam)
        for k, v in knobs:  # DIAGNOSTIC tuning (--knob)
            if scene.set_knob(k, v) != api.PTMI_OK:
                raise SystemExit("knob %d=%d unsupported by %s" % (k, v, api.LIB_PATH))
        if args.split and not scene.set_split(True):
            raise SystemExit("--split needs the study library (PTMI_LIB=pathtracer-ocl_amd/build/libptmi_study.so)")
        if rng:
            scene.set_rng(rng)  # the opt-in statistical mode: never the headline value
        npix = W * H
        seeds_host = layout.seeds_go_float64(npix, 1234)
        seeds = torch.tensor(seeds_host, dtype=torch.float64, device="cuda")
        sums = torch.empty(npix * 4, dtype=torch.float64, device="cuda")
        img = torch.empty(npix * 4, dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        s0, s1, t_stride, t_off = pdist.shard(rank, world, S, split)
        red_ev = []

        def step():
            scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=t_stride, tile_offset=t_off,
                         chunks=chunks, stream=stream)
            if world > 1:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                pdist.reduce_frame_to(sums, 0, via_host=shared)  # RCCL reduce over xGMI onto rank 0
                e1.record()
                red_ev.append((e0, e1))
            if rank == 0:
                scene.finalize(sums.data_ptr(), img.data_ptr(), S, stream=stream)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        scene.kernel_time()  # drop warmup launches
        red_ev.clear()
        scene.set_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        kms, klaunch = scene.kernel_time()
        scene.set_timing(False)
        red_ms = sum(a.elapsed_time(b) for a, b in red_ev) / max(len(red_ev), 1)
        # per-rank [wall, kernel ms per launch, reduce ms] gathered on every rank
        red_dev = "cpu" if shared else "cuda"
        mine = torch.zeros(world, 3, dtype=torch.float64, device=red_dev)
        mine[rank, 0] = el
        mine[rank, 1] = kms / max(klaunch, 1)
        mine[rank, 2] = red_ms
        if world > 1:
            dist.all_reduce(mine, op=dist.ReduceOp.SUM)
        per_rank = mine.cpu().numpy()
        el = float(per_rank[:, 0].max())
        res = None
        if rank == 0:  # sanity: a finite image with alpha 1
            im = img.view(H, W, 4)
            ok = bool(torch.isfinite(im).all().item()) and bool((im[..., 3] == 1.0).all().item())
            if save_image:
                np.save(save_image, im.cpu().numpy())
            avg_ms = float(per_rank[0, 1])
            my_samples_per_launch = npix * (s1 - s0) if split == "sample" else W * H * S / max(world, 1)
            par = "single GPU"
            if world > 1:
                par = "%s-split x%d + RCCL reduce" % (split, world) if not shared else \
                    "%s-split x%d ranks on %d device(s), gloo host reduce (rehearsal)" % (split, world, ndev)
            res = {"value": W * H * S * steps / el / 1e6, "ms_per_step": el / steps * 1e3, "image_ok": ok,
                   "avg_kernel_ms": avg_ms, "launches": klaunch, "per_rank": per_rank,
                   "rate": my_samples_per_launch / (avg_ms * 1e-3), "alg_key": alg_key, "split": split,
                   "samples_per_launch": my_samples_per_launch, "frame_samples": W * H * S,
                   "config": {"workload": desc, "scene": scene_name, "width": W, "height": H, "spp": S,
                              "aperture": aper, "focal_length": focal, "split": split, "parallelism": par}}
        scene.close()
        del seeds, sums, img
        return res, (objs, tris, grps, cam, S, seeds_host)

    def roofline(res):
        """The dominant kernel's roofline for one config's result (rank 0)."""
        try:
            with open(os.path.join(ROOT, "profiles", "alg_counts.json")) as f:
                ac = json.load(f)["workloads"][res["alg_key"]]
        except (OSError, KeyError) as e:
            return {"error": "alg counts unavailable: %s" % e}
        pmc_note = None
        try:
            with open(PMC_FROZEN) as f:
                frozen = json.load(f)
            pmc = frozen["workloads"].get(res["alg_key"])
            pmc_spp = int(frozen.get("spp", 2048))
            if frozen.get("build") != build_id():
                pmc_note = ("stale: profiles/pmc_measured.json holds counters of build %s, this build is %s; "
                            "measured levels omitted" % (frozen.get("build"), build_id()))
                pmc = None
        except (OSError, KeyError, ValueError):
            pmc, pmc_spp = None, 2048
        rate = res["rate"]  # samples/s of the kernel, rank 0
        kms = res["avg_kernel_ms"]
        f64 = ac["fp64_flops_per_sample"]
        achieved = f64 * rate / 1e12
        fp64 = {"bound": "valu_fp64",
                "bound_detail": "FP64 vector ALU issue (no MFMA-shaped work; HBM ~0.02 B/sample)",
                "achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP64_PEAK_TFLOPS, 4), "fp64_flops_per_sample": round(f64, 1),
                "flops_basis": "reference-rule algorithmic count (oracle -DPTO_COUNT), not executed"}
        # HBM bytes per launch measured by rocprofv3 PMC passes of this build (FETCH_SIZE x2 +
        # WRITE_SIZE, gfx950-corrected) on full W x H x pmc_spp frames, scaled to this
        # launch's samples.
        share = res["samples_per_launch"] / float(res["config"]["width"] * res["config"]["height"] * pmc_spp)
        traffic = None
        hbm = None
        if pmc and pmc.get("hbm_bytes_per_launch"):
            traffic = pmc["hbm_bytes_per_launch"] * share
            gbs = traffic / (kms * 1e-3) / 1e9
            hbm = {"achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(gbs / HBM_PEAK_GBS, 6), "bytes_per_launch": round(traffic),
                   "source": pmc.get("source")}
        tv = ac.get("traversal")
        if tv is None:  # C2 / C3: FP64-VALU bound
            roof = dict(fp64)
            if hbm:
                roof["hbm"] = hbm
        else:
            # C4 / C5 (SURVEY.md 8d memory hierarchy): the traversal's node / triangle bytes are
            # served by L2 (working set ~1-2 MB per XCD), so its bandwidth level is L2; HBM beside
            # it.  Neither binds: the counters show VALU issue with idle lanes and dependent
            # node-load latency (profiles/<round>/SUMMARY.md), hence the bound.
            l2_gbs = tv["bytes_per_sample"] * rate / 1e9
            ref_gbs = ac["bytes_per_sample"] * rate / 1e9
            l2 = {"achieved": round(l2_gbs, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                  "frac": round(l2_gbs / L2_PEAK_GBS, 4), "bytes_per_sample": round(tv["bytes_per_sample"], 1),
                  "bytes_basis": tv["basis"]}
            if pmc and pmc.get("l2_read_bytes_per_launch"):
                mb = pmc["l2_read_bytes_per_launch"] * share
                l2["measured"] = {"bytes_per_launch": round(mb), "GBs": round(mb / (kms * 1e-3) / 1e9, 1),
                                  "frac": round(mb / (kms * 1e-3) / 1e9 / L2_PEAK_GBS, 4),
                                  "l2_hit_rate": pmc.get("l2_hit_rate"), "source": pmc.get("source")}
            roof = {"bound": "valu_issue_latency",
                    "bound_detail": "VALU issue with idle lanes in the BVH walk phases and the latency of "
                                    "their dependent node loads bind (roofline.valu, profiles/<round>/SUMMARY.md); "
                                    "neither L2 nor HBM does.  achieved / peak / frac are the L2 level of the "
                                    "traversal's bytes (working set L2-resident), the memory level the "
                                    "walk's loads are served from; HBM beside it (roofline.hbm)",
                    "achieved": l2["achieved"], "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": l2["frac"],
                    "level": "l2", "l2": l2, "hbm": hbm,
                    "reference_rule": {"bytes_per_sample": round(ac["bytes_per_sample"], 1),
                                       "equivalent_GBs": round(ref_gbs, 1),
                                       "basis": "the reference's visit rules (tracer.cl:617-719: every "
                                                "triangle of every node whose box the line passes): the "
                                                "bytes its traversal would fetch at this sample rate"},
                    # (round 5 named this "fp64_reference_equivalent") the FP64 rate
                    # the reference's own visit rules would have to sustain at this sample rate -- a
                    # work-equivalent figure, not the kernel's utilisation
                    "reference_rule_work_rate": dict(fp64, bound="reference_rule_work_equivalent",
                                                     bound_detail="FP64 flops of the reference's visit rules at "
                                                                  "this sample rate (ptmi never executes them)")}
            if pmc and pmc.get("valu"):
                roof["valu"] = pmc["valu"]
        # The FP64 work the kernel actually executes (frozen PMC counters of this build, scaled to the
        # launch), beside the algorithmic fraction roofline.frac prices: the algorithmic
        # count credits work ptmi skips (structural zeros, the hemisphere table), the executed one is
        # the VALU's FP64 utilisation.
        pv = (pmc or {}).get("valu") or {}
        if pv.get("fp64_flops_executed_per_launch"):
            ex = pv["fp64_flops_executed_per_launch"] * share / (kms * 1e-3) / 1e12
            roof["fp64_executed"] = {"achieved": round(ex, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                     "frac": round(ex / FP64_PEAK_TFLOPS, 4),
                                     "basis": "rocprofv3 SQ_INSTS_VALU_{ADD,MUL,TRANS,FMA x2}_F64 x 64 x lane "
                                              "utilisation, this build (profiles/pmc_measured.json)"}
        if pmc_note:
            roof["pmc_status"] = pmc_note
        roof.update({"build": build_id(), "traffic": None if traffic is None else round(traffic),
                     "traffic_note": "HBM bytes per launch, rocprofv3 PMC passes of this build "
                                     "(profiles/pmc_measured.json <- profiles/<round>/)",
                     "kernel": "trace_kernel (rank 0)", "kernel_ms_avg": round(kms, 3),
                     "launches": res["launches"]})
        return roof

    res, (objs, tris, grps, cam, S, seeds_host) = run_config(args.config, args.steps, args.warmup, args.samples,
                                                             args.chunks, args.save_image,
                                                             rng=api.RNG_XOSHIRO if args.rng == "xoshiro" else 0)
    # The other BASELINE configurations at this GPU count, after the headline frames
    # (C3 / C5 are the reference's 8-GPU configurations; the driver's 1/2/4/8 runs then
    # measure their scaling too).  Secondary: `value` and `ms_per_step` are the headline's.
    extras = {}
    # The opt-in statistical RNG mode (xoshiro128**, ptmi_scene_set_rng) on the headline
    # config, reported under its own key: its images are not the reference's, so it is
    # never `value`.
    stat_rng = None
    if args.extra == "auto" and args.config == "c2" and not args.samples and not args.chunks:
        r, _ = run_config("c2", args.extra_steps, 1, rng=api.RNG_XOSHIRO)
        if rank == 0:
            stat_rng = {"value": round(r["value"], 2), "unit": "Msamples/s", "ms_per_step": round(r["ms_per_step"], 3),
                        "avg_kernel_ms": round(r["avg_kernel_ms"], 3), "steps": args.extra_steps, "warmup": 1,
                        "image_ok": r["image_ok"],
                        "what": "C2 with the opt-in statistical RNG (xoshiro128** per path instead of the "
                                "reference's noise3D): converges to the same image, does not equal it "
                                "(tests/test_gpu_rng_mode.py); not comparable to `value`"}
    extra = args.extra
    if extra == "auto":
        extra = "c3,c4,c5" if args.config == "c2" and not args.samples and not args.chunks else "none"
    for cfg in [c for c in extra.split(",") if c and c != "none" and c != args.config]:
        r, _ = run_config(cfg, args.extra_steps, 1)
        if rank == 0:
            rf = roofline(r)
            ex = {"value": round(r["value"], 2), "unit": "Msamples/s", "ms_per_step": round(r["ms_per_step"], 3),
                  "steps": args.extra_steps, "warmup": 1, "image_ok": r["image_ok"], "config": r["config"],
                  "roofline_frac": rf.get("frac"), "roofline": rf}
            if world > 1:
                ex["per_rank_kernel_ms"] = [round(float(x), 3) for x in r["per_rank"][:, 1]]
                ex["reduce_ms"] = round(float(r["per_rank"][0, 2]), 3)
            extras[cfg] = ex

    if rank == 0:
        scene_name, W, H = res["config"]["scene"], res["config"]["width"], res["config"]["height"]
        per_rank = res["per_rank"]
        value = res["value"]
        ok = res["image_ok"]
        el = res["ms_per_step"] * args.steps / 1e3
        roof = roofline(res)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(layout, objs, tris, grps, cam, S, seeds_host)
        # The drop-in call as the Go side makes it (host records and seeds in, host RGBA
        # out: scene conversion + BVH build, PCIe transfers, kernels): one frame.  The
        # bench contract fixes `value` to the HBM-resident rate; this is the rate the
        # Go caller of ocl.Trace sees (SURVEY.md 8d t_trace).
        inclusive = None
        if world == 1 and not args.no_trace_call:
            api.Trace(objs, tris, grps, device, S, cam, seeds=seeds_host)  # warm-up: host page-in, allocator
            t0 = time.perf_counter()
            api.Trace(objs, tris, grps, device, S, cam, seeds=seeds_host)
            t_call = time.perf_counter() - t0
            inclusive = {"ms": round(t_call * 1e3, 3), "value": round(W * H * S / t_call / 1e6, 2),
                         "unit": "Msamples/s", "what": "one ptmi_trace call: records + seeds from host memory, "
                                                       "scene upload and BVH build, kernels, RGBA read-back"}
        line = {
            "metric": "Msamples/sec (1280x960 ref scene)", "value": round(value, 2), "unit": "Msamples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: restated reference scene records, PCG64 per-pixel seeds",
            "config": res["config"],
            "image_ok": ok, "roofline": roof, "cpu_baseline": cpu, "ptmi_trace_call": inclusive,
        }
        line["comm"] = comm
        if world > 1:
            line["per_rank"] = {"kernel_ms": [round(float(x), 3) for x in per_rank[:, 1]],
                                "wall_s": [round(float(x), 4) for x in per_rank[:, 0]],
                                "reduce_ms": round(float(per_rank[0, 2]), 3), "shared_devices": shared}
        if extras:
            line["extra_configs"] = extras
        if stat_rng:
            line["statistical_rng"] = stat_rng
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

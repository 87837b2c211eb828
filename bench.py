#!/usr/bin/env python3
"""bench.py -- Msamples/s of the HIP path tracer on the 1280x960 reference Cornell
scene (BASELINE.json metric / configs[1]: 2048 spp, one frame per step).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

A step renders ONE complete frame (W*H*S primary samples) with the inputs (scene
records, per-pixel seeds) already resident in HBM: rank r renders its share of
the frame (sample split: samples [r*S/N, (r+1)*S/N); tile split for c5), the
per-GPU partial framebuffers are summed with an RCCL all-reduce over xGMI
(torch.distributed "nccl" backend), and the frame is normalised on device
(colors * 1/S, alpha 1; tracer.cl:1184-1187).  Total work per step is fixed
("scaling": "strong"); value = W*H*S*K / (max over ranks of the K-step time).

roofline: trace_kernel is FP64-VALU bound (the scene is 8 KB and HBM traffic is
~0.02 B/sample).  achieved = algorithmic FP64 flops per launch (frozen model,
profiles/alg_counts.json, ptmi/flops.py) / the kernel's average launch time,
measured with HIP events recorded on the launch stream around every launch in
the timed region.  peak = MI355X FP64 vector peak (78.6 TFLOP/s; equal to its
FP64 matrix peak, the "dense MFMA peak for the dtype").
cpu_baseline: the oracle's C restatement of the reference kernel (OpenMP) timed on
the host cores on a bounded sample of the same frame (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: its HIP runtime is the process's, see ptmi/_runtime.py)
import torch.distributed as dist  # noqa: E402

from ptmi import api, layout  # noqa: E402
from ptmi import dist as pdist  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

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
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (== FP64 matrix) peak, spec


def cpu_baseline(objs, tris, grps, cam, spp, seeds, budget_s=15.0):
    """Time the CPU restatement of the reference kernel on host cores (rank 0, N=1)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    if not pyoracle.cpu_available():
        return None
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16)
    w = int(np.asarray(cam).reshape(())["width"])
    h = int(np.asarray(cam).reshape(())["height"])
    t2, g2 = layout.pad_empty(tris, grps)
    # Calibrate on a centred band of rows at 2 samples, then size the sample to
    # ~budget_s: the whole frame at n_s samples when the rate allows, else a
    # centred band of rows at 1 sample.
    band = max(1, h // 16)
    t0 = time.time()
    pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, row0=(h - band) // 2, rows=band, sample_begin=0,
                       sample_end=2, threads=threads)
    rate = band * w * 2 / max(time.time() - t0, 1e-3)
    target = budget_s * rate
    if target >= w * h:
        rows, n_s = h, int(max(1, min(spp, target // (w * h))))
    else:
        rows, n_s = int(max(1, min(h, target // w))), 1
    for _ in range(3):  # re-size from the last measured run until it fills about half the budget
        row0 = (h - rows) // 2
        t0 = time.time()
        pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, row0=row0, rows=rows, sample_begin=0, sample_end=n_s,
                           threads=threads)
        el = time.time() - t0
        if el >= 0.5 * budget_s or (rows == h and n_s == spp):
            break
        work = rows * n_s * budget_s / max(el, 1e-3)
        if rows < h:
            rows = int(max(1, min(h, work)))
        else:
            n_s = int(max(1, min(spp, work // h)))
    return {"value": rows * w * n_s / el / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d rows x %d px x samples [0,%d) of the %d-spp frame (%.1f s)" % (rows, w, n_s, spp, el)}


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
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    scene_name, W, H, S, aper, focal, split, alg_key, desc = CONFIGS[args.config]
    if args.samples:
        S = args.samples
    objs, tris, grps, cam = scene_inputs(scene_name, W, H, aper, focal)
    scene = api.Scene(local, objs, tris, grps, cam)
    npix = W * H
    seeds_host = layout.seeds_go_float64(npix, 1234)
    seeds = torch.tensor(seeds_host, dtype=torch.float64, device="cuda")
    sums = torch.empty(npix * 4, dtype=torch.float64, device="cuda")
    img = torch.empty(npix * 4, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    s0, s1, t_stride, t_off = pdist.shard(rank, world, S, split)

    def step():
        scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=t_stride, tile_offset=t_off,
                     chunks=args.chunks, stream=stream)
        pdist.reduce_frame(sums)  # RCCL all-reduce over xGMI of the partial framebuffers (N > 1)
        scene.finalize(sums.data_ptr(), img.data_ptr(), S, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    scene.kernel_time()  # drop warmup launches
    scene.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kms, klaunch = scene.kernel_time()
    scene.set_timing(False)
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    # sanity: a finite image with alpha 1
    im = img.view(H, W, 4)
    ok = bool(torch.isfinite(im).all().item()) and bool((im[..., 3] == 1.0).all().item())
    if args.save_image and rank == 0:
        np.save(args.save_image, im.cpu().numpy())

    if rank == 0:
        total = W * H * S * args.steps
        value = total / el / 1e6
        roof = None
        try:
            with open(os.path.join(ROOT, "profiles", "alg_counts.json")) as f:
                ac = json.load(f)["workloads"][alg_key]
            f64 = ac["fp64_flops_per_sample"]
            my_samples_per_launch = npix * (s1 - s0) if split == "sample" else \
                W * H * S / max(world, 1)
            avg_ms = kms / max(klaunch, 1)
            achieved = f64 * my_samples_per_launch / (avg_ms * 1e-3) / 1e12
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
            if os.path.exists(pmc):
                with open(pmc) as f:
                    traffic = json.load(f).get("hbm_bytes_per_launch")
            roof = {"bound": "mfma", "bound_detail": "fp64 VALU (no MFMA; FP64 vector peak == FP64 matrix peak)",
                    "achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / FP64_PEAK_TFLOPS, 4), "traffic": traffic,
                    "kernel": "trace_kernel", "kernel_ms_avg": round(avg_ms, 3), "launches": klaunch,
                    "fp64_flops_per_sample": round(f64, 1)}
        except (OSError, KeyError) as e:
            roof = {"error": "alg counts unavailable: %s" % e}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(objs, tris, grps, cam, S, seeds_host)
        # The drop-in call as the Go side makes it (host records and seeds in, host
        # RGBA out: scene conversion + BVH build, PCIe transfers, kernels): one frame,
        # reported beside `value`, never as it.
        inclusive = None
        if world == 1 and not args.no_trace_call:
            t0 = time.perf_counter()
            api.Trace(objs, tris, grps, local, S, cam, seeds=seeds_host)
            t_call = time.perf_counter() - t0
            inclusive = {"ms": round(t_call * 1e3, 3), "value": round(W * H * S / t_call / 1e6, 2),
                         "unit": "Msamples/s", "what": "one ptmi_trace call: records + seeds from host memory, "
                                                       "scene upload and BVH build, kernels, RGBA read-back"}
        line = {
            "metric": "Msamples/sec (1280x960 ref scene)", "value": round(value, 2), "unit": "Msamples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: restated reference scene records, PCG64 per-pixel seeds",
            "config": {"workload": desc, "scene": scene_name, "width": W, "height": H, "spp": S,
                       "aperture": aper, "focal_length": focal, "split": split,
                       "parallelism": "%s-split x%d + RCCL allreduce" % (split, world) if world > 1 else "single GPU"},
            "image_ok": ok, "roofline": roof, "cpu_baseline": cpu, "ptmi_trace_call": inclusive,
        }
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

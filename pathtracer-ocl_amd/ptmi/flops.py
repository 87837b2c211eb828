"""Algorithmic FP64 flop model of the path (roofline numerator for bench.py).

Convention: mul / add / sub / div / sqrt = 1 flop, FMA = 2, a
transcendental = the FP64 arithmetic of its executed ocml path (FMA = 2):
    sin / cos (small-argument path: trigredsmall + sincosred2)   57
    pow (epln + expep, double-double log/exp)                    170
    rsqrt (as sqrt + div)                                          2
Vector helpers, as written in the kernel (and the reference builtins):
    mat_mul 28 (16 mul + 12 add), dot4 7 (mul + 3 fma), cross4 9 (3 x (mul + fma)),
    normalize4 13 (dot4 + rsqrt + 4 mul).
Events are counted by the oracle's instrumented build (oracle/pt_oracle.c,
-DPTO_COUNT) on a sample of the benchmark workload and frozen in
profiles/alg_counts.json; misses re-traced by the reference (tracer.cl:884) and
divergence waste are NOT algorithmic work and are not counted.
FP32 work (the noise3D RNG, ~28 flops per call) is reported separately.
"""
EVENTS = ["sample", "camera", "camera_dof", "obj_test", "plane", "sphere", "sphere_disc", "cyl", "cyl_disc",
          "cube", "group_box", "node_box", "tri_det", "tri_u", "tri_v", "tri_full", "hit", "nrm_sphere",
          "nrm_cyl", "nrm_cube", "nrm_tri", "reflect", "schlick", "schlick_tir_branch", "refract", "under",
          "diffuse", "reduce", "noise"]

FP64_COST = {
    "sample": 3,         # colors += accum (xyz)
    "camera": 79,        # 2 mul + 2 add + 2 sub + 2 mat_mul + sub4 + normalize4
    "camera_dof": 150,   # pos (8) + sunflower (2 sqrt, 2 div, ~12 mul/add, cos + sin) + origin/dir (8)
    "obj_test": 56,      # 2 mat_mul (ray into object space)
    "plane": 1,          # -o.y / d.y
    "sphere": 31,        # vtc (4) + 3 dot4 + 2 mul + disc (4)
    "sphere_disc": 7,    # sqrt + 2 x (sub, mul, div)
    "cyl": 16,
    "cyl_disc": 11,
    "cube": 12,          # 3 checkAxis (2 sub + 2 div)
    "group_box": 12,
    "node_box": 12,
    "tri_det": 16,       # cross4 + dot4
    "tri_u": 13,         # div + sub4 + dot4 + mul
    "tri_v": 18,         # cross4 + dot4 + mul + add
    "tri_full": 8,       # dot4 + mul
    "hit": 64,           # pos (8) + mat_mul(invT) + normalize4 + dot4 + overPoint (8)
    "nrm_sphere": 32, "nrm_cyl": 31, "nrm_cube": 28, "nrm_tri": 22,
    "reflect": 19,       # dot4 + 8 mul + 4 sub
    "schlick": 185,      # dot4 + pow + 8
    "schlick_tir_branch": 7,
    "refract": 29,
    "under": 8,
    "diffuse": 184,      # 2 cross4 + normalize4 + cos + sin + 3 sqrt + 24 vector ops + dot4
    "reduce": 12,        # accum += mask*em (6) + mask *= color, cos (6)
    "noise": 0,
}
FP32_COST = {"noise": 28}


def flops_per_sample(counts):
    """counts: {event: total} for N samples -> (fp64 flops/sample, fp32 flops/sample)."""
    n = counts["sample"]
    f64 = sum(FP64_COST[e] * counts[e] for e in EVENTS) / n
    f32 = sum(FP32_COST.get(e, 0) * counts[e] for e in EVENTS) / n
    return f64, f32


# Algorithmic bytes of the BVH scenes' memory traffic: under the
# reference's visit rules (tracer.cl:617-719) every node whose box is tested is fetched
# (64 B: its box + children, compact), every triangle tested fetches p1, e1, e2 (72 B of
# FP64) and every winning triangle its normals and colour (96 B).
BYTES = {"node_box": 64, "tri_det": 72, "nrm_tri": 96}


def bytes_per_sample(counts):
    """counts: {event: total} for N samples -> algorithmic HBM bytes per sample."""
    return sum(b * counts[e] for e, b in BYTES.items()) / counts["sample"]

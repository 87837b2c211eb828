"""DIAGNOSTIC: where do scratch (spill) ops sit relative to loops in a kernel's ISA?
    python tools/isa_loops.py <file.s> <kernel-substring>
A loop = [label, backward branch to it]; prints each loop's size and its scratch ops."""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_ZN4ptmi12trace_kernel" + sys.argv[2] + r"\w*):[^\n]*\n(.*?)\n\s*s_endpgm", s, re.S | re.M)
lines = m.group(2).split("\n")
ins, labels = [], {}
for l in lines:
    t = l.split(";")[0].strip()
    if not t:
        continue
    if t.endswith(":"):
        labels[t[:-1]] = len(ins)
        continue
    if t.startswith("."):
        continue
    ins.append(t)
loops = []
for i, t in enumerate(ins):
    mm = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", t)
    if mm and mm.group(2) in labels and labels[mm.group(2)] <= i:
        loops.append((labels[mm.group(2)], i))
print("instructions", len(ins), "loops", len(loops))
for a, b in sorted(loops, key=lambda x: x[1] - x[0]):
    sc = [j for j in range(a, b + 1) if "scratch_" in ins[j]]
    f64 = sum(1 for j in range(a, b + 1) if "_f64" in ins[j])
    print("loop [%5d,%5d] size %5d  f64 %4d  scratch %3d" % (a, b, b - a + 1, f64, len(sc)))

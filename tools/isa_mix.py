"""Instruction mix of one kernel in a hipcc -S listing (static counts, whole body or a loop).

    python tools/isa_mix.py listing.s KERNEL_SUBSTRING
"""
import collections
import re
import sys

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = [l.strip() for l in lines[start:end] if l.startswith("\t") and not l.strip().startswith((";", "."))]
cls = collections.Counter()
ops = collections.Counter()
for l in body:
    op = l.split()[0]
    ops[op] += 1
    if op.startswith("v_mfma"):
        cls["mfma"] += 1
    elif op.startswith("v_"):
        cls["valu"] += 1
    elif op.startswith("ds_"):
        cls["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cls["vmem"] += 1
    elif op.startswith("s_"):
        cls["salu"] += 1
print(lines[start][:100])
print(dict(cls), "valu/mfma", round(cls["valu"] / max(cls["mfma"], 1), 2))
for op, n in ops.most_common(45):
    print(f"  {op:32s} {n}")

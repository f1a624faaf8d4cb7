"""Symbolize tools/hostbench/sprof.c samples: per-function sample counts
(each object's symbol table via nm, offsets bisected), top N."""
import bisect
import collections
import subprocess
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/sprof.txt"
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
by_obj = collections.defaultdict(list)
total = 0
for ln in open(path):
    c, obj, off = ln.split()
    by_obj[obj].append((int(off, 16), int(c)))
    total += int(c)


def symbols(obj):
    out = subprocess.run(["nm", "-C", "--defined-only", "-n", obj], capture_output=True, text=True).stdout
    if not out.strip():
        out = subprocess.run(["nm", "-D", "-C", "--defined-only", "-n", obj], capture_output=True, text=True).stdout
    addrs, names = [], []
    for ln in out.splitlines():
        parts = ln.split(" ", 2)
        if len(parts) == 3 and parts[1] in "tTwW":
            addrs.append(int(parts[0], 16))
            names.append(parts[2])
    return addrs, names


funcs = collections.Counter()
for obj, offs in by_obj.items():
    if obj == "?":
        funcs["?"] += sum(c for _, c in offs)
        continue
    addrs, names = symbols(obj)
    for off, c in offs:
        k = bisect.bisect_right(addrs, off) - 1
        name = names[k] if k >= 0 else "?"
        funcs[f"{obj.rsplit('/', 1)[-1]}: {name[:120]}"] += c
print(f"{total} samples")
for name, c in funcs.most_common(top):
    print(f"{100.0 * c / total:6.2f}%  {c:7d}  {name}")

"""Diff two tools/trace_steps.py step breakdowns: per-kernel ms/step A - B."""
import re
import sys


def load(p):
    d = {}
    for line in open(p):
        m = re.match(r"\s+([\d.]+) ms\s+[\d.]+%\s+n=\s*(\d+) avg=\s*([\d.]+)us\s+(.*)", line)
        if m:
            d[m.group(4).strip()] = (float(m.group(1)), int(m.group(2)))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
rows = sorted(((a.get(k, (0, 0))[0] - b.get(k, (0, 0))[0], k) for k in set(a) | set(b)), reverse=True)
n = int(sys.argv[3]) if len(sys.argv) > 3 else 15
for r in rows[:n]:
    print(f"{r[0]:+.3f} ms  A {a.get(r[1], (0, 0))[0]:.3f}  B {b.get(r[1], (0, 0))[0]:.3f}  {r[1][:95]}")
print("...")
for r in rows[-5:]:
    print(f"{r[0]:+.3f} ms  A {a.get(r[1], (0, 0))[0]:.3f}  B {b.get(r[1], (0, 0))[0]:.3f}  {r[1][:95]}")
for p in sys.argv[1:3]:
    print(open(p).readline().strip())

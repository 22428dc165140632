"""Find global loads the compiler waits on immediately (s_waitcnt vmcnt(0) right after the load): each
is a full memory round trip the wave cannot overlap with its other loads -- typically a per-lane guarded
load whose value is converted inside the guard.  Compiles each .hip to gfx950 assembly (--save-temps).

    python tools/asm_serial_loads.py [file.hip ...]      (default: every csrc/*.hip)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "outlook-grid-vision-transformer_amd",
                    "csrc")


def demangle(n):
    return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()


def scan(path):
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", path, "-o",
                        os.path.join(d, "x.o"), "--save-temps"], cwd=d, capture_output=True)
        s = glob.glob(os.path.join(d, "*gfx950.s"))
        if not s:
            print("  (no assembly)", path)
            return
        lines = open(s[0]).read().split("\n")
    cur, stats = None, {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur = m.group(1)
            stats[cur] = [0, 0]
        if cur and re.search(r"\b(global|buffer)_load", l):
            stats[cur][0] += 1
            for j in range(i + 1, min(i + 4, len(lines))):
                t = lines[j].strip()
                if not t or t.startswith(";"):
                    continue
                if t.startswith("s_waitcnt vmcnt(0)"):
                    stats[cur][1] += 1
                break
    for k, (a, b) in stats.items():
        if b:
            print(f"  {b:3d}/{a:3d}  {re.sub(r'[(].*', '', demangle(k))[:110]}")


def main(files):
    for f in [os.path.abspath(x) for x in files] or sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        print(os.path.basename(f))
        scan(f)


if __name__ == "__main__":
    main(sys.argv[1:])

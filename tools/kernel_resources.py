"""Compact per-kernel register / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.   python tools/kernel_resources.py file.hip [...]"""
import re
import subprocess
import sys

CSRC = "outlook-grid-vision-transformer_amd/csrc"


def main(files):
    for f in files:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", f,
                              "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                             capture_output=True, text=True).stderr
        cur = None
        rows = []
        for line in out.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
            if m and cur is not None:
                cur[m.group(1).split()[0]] = int(m.group(2))
        for r in rows:
            name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
            name = re.sub(r"\(.*", "", name)
            print(f"{name[:78]:78s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize')} "
                  f"occ={r.get('Occupancy')} lds={r.get('LDS')}")


if __name__ == "__main__":
    main(sys.argv[1:])

"""Print per-kernel VGPR/AGPR/scratch/occupancy of a HIP source (hipcc resource remarks).
usage: python scripts/kres.py path/to/file.hip [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*)$", line)
    if not m:
        continue
    t = m.group(1).replace("[-Rpass-analysis=kernel-resource-usage]", "").strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{name[:90]:90s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize [bytes/lane]')} "
          f"occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")

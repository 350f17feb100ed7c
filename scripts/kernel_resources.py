"""Per-kernel VGPRs / scratch / occupancy / LDS of the HIP library, from the compiler's
resource-usage remarks (no GPU needed).  Flags any kernel with scratch (private memory):
on this path scratch means a register array mirrored to memory, a large hidden cost.

    python scripts/kernel_resources.py [--all]
"""
import re
import subprocess
import sys

SRC = "maskclustering_amd/csrc/mc_api.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-c",
       "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage", SRC, "-o", "/tmp/_mc_res.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip().split("(")[0]}
        rows.append(cur)
    else:
        cur[k.split()[0]] = int(v)
bad = 0
for r in rows:
    if "--all" in sys.argv or r.get("ScratchSize", 0):
        print(f"{r['name']:40s} vgpr {r.get('VGPRs'):4d} scratch {r.get('ScratchSize'):4d} occ {r.get('Occupancy'):2d} "
              f"lds {r.get('LDS'):6d}")
    bad += r.get("ScratchSize", 0) > 0
print(f"{len(rows)} kernels, {bad} with scratch")

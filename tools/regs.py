"""Per-kernel register / spill / LDS table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/regs.py nerf-or-nothing_amd/csrc/kernels/mlp_fwd16.hip [more.hip ...]
"""
import re
import subprocess
import sys

FLAGS = [*__import__("os").environ.get("REGS_DEFS", "").split(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fhip-fp32-correctly-rounded-divide-sqrt", "-c",
         "-o", "/tmp/regs.o", "-Rpass-analysis=kernel-resource-usage"]
for src in sys.argv[1:]:
    out = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, src], capture_output=True, text=True).stderr
    cur, d = None, {}
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur, d = m.group(1), {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            d[m.group(1)] = m.group(2)
            if m.group(1).startswith("LDS"):
                print(f"{cur[:64]:64s} vgpr={d.get('VGPRs')} agpr={d.get('AGPRs')} spill={d.get('VGPRs Spill')} "
                      f"lds={d[m.group(1)]}")

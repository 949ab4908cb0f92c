"""Print per-kernel VGPR/SGPR/spill/occupancy from hipcc -Rpass-analysis=kernel-resource-usage."""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "netcode_amd/csrc/ntc_gf256.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude", "-c", src,
       "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v; rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for f, d in rows.items():
    print(f"{f[:60]:60s} VGPR={d.get('VGPRs'):>4} AGPR={d.get('AGPRs','-'):>3} SGPR={d.get('TotalSGPRs'):>4} "
          f"Sspill={d.get('SGPRs Spill'):>4} Vspill={d.get('VGPRs Spill','-'):>3} scratch={d.get('ScratchSize [bytes/lane]'):>4} occ={d.get('Occupancy [waves/SIMD]')} lds={d.get('LDS Size [bytes/block]')}")

"""Per-kernel register / LDS / spill table of one HIP source (gfx950), from
hipcc's -Rpass-analysis=kernel-resource-usage remarks.

usage: python tools/kres.py diffopt.jl_amd/csrc/qp_nopiv.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", src,
       "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?)(?: \[-Rpass)", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    if flt and flt not in name:
        continue
    print(f"{name[:110]:110s} V={r.get('VGPRs','?'):>4s} A={r.get('AGPRs','?'):>3s} "
          f"spV={r.get('VGPRs Spill','?'):>3s} spS={r.get('SGPRs Spill','?'):>3s} "
          f"LDS={r.get('LDS Size [bytes/block]','?'):>6s} occ={r.get('Occupancy [waves/SIMD]','?')}")

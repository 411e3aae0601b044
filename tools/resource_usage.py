"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output per kernel."""
import re
import subprocess
import sys

cmd = sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: \s*([A-Za-z \[\]/]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"gbp::TerrainView<(\w+)>", r"TV<\1>", name)
    name = name.split("(")[0] + ("<f32>" if "TV<float>" in name else "")
    print(f"{name[:60]:60s} vgpr={v.get('VGPRs'):>4} agpr={v.get('AGPRs','-'):>3} "
          f"sgpr={v.get('TotalSGPRs'):>4} scratch={v.get('ScratchSize [bytes/lane]'):>4} "
          f"occ={v.get('Occupancy [waves/SIMD]')}")

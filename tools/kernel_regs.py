"""Print per-kernel register/LDS/spill metadata from a hipcc -S device assembly file."""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    def f(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, blk)
        return m.group(1) if m else "-"
    name = f("name")
    if len(sys.argv) > 2 and not re.search(sys.argv[2], name):
        continue
    print(f"{name[:70]:70s} vgpr={f('vgpr_count'):>4} agpr={f('agpr_count'):>4} "
          f"sgpr={f('sgpr_count'):>4} vspill={f('vgpr_spill_count'):>4} sspill={f('sgpr_spill_count'):>4} "
          f"lds={f('group_segment_fixed_size'):>6} scratch={f('private_segment_fixed_size')}")

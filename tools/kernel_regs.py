"""Per-kernel register / scratch / LDS figures from a gfx950 .s (hipcc -save-temps) metadata
block: usage python tools/kernel_regs.py file.s [name-substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = f.get("name", "?")
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    print(f"{name[:70]:70s} vgpr {f.get('vgpr_count')} agpr {f.get('agpr_count')} "
          f"sgpr {f.get('sgpr_count')} scratch {f.get('private_segment_fixed_size')} "
          f"lds {f.get('group_segment_fixed_size')}")

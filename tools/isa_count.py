"""Static instruction mix of one kernel in a gfx950 .s (hipcc -save-temps):
usage python tools/isa_count.py file.s name-substring"""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = None
for i, ln in enumerate(txt):
    if re.match(r"^[A-Za-z_]\w*:", ln) and pat in ln.split(":")[0]:
        start = i
        break
if start is None:
    sys.exit("kernel not found")
cnt = collections.Counter()
for ln in txt[start + 1:]:
    if ln.startswith("\t.size") or ln.startswith(".Lfunc_end"):
        break
    s = ln.strip()
    if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
        continue
    op = s.split()[0]
    cnt[op] += 1
tot = sum(cnt.values())
valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
f64 = sum(v for k, v in cnt.items() if k.startswith("v_") and "f64" in k)
print(f"{txt[start].split(':')[0][:60]}: total {tot} valu {valu} f64 {f64} "
      f"salu {sum(v for k, v in cnt.items() if k.startswith('s_'))} "
      f"vmem {sum(v for k, v in cnt.items() if k.startswith(('global_', 'buffer_')))} "
      f"lds {sum(v for k, v in cnt.items() if k.startswith('ds_'))}")
for k, v in cnt.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
    print(f"  {k:28s} {v}")

"""Static instruction mix of the kernels in a hipcc -S (gfx950) listing whose symbol contains every
given substring.  usage: python3 tools/isa_count.py file.s substr [substr ...]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
keys = sys.argv[2:]
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    if not all(k in name for k in keys):
        continue
    end = s.find(".Lfunc_end", m.end())
    ins = []
    for line in s[m.end():end].splitlines():
        t = line.strip()
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        ins.append(t.split()[0])
    c = collections.Counter(ins)
    valu = sum(n for k, n in c.items() if k.startswith("v_"))
    tail = s[end:end + 4000]
    vg = re.search(r"NumVgprs: (\d+)", s[m.start():end + 200000])
    print(f"{name[:90]}\n  total {len(ins)}  valu {valu}  vgprs {vg.group(1) if vg else '?'}")
    print("  " + ", ".join(f"{k} {n}" for k, n in c.most_common(40)))

"""Instruction mix of the main loop of each kernel in a hipcc -S listing (diagnostic).
    python scripts/loopmix.py LISTING.s [name-substring ...]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
pats = sys.argv[2:]
starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
for st in starts:
    name = lines[st].split(":")[0]
    if pats and not any(p in name for p in pats):
        continue
    en = st + 1
    while not lines[en].startswith(".Lfunc_end"):
        en += 1
    b = lines[st:en]
    hdrs = [l for l in b if "Loop Header: Depth=1" in l]
    if not hdrs:
        continue
    hb = hdrs[0].split(":")[0].strip().lstrip(".L")
    inloop, lb = False, []
    for l in b:
        if re.match(r"^\.LBB\d+_\d+:", l) or l.startswith("; %bb."):
            inloop = (hb in l and "Loop Header" in l) or (f"Header={hb} " in l)
            continue
        t = l.strip()
        if inloop and t and not t.startswith((".", ";")):
            lb.append(t)
    c = collections.Counter(x.split()[0] for x in lb)
    cnt = lambda p: sum(v for k, v in c.items() if re.match(p, k))
    print(f"{name[:90]}\n   instrs {len(lb)} mfma {cnt(r'v_mfma')} valu {cnt(r'v_(?!mfma)')} "
          f"salu {cnt(r's_(?!waitcnt|cbranch|branch|barrier)')} branch {cnt(r's_c?branch')} "
          f"vmem {cnt(r'(global|buffer)_load')} ds {cnt(r'ds_')} wait {cnt(r's_waitcnt')}")

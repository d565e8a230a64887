"""LDS bank model of the halo conv (halo_conv.hip) A-fragment reads (ds_read_b128, gfx950 lane groups) and staging
writes (ds_write_b64) for the padded rows (lds_stride) and XOR-swizzled compact rows: worst multiplicity per
access (1 = conflict-free), per channel-chunk width and kernel size.  Diagnostic: python scripts/halo_swizzle_check.py"""
# LDS bank model for the halo conv A-fragment reads (ds_read_b128) and staging writes (ds_write_b64) under
# candidate layouts.  B128 lane groups from scripts/lds_swizzle_check.py (gfx950).
from collections import Counter
B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128 += [[l + 32 for l in g] for g in B128]

def read_worst(CC, KW, KH, HWd, SA, addr):
    ntap = KH * KW; steps = -(-ntap * CC // 32)
    w = 1
    for wv in range(8):
        for a in range(2):
            for s in range(steps):
                slots = {}
                for lane in range(64):
                    q, r16 = lane >> 4, lane & 15
                    r0 = s * 32 + 8 * q
                    tap, cc = r0 // CC, r0 % CC
                    if tap >= ntap: tap, cc = 0, 0
                    kh, kw = tap // KW, tap % KW
                    row = (2 * wv + a) * HWd + r16 + kh * HWd + kw
                    slots[lane] = (addr(row, cc >> 3) // 16) % 16
                for g in B128:
                    w = max(w, max(Counter(slots[l] for l in g).values()))
    return w

def write_worst(CC, HP, SA, addr, NT=512):
    # stage_a: idx = base + u*NT + tid; hp = idx // (CC/4), c4 = idx % (CC/4): ds_write_b64 (bank (a/4)%32; halves of 32 lanes)
    nc4 = CC // 4; total = HP * nc4; w = 1
    for base in range(0, total, 64):
        offs = []
        for lane in range(64):
            idx = base + lane
            if idx >= total: continue
            hp, c4 = idx // nc4, idx % nc4
            offs.append((lane, addr(hp, c4 >> 1) + 8 * (c4 & 1)))
        for half in range(2):
            # 8-byte writes: each lane covers 2 banks of 4 B; count per 4-B bank over 32 banks
            cnt = Counter()
            for lane, o in offs:
                if lane // 32 == half:
                    cnt[(o // 4) % 32] += 1; cnt[(o // 4 + 1) % 32] += 1
            if cnt: w = max(w, max(cnt.values()) / 2)   # a conflict-free b64 half-wave touches each bank twice (2 passes)
    return w

def lds_stride(cc):
    s = cc
    while (s // 8) % 4 != 2: s += 8
    return s

for CC, KW, KH in ((32, 7, 7), (24, 3, 3), (64, 5, 5), (16, 3, 3), (32, 3, 3), (64, 3, 3)):
    HWd = 16 + KW - 1; HP = (16 + KH - 1) * HWd
    sa0 = lds_stride(CC)
    cur = lambda r, c, sa=sa0: r * sa * 2 + 16 * c
    res = [f"CC{CC} k{KW}: current SA {sa0}: read {read_worst(CC, KW, KH, HWd, sa0, cur)} write {write_worst(CC, HP, sa0, cur)}"]
    sa = 32 if CC <= 32 else 64
    cpr = sa // 8
    for name, f in (("(r>>2)", lambda r, m=cpr - 1: (r >> 2) & m), ("r", lambda r, m=cpr - 1: r & m),
                    ("(r>>1)", lambda r, m=cpr - 1: (r >> 1) & m), ("r^(r>>2)", lambda r, m=cpr - 1: (r ^ (r >> 2)) & m),
                    ("(r>>2)^(r>>4)", lambda r, m=cpr - 1: ((r >> 2) ^ (r >> 4)) & m)):
        ad = lambda r, c, sa=sa, f=f: r * sa * 2 + 16 * (c ^ f(r))
        res.append(f"  SA {sa} swz {name}: read {read_worst(CC, KW, KH, HWd, sa, ad)} write {write_worst(CC, HP, sa, ad)}")
    print("\n".join(res))
print("---")
for CC, KW, KH in ((56, 3, 3), (56, 5, 5), (24, 7, 7), (24, 5, 5), (64, 7, 7), (32, 5, 5)):
    HWd = 16 + KW - 1; HP = (16 + KH - 1) * HWd
    sa = 32 if CC <= 32 else 64
    f = (lambda r: (r >> 1) & 3) if sa == 32 else (lambda r: r & 7)
    ad = lambda r, c, sa=sa, f=f: r * sa * 2 + 16 * (c ^ f(r))
    sa0 = lds_stride(CC); cur = lambda r, c, sa=sa0: r * sa * 2 + 16 * c
    print(CC, KW, "cur", sa0, read_worst(CC, KW, KH, HWd, sa0, cur), "swz", sa, read_worst(CC, KW, KH, HWd, sa, ad), write_worst(CC, HP, sa, ad))

"""LDS bank model of the B-fragment reads (ds_read_b128) and search for XOR swizzle keys.

A 16x16x32 MFMA operand read puts lane 16 q + n on row n (the pixel / row of the tile) and 16-B chunk
4 c + q (bf16; f32 operands read chunks 8 c + 2 q, + 1). ds_read_b128 serves a wave in four 16-lane groups
(MI355X_MICROARCH.md, LDS table): {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, and the same + 32. A group
is conflict-free when its 16 lanes hit 16 different 16-B bank slots ((row * row_bytes / 16 + chunk) mod 16).
Rows n = 0-3, 12-15 of quarter q share a group with rows 4-11 of quarter q ^ 1, so a key that separates
16 rows (key = row & 15) is not enough once the tile's rows are shifted (a 3x3 tap): key = y left the
shifted thirds of repblocks.hip's reads and the odd shifts of conv_halo.hip's reads 2-way conflicted.

  python tools/swizzle_search.py          # report the kernels' keys under the model, then search
"""
import sys

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def ways(rows, key, row_bytes=512, f32=False, c=0, h=0):
    """Worst bank-slot multiplicity over the four lane groups; rows[n] = the row lane n reads."""
    worst = 0
    for g in GROUPS:
        slots = {}
        for lane in g:
            q, n = lane >> 4, lane & 15
            r = rows[n]
            chunk = ((8 * c + 2 * q + h) if f32 else (4 * c + q)) ^ key(r)
            s = (r * row_bytes // 16 + chunk) % 16
            slots[s] = slots.get(s, 0) + 1
        worst = max(worst, max(slots.values()))
    return worst


def hkey(r):  # conv_halo.hip / repblocks.hip (256- and 512-B rows)
    return ((r << 1) & 6) | (((r >> 2) & 1) * 9)


def xkey(r):  # conv_x6.hip (f32 rows): hkey with bits 0 and 1 swapped
    return (r & 1) | (((r >> 2) & 1) * 10) | (((r >> 1) & 1) << 2)


def stem_key(r):  # repblocks.hip 128-B rows (the stem input)
    return (0x7662265544022100 >> (4 * r)) & 7


def report():
    for name, key in (("row & 15", lambda r: r & 15), ("hkey", hkey)):
        sh = [ways([r0 + n for n in range(16)], key) for r0 in range(32)]
        tr = [ways([(n + dy) & 15 for n in range(16)], key) for dy in (-1, 0, 1)]
        print(f"bf16 {name:9s} any-shift windows: max {max(sh)}-way; repblocks dy=-1,0,1: {tr}")
    for name, key in (("row & 15", lambda r: r & 15), ("xkey", xkey)):
        sh = [ways([r0 + n for n in range(16)], key, 1024, True, 0, h) for r0 in range(32) for h in (0, 1)]
        print(f"f32  {name:9s} any-shift windows: max {max(sh)}-way")
    for name, key in (("y >> 1", lambda r: r >> 1), ("stem_key", stem_key)):
        tr = [max(ways([(n + dy) & 15 for n in range(16)], key, 128, False, c) for c in (0, 1)) for dy in (-1, 0, 1)]
        print(f"128-B {name:8s} repblocks dy=-1,0,1: {tr}")
    # ds_write_b64 of a 16-row write-back (bank = (addr / 4) mod 32: slot = key & 7): 2-way is the minimum
    from collections import Counter
    print("hkey write-back slots per 16 rows:", max(Counter(hkey(r) & 7 for r in range(16)).values()), "-way")


def search(period=16, write_two_way=True):
    """DFS for a key over `period` rows (values 0..15) conflict-free for every consecutive 16-row window."""
    a_rows = [0, 1, 2, 3, 12, 13, 14, 15]
    b_rows = list(range(4, 12))

    def ok(k):
        n = len(k)
        for r0 in range(period):
            ya = [(r0 + i) % period for i in a_rows if (r0 + i) % period < n]
            yb = [(r0 + i) % period for i in b_rows if (r0 + i) % period < n]
            vals = [k[y] for y in ya] + [k[y] ^ 1 for y in yb]
            if len(vals) != len(set(vals)):
                return False
        if write_two_way:
            cnt = {}
            for v in k:
                cnt[v & 7] = cnt.get(v & 7, 0) + 1
            if max(cnt.values()) > 2:
                return False
        return True

    k = []

    def dfs():
        if len(k) == period:
            return True
        for v in range(16):
            k.append(v)
            if ok(k) and dfs():
                return True
            k.pop()
        return False

    return list(k) if dfs() else None


if __name__ == "__main__":
    report()
    if "--search" in sys.argv:
        print("search:", search())

"""The LDS bank model of the MFMA operand reads (tools/swizzle_search.py) and the swizzle keys the kernels use:
repblocks.hip rf::key (256/512-B rows: every dy shift; 128-B stem rows: a table), conv_halo.hip hkey (any 16
consecutive rows), conv_x6.hip xkey (f32 rows, chunks 8c + 2q): conflict-free in every ds_read_b128 lane group,
and the round-3 keys reproduce the conflicts the SQ counters measured. CPU only."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("swizzle_search", os.path.join(ROOT, "tools", "swizzle_search.py"))
sw = importlib.util.module_from_spec(spec)
spec.loader.exec_module(sw)


def test_lane_groups_partition_the_wave():
    lanes = sorted(lane for g in sw.GROUPS for lane in g)
    assert lanes == list(range(64)) and all(len(g) == 16 for g in sw.GROUPS)


def test_halo_key_any_shift_conflict_free_and_row_key_is_not():
    for rb in (256, 512):
        assert max(sw.ways([r0 + n for n in range(16)], sw.hkey, rb) for r0 in range(64)) == 1
    # key = row & 15 (round 3): 2-way at odd shifts
    assert max(sw.ways([r0 + n for n in range(16)], lambda r: r & 15) for r0 in range(16)) == 2


def test_repblocks_keys_every_row_shift():
    for dy in (-1, 0, 1):
        rows = [(n + dy) & 15 for n in range(16)]  # out-of-image lanes read the wrapped row
        for rb in (256, 512):
            assert sw.ways(rows, sw.hkey, rb) == 1
        assert max(sw.ways(rows, sw.stem_key, 128, False, c) for c in (0, 1)) == 1
    assert sw.ways([n + 1 if n < 15 else n for n in range(16)], lambda r: r) == 2  # key = y, clamped row


def test_x6_key_f32_rows():
    for r0 in range(32):
        rows = [r0 + n for n in range(16)]
        assert all(sw.ways(rows, sw.xkey, rb, True, 0, h) == 1 for rb in (512, 1024) for h in (0, 1))
    assert max(sw.ways([n + 3 for n in range(16)], sw.hkey, 1024, True, 0, h) for h in (0, 1)) == 2


def test_write_back_two_way_minimum():
    slots = [sw.hkey(r) & 7 for r in range(16)]
    assert max(slots.count(v) for v in set(slots)) == 2

"""Bank-conflict model of the training kernels' LDS layouts (csrc/hpe_mlp2.hip): the 12-wave
mlp2_kernel, the 4-wave mlp2_kernel (narrow layers at P < 2^15 rows, the split path that splits X
per wave) and mlp2r_kernel (F <= 64, large launches).

The lane groups and bank rules are MI355X_MICROARCH.md §LDS's table: ds_read_b128 serves a wave in
four 16-lane groups, bank of dword d = d mod 64, one LDS cycle per group when every bank holds at
most one distinct address; ds_read_b32 / ds_write_b32 in two 32-lane groups, bank = d mod 32.  The
constants below restate the kernel's (MLP2_FS, MLP2_TS, a1_row); each test walks the lanes of one
access exactly as the kernel computes its address and counts the LDS cycles.
"""
import pytest

B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
B128_GROUPS += [[lane + 32 for lane in g] for g in B128_GROUPS]
B32_GROUPS = [list(range(32)), list(range(32, 64))]

MLP2_FS = 104   # halves per row of the forward image
MLP2_TS = 40    # halves per channel of the transposed image


def a1_row(g):  # csrc/hpe_mlp2.hip a1_row
    return 68 * (g ^ ((g >> 1) & 4))


def cycles(addr, groups, width, nbanks):
    """LDS cycles of one wave-instruction: addr[lane] = first dword the lane touches."""
    total = 0
    for grp in groups:
        banks = {}
        for lane in grp:
            for d in range(width):
                banks.setdefault((addr[lane] + d) % nbanks, set()).add(addr[lane] + d)
        total += max(len(v) for v in banks.values())
    return total


def test_a1_park_head_reads_conflict_free():
    # head partials: lane (r = l32, half h) reads row gr = (r & 3) + 4 (r >> 3), dwords
    # hh 32 + 16 h + i .. + 3 (hh = (r >> 2) & 1), i = 0, 4, 8, 12
    for i in (0, 4, 8, 12):
        addr = {}
        for lane in range(64):
            r, h = lane & 31, lane >> 5
            hh, gr = (r >> 2) & 1, (r & 3) + 4 * (r >> 3)
            addr[lane] = a1_row(gr) + hh * 32 + 16 * h + i
        assert cycles(addr, B128_GROUPS, 4, 64) == 4
        # the previous layout (rows 64 dwords apart) is 8-way in every group
        old = {lane: a - a1_row((((lane & 31) & 3) + 4 * ((lane & 31) >> 3))) +
               64 * (((lane & 31) & 3) + 4 * ((lane & 31) >> 3)) for lane, a in addr.items()}
        assert cycles(old, B128_GROUPS, 4, 64) == 32


def test_a1_park_rows_disjoint_and_b32_conflict_free():
    rows = sorted(a1_row(g) for g in range(16))
    assert all(b - a >= 64 for a, b in zip(rows, rows[1:]))
    assert rows[-1] + 64 == 15 * 68 + 64          # MLP2_A1W
    assert all(r % 4 == 0 for r in rows)          # 16-B aligned rows
    for g in range(16):                           # the park stores / dz_of reads: row g, all lanes
        addr = {lane: a1_row(g) + lane for lane in range(64)}
        assert cycles(addr, B32_GROUPS, 1, 32) == 2


@pytest.mark.parametrize('s', range(6))
def test_forward_image_reads_conflict_free(s):
    # fp = xf + l32 MLP2_FS + 48 half (halves), + 8 s: one b128 per K-step and fragment
    addr = {lane: ((lane & 31) * MLP2_FS + 48 * (lane >> 5) + 8 * s) // 2 for lane in range(64)}
    assert cycles(addr, B128_GROUPS, 4, 64) == 4


@pytest.mark.parametrize('kb,step', [(kb, st) for kb in range(3) for st in range(2)])
def test_transposed_image_reads_conflict_free(kb, step):
    # th = xt + l32 MLP2_TS + 8 half (halves), + 16 step + kb 32 MLP2_TS
    addr = {lane: ((lane & 31) * MLP2_TS + 8 * (lane >> 5) + 16 * step + kb * 32 * MLP2_TS) // 2
            for lane in range(64)}
    assert cycles(addr, B128_GROUPS, 4, 64) == 4


MLP2_XS = 100   # floats per row of the raw X tile (the 4-wave kernel and mlp2r at C_in = 96)


@pytest.mark.parametrize('kh,s', [(kh, s) for kh in (44, 48) for s in range(12)])
def test_four_wave_forward_reads_conflict_free(kh, s):
    # ap = xs + l32 MLP2_XS + half KH, + 4 s (two b128 per K-step: 8 s and 8 s + 4)
    addr = {lane: (lane & 31) * MLP2_XS + (lane >> 5) * kh + 4 * s for lane in range(64)}
    assert cycles(addr, B128_GROUPS, 4, 64) == 4


@pytest.mark.parametrize('xs', [MLP2_XS, 88])
def test_transposed_b32_reads_conflict_free(xs):
    # dW1 K-step s, block kb: lane reads X[4 half + 16 s + 8 (j >> 2) + (j & 3)][32 kb + l32]
    for kb in range(3):
        for s in range(2):
            for j in range(8):
                addr = {lane: (4 * (lane >> 5) + 16 * s + 8 * (j >> 2) + (j & 3)) * xs + 32 * kb + (lane & 31)
                        for lane in range(64)}
                assert cycles(addr, B32_GROUPS, 1, 32) == 2


def test_rows_kernel_packed_rows_cost_two_way_forward_reads():
    # mlp2r at C_in = 88: rows packed at stride 88 (11 full LDS-DMA pieces per tile instead of 32
    # one-row pieces); the forward's b128 reads become 2-way (8 cycles instead of 4, 12 reads per
    # tile: +48 LDS cycles against ~2.5 k cycles of DMA issue saved, measured 0.875 -> 0.797 ms)
    for s in range(12):
        addr = {lane: (lane & 31) * 88 + (lane >> 5) * 44 + 4 * s for lane in range(64)}
        assert cycles(addr, B128_GROUPS, 4, 64) == 8


def test_rows_kernel_broadcast_reads():
    # the head's W2 rows (w2t + (32 u + 16 h + i) 4) and the backward's dZ2 rows (dz2 + r(g) 4):
    # one address per half-wave, one LDS cycle per lane group
    for u in range(2):
        for i in range(16):
            addr = {lane: (32 * u + 16 * (lane >> 5) + i) * 4 for lane in range(64)}
            assert cycles(addr, B128_GROUPS, 4, 64) == 4
    for g in range(16):
        addr = {lane: ((g & 3) + 8 * (g >> 2) + 4 * (lane >> 5)) * 4 for lane in range(64)}
        assert cycles(addr, B128_GROUPS, 4, 64) == 4


def test_unit_split_head_reads():
    # mlp2_kernel's head: thread it sums part[(w T + r) 4 + j], r = it / 3, j = it % 3 (b32);
    # rows 8.. of the first 32 lanes wrap onto banks 0.. (2-way: 4 cycles on the first wave), the
    # per-thread loss accumulators hacc[tid HS + k] (HS = 3 on the 4-wave kernel) are conflict-free
    first = {lane: 4 * (lane // 3) + lane % 3 for lane in range(64)}
    assert cycles(first, B32_GROUPS, 1, 32) == 4
    second = {lane: 4 * ((64 + lane) // 3) + (64 + lane) % 3 for lane in range(32)}
    assert cycles(second, [list(range(32))], 1, 32) == 2
    assert cycles({lane: 3 * lane for lane in range(64)}, B32_GROUPS, 1, 32) == 2

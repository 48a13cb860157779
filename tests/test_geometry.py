"""Fused-sweep geometry (csrc/engine/geometry.cpp) on the CPU: padded widths and persistent grids.

The reference's kernels run at any voxel count (grid ceil(V/256), reference sart_kernels.cu:269-283;
cublasSgemv takes any V, sartsolver_cuda.cpp:248-249). The fused sweep's fast variant 6 must therefore
cover every width a real voxel grid produces, not only powers of two.
"""
import pytest

from mpi_cuda_sartsolver_amd.models import rtm
from mpi_cuda_sartsolver_amd.ops import hip

CUS = 256  # MI355X: 8 XCDs x 32 CUs


def _check_v6(ld, g):
    assert g is not None and g.variant == 6 and g.kw in (5, 6, 7, 8, 9)
    assert g.kw not in (5, 9) or g.T == 1  # 5- and 9-KiB slabs: T = 1
    slab = 1024 * g.kw // g.T
    assert g.T in (1, 2, 4) and ld % slab == 0 and ld // slab == g.J
    assert g.J * g.T <= 256 and g.grid == g.I * g.J <= CUS
    if g.xl:  # XCD-local row groups: as many per XCD as fit
        assert g.J <= CUS // 8 and g.I % 8 == 0 and g.I // 8 == (CUS // 8) // g.J
    else:  # chip-wide row groups (T = 1): as many as fit the chip
        assert g.T == 1 and g.J <= CUS and g.I == CUS // g.J


@pytest.mark.parametrize("nvox", [20480, 30000, 60000, 61440, 65536, 70000, 100000, 131072, 150000, 200000,
                                  229376, 262144, 300000, 524288, 1000000, 1048576])
def test_every_width_gets_variant6(nvox):
    ld = rtm.choose_ld(nvox)
    assert nvox <= ld <= 1.10 * nvox
    _check_v6(ld, rtm.fused_geometry(ld, CUS, 6))
    # bf16 shards: the wide tiles (16 bytes of 8 bf16 per lane, T = 4 / 2, slab 2048 kw / T, kw 5 ... 8) at every
    # width, in XCD-local row groups (J <= 32) or chip-wide ones (J <= 128, I = CUs // J)
    ldb = rtm.choose_ld(nvox, storage="bf16")
    gw = hip().fused_geometry_bf16_wide(ldb, CUS)
    assert nvox <= ldb <= 1.10 * nvox and gw.valid() and gw.cpl == 8 and gw.T in (2, 4) and 5 <= gw.kw <= 8
    assert ldb == gw.J * 2048 * gw.kw // gw.T
    if gw.xl:
        assert gw.J <= CUS // 8 and gw.I == 8 * ((CUS // 8) // gw.J)
    else:
        assert gw.J <= 128 and gw.I == CUS // gw.J


def test_width_sweep_variant6_and_waste():
    """Every width from 20k to 1M voxels gets variant 6 with at most 10 % padding (XCD-local row groups up to 32
    slabs, chip-wide ones beyond: measured 1.2-1.55x slower per CU where both exist)."""
    used = []
    for nvox in list(range(20480, 262145, 997)) + list(range(262144, 1048577, 8191)):
        ld = rtm.choose_ld(nvox)
        assert ld % 64 == 0 and nvox <= ld <= 1.10 * nvox, nvox
        g = rtm.fused_geometry(ld, CUS, 6)
        _check_v6(ld, g)
        used.append(g.grid / CUS)
    assert min(used) >= 0.65 and sum(used) / len(used) >= 0.9, (min(used), sum(used) / len(used))


@pytest.mark.parametrize("ld,T,kw,J,I,xl", [(65536, 4, 8, 32, 8, True), (131072, 1, 8, 16, 16, True),
                                            (262144, 1, 8, 32, 8, True), (61440, 4, 8, 30, 8, True),
                                            (16384, 4, 8, 8, 32, True), (106496, 1, 8, 13, 16, True),
                                            (100352, 1, 7, 14, 16, True), (200704, 1, 7, 28, 8, True),
                                            (71680, 1, 7, 10, 24, True), (153600, 1, 6, 25, 10, False), (163840, 1, 8, 20, 12, False),
                                            (150528, 1, 7, 21, 12, False),
                                            (229376, 1, 7, 32, 8, True), (524288, 1, 8, 64, 4, False),
                                            (1048576, 1, 8, 128, 2, False), (301056, 1, 7, 42, 6, False),
                                            (147456, 1, 9, 16, 16, True), (73728, 1, 9, 8, 32, True),
                                            (294912, 1, 9, 32, 8, True), (368640, 1, 9, 40, 6, False)])
def test_production_geometries(ld, T, kw, J, I, xl):
    g = rtm.fused_geometry(ld, CUS, 6)
    assert (g.T, g.kw, g.J, g.I, g.xl) == (T, kw, J, I, xl)


def test_xl_override(monkeypatch):
    """SART_FUSED_XL=1 keeps XCD-local groups only (wider rows then fall back to variant 3), 0 chip-wide only."""
    monkeypatch.setenv("SART_FUSED_XL", "1")
    g = rtm.fused_geometry(200704, CUS, 6)
    assert g.xl and (g.J, g.I) == (28, 8)
    monkeypatch.setenv("SART_FUSED_XL", "0")
    g = rtm.fused_geometry(200704, CUS, 6)
    assert not g.xl and (g.J, g.I) == (28, 9)
    monkeypatch.setenv("SART_FUSED_XL", "1")
    assert rtm.fused_geometry(524288, CUS, 6).variant == 3
    monkeypatch.setenv("SART_FUSED_XL", "0")
    g = rtm.fused_geometry(65536, CUS, 6)
    assert not g.xl and (g.T, g.J, g.I) == (1, 8, 32)


def test_lowest_cost_rows_per_tile():
    # 70000 columns with 8-KiB slabs: T = 2 needs J = 18 (one group per XCD, 18 of 32 CUs); T = 1 gives J = 9
    # and three groups per XCD (27 CUs), a lower time per row. 7-KiB slabs: J = 10, three groups (30 CUs).
    g = rtm.fused_geometry(73728, CUS, 6, narrow_slabs=False, chip_wide=False)  # bf16 narrow tiles (kw 8)
    assert (g.T, g.J, g.I) == (1, 9, 24)
    ld = rtm.choose_ld(70000)
    g = rtm.fused_geometry(ld, CUS, 6)
    # 7-KiB slabs at J = 10 (30 CUs per XCD) against 9-KiB slabs at ld 73728 (J = 8, all 32 CUs, 5 % padding):
    # measured 348 vs 344 it/s, kept 7 KiB (profiles/ab_r3_kw9.jsonl); 73728 itself takes the 9-KiB slabs
    assert (ld, g.T, g.kw, g.J, g.I) == (71680, 1, 7, 10, 24)
    assert rtm.fused_geometry(73728, CUS, 6).kw == 9


def test_t2_penalty_prefers_t1():
    # 100000 columns: T = 2 at ld 102400 (J = 25, one group per XCD) against T = 1 at ld 106496 (J = 13, two
    # groups per XCD): equal slab / G, T = 2 measured slower per byte (profiles/probe_r2_t1_sched5.jsonl)
    assert rtm.fused_geometry(106496, CUS, 6, narrow_slabs=False, chip_wide=False).T == 1
    g2 = rtm.fused_geometry(131072, CUS, 6, 2)
    assert (g2.T, g2.J, g2.I) == (2, 32, 8)  # still available when forced


def test_forced_rows_per_tile_and_fallback():
    g = rtm.fused_geometry(65536, CUS, 6, 1)
    assert (g.T, g.J, g.I) == (1, 8, 32)
    # wider than 32 slabs of 8192: chip-wide variant 6; without chip-wide groups variant 3 (K = 8)
    g6 = rtm.fused_geometry(1 << 20, CUS, 6)
    assert g6.variant == 6 and not g6.xl and (g6.J, g6.I) == (128, 2)
    g3 = rtm.fused_geometry(1 << 20, CUS, 6, chip_wide=False)
    assert g3.variant == 3 and g3.K == 8 and g3.J == 128
    assert rtm.fused_geometry(65536, CUS, 3).variant == 3
    # not a multiple of 1024: no fused path
    assert rtm.fused_geometry(64 * 1001, CUS, 6) is None


@pytest.mark.parametrize("ld,T,J,I,xl", [(65536, 4, 16, 16, True), (131072, 4, 32, 8, True), (262144, 4, 64, 4, False),
                                         (204800, 4, 50, 5, False), (4096, 4, 1, 256, True), (524288, 2, 64, 4, False)])
def test_bf16_wide_geometry(ld, T, J, I, xl, monkeypatch):
    """Wide bf16 tiles: T = 4 (slab 4096) where it fits an XCD, else T = 2 (slab 8192, schedule 7), or chip-wide row
    groups where those cost less (204800: J = 50 at T = 4 on 250 CUs instead of 25 slabs at T = 2 on 200). With
    XCD-local groups only (SART_BF16_XL=1) rows of more than 32 slabs have no fused geometry."""
    g = hip().fused_geometry_bf16_wide(ld, CUS)
    assert g.valid() and (g.cpl, g.T, g.J, g.I, g.xl) == (8, T, J, I, xl)
    monkeypatch.setenv("SART_BF16_XL", "1")
    assert not hip().fused_geometry_bf16_wide(524288, CUS).valid()
    assert hip().fused_geometry_bf16_wide(204800, CUS).T == 2
    g2 = hip().fused_geometry_bf16_wide(262144, CUS)
    assert (g2.T, g2.J, g2.I, g2.xl) == (2, 32, 8, True)


def test_t1_fold_period(monkeypatch):
    """T = 1 sweeps fold their back-projection chains every ~sqrt(rows per group) tiles (two-level sums: the
    single-chain version measured 26x the two-pass error at 524288 rows); T >= 2 and variant 3 never fold."""
    k = hip()
    monkeypatch.delenv("SART_FUSED_FOLD", raising=False)
    g1 = k.fused_geometry(262144, CUS, 6, 1)
    assert g1.T == 1
    for rows in (4096, 65536, 524288):
        f = k.fused_fold_tiles(g1, rows)
        per_group = -(-rows // g1.I)
        assert 16 <= f and (f - 1) ** 2 < max(per_group, 256) <= f * f + 2 * f
    assert k.fused_fold_tiles(k.fused_geometry(65536, CUS, 6, 4), 65536) == 0
    assert k.fused_fold_tiles(k.fused_geometry(65536, CUS, 3, 0), 65536) == 0
    monkeypatch.setenv("SART_FUSED_FOLD", "0")
    assert k.fused_fold_tiles(g1, 65536) == 0


def test_segment_plan(monkeypatch):
    """T >= 2 split schedules run row groups longer than 2240 tiles (wide bf16 tiles: 700) in segments, one partial
    block per segment and tile row; shorter groups (the 64k x 64k fp32 headline: 2048 tiles per group) keep one
    chain."""
    k = hip()
    monkeypatch.delenv("SART_FUSED_SEG", raising=False)
    g4 = k.fused_geometry(65536, CUS, 6, 4)
    assert k.fused_chain_plan(g4, 65536, True) == (0, g4.I)
    monkeypatch.setenv("SART_BF16_XL", "1")
    gw = k.fused_geometry_bf16_wide(262144, CUS)  # XCD-local T = 2, I = 8: 32768 tiles per group at 512k rows
    assert k.fused_chain_plan(gw, 524288, True) == (700, 8 * 2 * 47)
    assert k.fused_chain_plan(gw, 524288, False) == (0, 8)  # non-split schedules keep one chain
    monkeypatch.setenv("SART_FUSED_SEG", "1000")  # rounded up to a multiple of 140
    assert k.fused_chain_plan(gw, 524288, True) == (1120, 8 * 2 * 30)
    monkeypatch.setenv("SART_FUSED_SEG", "0")
    assert k.fused_chain_plan(gw, 524288, True) == (0, 8)
    assert k.fused_split_schedule(2, True) and k.fused_split_schedule(4, False)


def test_python_is_native():
    k = hip()
    for n in (1, 63, 64, 1000, 1024, 5000, 60000, 65536, 100000, 250000, 1 << 20):
        assert rtm.choose_ld(n) == k.choose_ld(n)


def test_kw9_opt_out(monkeypatch):
    """SART_FUSED_KW9=0 removes the 9-KiB slabs: 147456 voxels then run 6-KiB slabs on 24 CUs per XCD (XCD-local
    groups, SART_FUSED_XL=1)."""
    monkeypatch.setenv("SART_FUSED_KW9", "0")
    monkeypatch.setenv("SART_FUSED_XL", "1")
    g = rtm.fused_geometry(147456, CUS, 6)
    assert (g.kw, g.J, g.I) == (6, 24, 8)
    assert rtm.fused_geometry(73728, CUS, 6).kw == 8


def test_kw5_opt_out(monkeypatch):
    """With XCD-local groups only (SART_FUSED_XL=1), 5-KiB slabs fill the XCDs at 148480 ... 163840 voxels (150000:
    J = 30 instead of 6-KiB slabs at J = 25); SART_FUSED_KW5=0 removes them. (By default 150000 voxels take chip-wide
    groups of 7-KiB slabs on 252 CUs: 337 against 308 it/s, profiles/cw_r4_xl_vs_cw.txt.)"""
    assert (rtm.choose_ld(150000), rtm.fused_geometry(150528, CUS, 6).kw) == (150528, 7)
    monkeypatch.setenv("SART_FUSED_XL", "1")
    assert rtm.fused_geometry(153600, CUS, 6).kw == 5
    monkeypatch.setenv("SART_FUSED_KW5", "0")
    g = rtm.fused_geometry(153600, CUS, 6)
    assert (g.kw, g.J, g.I) == (6, 25, 8)


@pytest.mark.parametrize("nvox,ld,T,J,kw", [(65536, 65536, 4, 16, 8), (100000, 100352, 4, 28, 7),
                                           (150000, 150528, 4, 42, 7), (200000, 200704, 4, 49, 8),
                                           (262144, 262144, 4, 64, 8), (70000, 73728, 4, 18, 8)])
def test_bf16_wide_kw(nvox, ld, T, J, kw, monkeypatch):
    """Wide bf16 tiles take 7 / 6 / 5 lane-vectors per lane where 8-KiB-equivalent slabs leave CUs idle (150000
    voxels: chip-wide J = 42 at T = 4); SART_BF16_KW=8 keeps the 8-wide slabs."""
    ldb = rtm.choose_ld(nvox, storage="bf16")
    g = hip().fused_geometry_bf16_wide(ldb, CUS)
    assert (ldb, g.T, g.J, g.kw) == (ld, T, J, kw)
    monkeypatch.setenv("SART_BF16_KW", "8")
    g8 = hip().fused_geometry_bf16_wide(rtm.choose_ld(nvox, storage="bf16"), CUS)
    assert g8.kw == 8


def test_granule_rows_padded_to_lines():
    """Chip-wide row groups pad every tile's granule row to whole 128-byte lines (16 granules), so no line holds the
    granules of two tiles (round 4: 303104 ... 557056 voxels 4.3-5.8 -> 6.0-6.7 TB/s); the buffer covers it."""
    k = hip()
    assert k.fused_granules(4096, 33, False) == 4096 * 48
    assert k.fused_granules(4096, 64, False) == 4096 * 64
    assert k.fused_granules(4096, 30, True) >= 4096 * 30


def test_chip_wide_group_map_is_balanced():
    """The XCD-balanced map of chip-wide workgroups (fused_sweep.hip: p = workgroups of lower XCDs + b / 8, group
    p % I): a bijection for every grid, and with I even every group gets J / 8 (+-1) workgroups on every XCD."""
    for I, J in [(4, 57), (6, 40), (4, 64), (5, 49), (2, 128), (12, 21)]:
        grid = I * J
        seen, per = set(), {}
        for b in range(grid):
            x = b & 7
            p = x * (grid >> 3) + min(x, grid & 7) + (b >> 3)
            seen.add(p)
            per.setdefault((p % I, x), 0)
            per[(p % I, x)] += 1
        assert seen == set(range(grid))
        counts = [per.get((g, x), 0) for g in range(I) for x in range(8)]
        assert max(counts) - min(counts) <= 2 and min(counts) >= J // 8 - 1

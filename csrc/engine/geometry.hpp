// Shard layout and persistent-grid geometry of the fused sweep (single source of truth for the C++
// engine, the driver and the Python package).
#pragma once

#include <cstdint>

namespace sart {

struct FusedGeometry {
    int K = 0;        // variant 3: float4 per lane per row slab / 256 (slab 1024 * K); variant 6: rows per tile
    int J = 0;        // workgroups per row (column slabs)
    int I = 0;        // row groups
    int grid = 0;     // I * J persistent workgroups
    int variant = -1; // 6 (XCD-local row groups), 3 (generic fallback), -1: no fused path for this width
    int T = 0;        // rows per tile
    int cpl = 4;      // variant 6: columns per lane per k-slot (8: wide bf16 tiles, slab 16384 / T)
    int kw = 8;       // variant 6 fp32: lane-vectors per lane per row (slab 1024 kw / T; 7 / 6 fill more CUs)
    // variant 6: true = XCD-local row groups (per-XCD tickets, granules stay in the XCD's L2; J <= CUs per XCD,
    // I a multiple of 8); false = row groups by block index with granules written through to memory (any
    // J <= CUs, I = CUs / J): rows wider than an XCD's slabs, and widths whose J wastes CUs of every XCD
    bool xl = true;
    bool valid() const { return variant >= 0; }
};

// Padded row length of a dense shard: the variant 6 width (J slabs of 1024 kw / T columns: J <= 32 XCD-local,
// or J <= 256 chip-wide at T = 1) with the lowest estimated time per row when that wastes at most max_waste of
// the row, else a multiple of 8192 (variant 3), else the next multiple of 64 floats (256 B rows).
// narrow_slabs: also consider fp32 slabs of 7 / 6 KiB columns (kw 7 / 6); bf16 shards keep kw = 8.
int64_t choose_ld(int64_t nvoxel, double max_waste = 0.10, bool narrow_slabs = true);

// Geometry for `variant` (6 default, or 3), falling back to variant 3 when variant 6 cannot split the
// width. rows_per_tile = 0: SART_FUSED_T or the lowest-cost T. chip_wide: also consider chip-wide row groups
// (fp32 T = 1; the bf16 kernels run XCD-local groups only).
FusedGeometry fused_geometry(int64_t ld, int num_cus, int variant, int rows_per_tile, bool narrow_slabs = true,
                             bool chip_wide = true);
// Variant 6 geometry of the wide bf16 tiles (16-byte loads of 8 bf16 per lane: T = 4 with slab 4096 columns, or
// T = 2 with slab 8192); invalid when the width does not split into J <= 32 such slabs.
FusedGeometry fused_geometry_bf16_wide(int64_t ld, int num_cus);
// Fold period of the T = 1 sweep's two-level back-projection sums (variant 6): ~sqrt(tiles per row group), so
// no fp32 chain exceeds ~2 sqrt(P / I) terms (SART_FUSED_FOLD overrides; 0 = one chain per group). 0 for T >= 2.
int64_t fused_fold_tiles(const FusedGeometry& g, int64_t nrows_pad);
// Back-projection chain plan of the fused sweep (launch_fused_sweep's chain_tiles): T = 1 folds (above);
// T >= 2 with a split schedule runs segments of 2240 tiles (SART_FUSED_SEG, rounded up to a multiple of 140)
// when a row group has more tiles than that. blocks = partial-sum rows (of ld floats) the sweep writes.
struct ChainPlan {
    int64_t chain_tiles = 0;
    int64_t blocks = 0;
};
ChainPlan fused_chain_plan(const FusedGeometry& g, int64_t nrows_pad, bool split_schedule);

}  // namespace sart

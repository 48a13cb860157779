#include "geometry.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace sart {

namespace {

// Variant 6 geometry for a padded width `ld` at T rows per tile and kw lane-vectors per lane: J = ld / slab
// workgroups per row (slab = 1024 kw / T columns: the four compute waves cover T rows x 4 / T sub-slabs of
// 256 kw columns).
//   XCD-local (xl): G = per_xcd / J row groups per XCD, I = 8 G (the XCD's remaining per_xcd - G J CUs idle).
//   chip-wide (!xl, T = 1 only): I = num_cus / J row groups of any J <= num_cus, granules through memory.
// cost = slab / I is the time per matrix row relative to the other candidates (each CU streams slab columns of
// P / I rows), times the measured per-CU rate penalties.
struct V6Candidate {
    int T = 0, J = 0, I = 0, kw = 8;
    bool xl = true;
    double cost = 0.0;
};

// kw < 8 streams fewer bytes per pipeline step for the same per-step exchange work: per CU, kw 7 measured
// 26.4 GB/s and kw 6 23.2 GB/s against 26.6 at kw 8 (bench --nvox 200000 / 150000 / 65536,
// profiles/bench_r2_widths_kw.jsonl)
// kw 9 (T = 1 only, 3 register tiles in flight): 4-10 % below kw 8's per-CU rate (70000 voxels: 344 it/s at kw 9,
// J = 8 on 256 CUs, against 348 at kw 7, J = 10 on 240 CUs; profiles/ab_r3_kw9.jsonl)
constexpr double narrow_slab_penalty(int kw) {
    return kw == 8 ? 1.0 : (kw == 9 ? 1.06 : (kw == 7 ? 1.02 : (kw == 6 ? 1.15 : 1.3)));
}

// kw candidates: 8, 7, 6, 5, 9 (narrow_slabs; 5 / 9 unless SART_FUSED_KW5=0 / SART_FUSED_KW9=0); forced:
// SART_FUSED_KW=k keeps only k for the geometry of a given width (A/B runs; the width itself is chosen without it)
bool kw_allowed(int kw, bool narrow_slabs, bool forced = true) {
    if (const char* e = std::getenv("SART_FUSED_KW"); forced && e && *e) return kw == std::atoi(e) && (kw == 8 || narrow_slabs);
    if (kw == 8) return true;
    if (!narrow_slabs) return false;
    if (kw == 5) {  // (on by default since the 16-byte flag reads: +3.6-4 % at 150000 ... 163840, profiles/ab_r3_kw5_flag4.jsonl)
        const char* e = std::getenv("SART_FUSED_KW5");
        return !(e && *e && std::atoi(e) == 0);
    }
    if (kw == 9) {
        const char* e = std::getenv("SART_FUSED_KW9");
        return !(e && *e && std::atoi(e) == 0);
    }
    return true;
}

// Chip-wide row groups hand granules off through memory instead of the XCD's L2. Until round 4 they streamed
// 1.22-1.55x slower per CU than XCD-local groups: a tile's J 8-byte granules shared 128-byte lines with the next
// tile's, so the J writers of tile u + 1 (on other XCDs) stored into lines the gatherers of tile u were still
// re-polling through memory. With every tile's granule row padded to whole lines (fused_sweep.hip, fused_granules)
// they stream at the XCD-local rate: 24.2-27.3 GB/s per CU at kw 6 ... 9 (kw 5: 21.0-21.4) at 301056 ... 344064
// voxels (profiles/cw_r4_kw_padded.txt), 5.9-6.3 TB/s at 303104 ... 557056 (profiles/cw_r4_granule_pad_ab.jsonl,
// unpadded 4.6-5.8). kChipWidePenalty is fitted where both kinds exist (profiles/cw_r4_xl_vs_cw.txt): chip-wide
// groups win at 150000 ... 172032 voxels (6.56-6.78 against 6.21-6.57 TB/s: wider slabs on more CUs than the kw 5 / 6
// XCD-local grids) and lose at 100000 and 180224 ... 245760 (-1 ... -6 %; profiles/width_r4_sweep_default_vs_xl_box1.jsonl:
// 180224 / 188416 by 1-2 % at 1.16), which 1.19 reproduces.
// SART_FUSED_XL=0 / 1 forces one kind where both exist.
constexpr double kChipWidePenalty = 1.19;

// Per-CU time of a chip-wide slab of kw lane-vectors relative to an XCD-local kw 8 slab (chip-wide groups run schedule
// 5 at kw 8 / 9 / 5 and schedule 8 at kw 6 / 7, fused_sweep.hip launch_rows). (The grid size showed no consistent
// effect once the granule rows were padded: kw 7 at 252 workgroups 24.6 GB/s per CU at 301056 voxels, 26.4 at 150528.)
double chip_wide_penalty(int kw) {
    // kw 7 (schedule 8) as kw 8 / 9: 150528 voxels at kw 7 (J = 21) 337 it/s against 310 at kw 9 (J = 17, ld 156672)
    const double per_kw = kw >= 7 ? 1.0 : (kw == 6 ? 1.08 : 1.26);
    return kChipWidePenalty * per_kw;
}

int xl_mode() {
    const char* e = std::getenv("SART_FUSED_XL");
    return (e && *e) ? std::atoi(e) : -1;  // -1 auto, 0 chip-wide only, 1 XCD-local only
}

V6Candidate v6_candidate(int64_t ld, int T, int kw, int num_cus, bool xl) {
    V6Candidate c;
    const int per_xcd = num_cus / 8;
    const int64_t slab = 1024 * (int64_t)kw / T;
    if (ld % slab != 0) return c;
    const int64_t J = ld / slab;
    if (J < 1 || J * T > 256 /* exchange gather registers */) return c;
    if (xl) {
        if (J > per_xcd) return c;
        c.I = 8 * (per_xcd / (int)J);
    } else {
        // chip-wide: T = 1 (schedule 5 / 8) at any kw; T = 2 / 4 (schedule 4, kw 6 ... 8) only with SART_FUSED_CW_T=2 / 4:
        // no faster than T = 1 where measured (100000 / 150000 / 393216 / 524288 voxels: -1 ... -20 %, 303104 equal;
        // profiles/cw_r4_multirow_t_ab.jsonl) and T = 2 at 303104 voxels missed the 1.25x error bound (1.58x)
        const char* e = std::getenv("SART_FUSED_CW_T");
        const int tmax = (e && *e) ? std::atoi(e) : 1;
        if (J > num_cus || T > tmax || (T != 1 && (kw < 6 || kw > 8))) return c;
        c.I = num_cus / (int)J;
    }
    c.T = T, c.J = (int)J, c.kw = kw, c.xl = xl;
    // T = 2 (schedule 4) measured 4-10 % slower per byte than T = 1 (schedule 5) at equal slab / G
    // (131072 / 106496 columns, profiles/probe_r2_t1_sched5.jsonl); T = 4 and T = 1 tie at 65536
    c.cost = (double)slab / c.I * (T == 2 ? 1.08 : 1.0) * (xl ? narrow_slab_penalty(kw) : chip_wide_penalty(kw));
    return c;
}

// The lower-cost row-group kind at (ld, T, kw) (I == 0: none), per SART_FUSED_XL and chip_wide.
V6Candidate best_kind(int64_t ld, int T, int kw, int num_cus, bool chip_wide) {
    V6Candidate best;
    const int xm = xl_mode();
    for (const bool xl : {true, false}) {
        if ((xm == 0 && xl) || (xm == 1 && !xl) || (!xl && !chip_wide)) continue;
        const V6Candidate c = v6_candidate(ld, T, kw, num_cus, xl);
        if (c.I > 0 && (best.I == 0 || c.cost < best.cost)) best = c;
    }
    return best;
}

// The lowest-cost candidate over (kw, T, kind) for width ld (I == 0: none). rows_per_tile > 0 fixes T.
V6Candidate best_v6(int64_t ld, int num_cus, int rows_per_tile, bool narrow_slabs, bool chip_wide) {
    V6Candidate best;
    for (const int kw : {8, 7, 6, 5, 9}) {
        if (!kw_allowed(kw, narrow_slabs)) continue;
        for (const int T : {4, 2, 1}) {
            if (T != 1 && (kw == 5 || kw == 9)) continue;
            if (rows_per_tile > 0 && T != rows_per_tile) continue;
            const V6Candidate c = best_kind(ld, T, kw, num_cus, chip_wide);
            if (c.I > 0 && (best.I == 0 || c.cost < best.cost)) best = c;
        }
    }
    return best;
}

// Wide bf16 tiles (16-byte loads of 8 bf16 per lane, x slab in LDS): T = 4 (schedule 4) or T = 2 (schedule 7), slab
// 2048 kw / T columns of kw = 8 (16384 / T) or, so that J fills more of an XCD's 32 CUs, kw = 7 / 6 / 5 (kw 9 does
// not fit the registers next to the wide tiles' two accumulator halves). XCD-local groups only. Cost as v6_candidate:
// slab / G times the narrow-slab penalty; T = 4 and kw 8 first on ties. SART_BF16_KW=k keeps only k (A/B runs).
// Wide bf16 tiles at T = 2 (schedule 7) stream ~12 % slower per CU than at T = 4 (200000 voxels, T = 2: 23.2 GB/s per CU;
// 150000 chip-wide at T = 4: 26.1; profiles/bf16_r4_widths_cw_vs_xl.jsonl).
double bf16_t2_penalty(int T) { return T == 2 ? 1.12 : 1.0; }

V6Candidate bf16_wide_candidate(int64_t ld, int T, int kw, int num_cus) {
    V6Candidate c;
    if (const char* e = std::getenv("SART_BF16_KW"); e && *e && std::atoi(e) != kw) return c;
    if (const char* e = std::getenv("SART_BF16_T"); e && *e && std::atoi(e) != T) return c;  // A/B runs
    const int per_xcd = num_cus / 8;
    const int64_t slab = 2048 * (int64_t)kw / T;
    if (num_cus % 8 != 0 || ld % slab != 0) return c;
    const int64_t J = ld / slab;
    if (J < 1 || J > per_xcd) return c;
    c.T = T, c.J = (int)J, c.kw = kw, c.xl = true;
    c.I = 8 * (per_xcd / (int)J);
    c.cost = (double)slab / (per_xcd / (int)J) * narrow_slab_penalty(kw) * bf16_t2_penalty(T);
    return c;
}

// Wide bf16 tiles in chip-wide row groups (I = num_cus / J groups of any J <= 128, granules through memory): for rows
// of more than an XCD's 32 slabs at T = 4, or where the XCD-local grid leaves CUs idle. Same cost scale as
// bf16_wide_candidate (slab / groups per XCD, I / 8 here) times chip_wide_penalty. SART_BF16_XL=0 / 1 keeps only
// chip-wide / XCD-local groups. Chip-wide and XCD-local sweeps of the same grid give the same iterate (131072 voxels,
// J = 32: self-check 1.195x the two-pass error both); 32768 x 150000 voxels run at 6.54 TB/s chip-wide (T = 4, J = 42,
// 700-tile segments) against 4.64 XCD-local in round 3.
V6Candidate bf16_wide_cw_candidate(int64_t ld, int T, int kw, int num_cus) {
    V6Candidate c;
    if (const char* e = std::getenv("SART_BF16_KW"); e && *e && std::atoi(e) != kw) return c;
    if (const char* e = std::getenv("SART_BF16_T"); e && *e && std::atoi(e) != T) return c;
    if (const char* e = std::getenv("SART_BF16_XL"); e && *e && std::atoi(e) == 1) return c;
    const int64_t slab = 2048 * (int64_t)kw / T;
    if (ld % slab != 0) return c;
    const int64_t J = ld / slab;
    if (J < 2 || J * T > 256 || J > num_cus) return c;  // the gatherer's J T granules per tile (kRowsGather)
    c.T = T, c.J = (int)J, c.kw = kw, c.xl = false;
    c.I = num_cus / (int)J;
    // priced like XCD-local wide tiles: chip-wide and XCD-local grids of the same J stream alike (131072 voxels: 781
    // against 778 it/s, profiles/bf16_r4_widths_cw_vs_xl.jsonl)
    c.cost = (double)slab / (c.I / 8.0) * narrow_slab_penalty(kw) * bf16_t2_penalty(T);
    return c;
}

bool bf16_xl_allowed() {
    const char* e = std::getenv("SART_BF16_XL");
    return !(e && *e && std::atoi(e) == 0);
}

}  // namespace

int64_t choose_ld(int64_t nvoxel, double max_waste, bool narrow_slabs) {
    if (!narrow_slabs && nvoxel >= 1024) {
        // bf16 storage: the widths of the wide tiles first (the engine runs them wherever they are valid)
        int64_t best_ld = 0;
        double best_cost = 0.0;
        for (const int kw : {8, 7, 6, 5})
            for (const int T : {4, 2}) {
                const int64_t slab = 2048 * (int64_t)kw / T;
                const int64_t ld = (nvoxel + slab - 1) / slab * slab;
                if ((double)(ld - nvoxel) > max_waste * (double)nvoxel) continue;
                for (const V6Candidate& c : {bf16_xl_allowed() ? bf16_wide_candidate(ld, T, kw, 256) : V6Candidate{},
                                             bf16_wide_cw_candidate(ld, T, kw, 256)}) {
                    if (c.I == 0) continue;
                    if (best_ld == 0 || c.cost < best_cost || (c.cost == best_cost && ld < best_ld)) {
                        best_ld = ld;
                        best_cost = c.cost;
                    }
                }
            }
        if (best_ld) return best_ld;
    }
    // Widths the fused sweep (variant 6) can split into whole slabs: at each (T, kw) the smallest multiple of the
    // slab covering nvoxel. Take the one with the lowest time per row (ties: less padding, then the larger T and
    // kw, measured fastest at equal cost), if it pads by at most max_waste.
    if (nvoxel >= 1024) {
        constexpr int kCus = 256;  // MI355X: 256 CUs in 8 XCDs
        int64_t best_ld = 0;
        double best_cost = 0.0;
        for (const int kw : {8, 7, 6, 5, 9}) {
            if (!kw_allowed(kw, narrow_slabs, false)) continue;
            for (const int T : {4, 2, 1}) {
                if (T != 1 && (kw == 5 || kw == 9)) continue;
                const int64_t slab = 1024 * (int64_t)kw / T;
                const int64_t ld = (nvoxel + slab - 1) / slab * slab;
                if ((double)(ld - nvoxel) > max_waste * (double)nvoxel) continue;
                const V6Candidate c = best_kind(ld, T, kw, kCus, narrow_slabs);  // bf16 (!narrow): XCD-local only
                if (c.I == 0) continue;
                if (best_ld == 0 || c.cost < best_cost || (c.cost == best_cost && ld < best_ld)) {
                    best_ld = ld;
                    best_cost = c.cost;
                }
            }
        }
        if (best_ld) return best_ld;
        // wider than 256 slabs of 8192: a multiple of 8192 keeps the variant 3 fallback (K = 8) available
        const int64_t ld = (nvoxel + 8191) / 8192 * 8192;
        if ((double)(ld - nvoxel) <= max_waste * (double)nvoxel) return ld;
    }
    const int64_t n = std::max<int64_t>(nvoxel, 64);
    return (n + 63) / 64 * 64;
}

FusedGeometry fused_geometry(int64_t ld, int num_cus, int variant, int rows_per_tile, bool narrow_slabs,
                             bool chip_wide) {
    FusedGeometry g;
    if (rows_per_tile <= 0) {
        const char* e = std::getenv("SART_FUSED_T");
        rows_per_tile = (e && *e) ? std::atoi(e) : 0;
    }
    if (variant == 6 && num_cus % 8 == 0) {
        // Rows per tile, slab and row-group kind: the requested T, else the candidate with the lowest time per row
        // (ties: the larger T and kw, XCD-local; T = 4 at ld = 64k, 2 at 128k, 1 at 256k measured 6.5-6.9 TB/s,
        // against 4.0-4.7 TB/s for variant 3, profiles/probe_r1_fused_T.jsonl). Rows wider than an XCD's slabs use
        // chip-wide row groups of I = num_cus / J (kChipWidePenalty).
        const V6Candidate best = best_v6(ld, num_cus, rows_per_tile, narrow_slabs, chip_wide);
        if (best.I > 0) {
            g.K = best.T, g.J = best.J, g.I = best.I, g.grid = g.I * g.J, g.variant = 6, g.T = best.T;
            g.kw = best.kw;
            g.xl = best.xl;
            return g;
        }
    }
    // Variant 3 (generic fallback): slabs of 1024 * K columns, K the smallest power of two giving <= 32
    // slabs (any count at K = 8), T = 8 / K rows per tile, num_cus / J row groups.
    for (int K = 1; K <= 8; K *= 2) {
        const int64_t wc = 1024 * (int64_t)K;
        if (ld % wc) continue;
        const int64_t J = ld / wc;
        if (J <= 32 || K == 8) {
            const int T = 8 / K;
            if (J > num_cus || J * T > 512) return g;
            g.K = K, g.J = (int)J, g.I = std::max(1, num_cus / (int)J), g.grid = g.I * g.J, g.variant = 3, g.T = T;
            return g;
        }
    }
    return g;
}

FusedGeometry fused_geometry_bf16_wide(int64_t ld, int num_cus) {
    FusedGeometry g;
    // T = 4 (schedule 4) or T = 2 (schedule 7: 3-slot ring, lag 4) at kw 8 ... 5 (bf16_wide_candidate); the lower
    // cost slab / G wins, T = 4 and kw 8 on ties (the deeper lag measured faster at 64k x 64k)
    double best_cost = 0.0;
    for (const int kw : {8, 7, 6, 5})
        for (const int T : {4, 2})
            for (const V6Candidate& c : {(bf16_xl_allowed() && num_cus % 8 == 0) ? bf16_wide_candidate(ld, T, kw, num_cus)
                                                                             : V6Candidate{},
                                         bf16_wide_cw_candidate(ld, T, kw, num_cus)}) {
                if (c.I == 0 || (g.valid() && c.cost >= best_cost)) continue;
                best_cost = c.cost;
                g.K = T, g.T = T, g.cpl = 8, g.J = c.J, g.I = c.I, g.grid = g.I * g.J, g.variant = 6, g.kw = kw;
                g.xl = c.xl;
            }
    return g;
}

int64_t fused_fold_tiles(const FusedGeometry& g, int64_t nrows_pad) {
    if (g.variant != 6 || g.K != 1 || g.I <= 0) return 0;
    if (const char* e = std::getenv("SART_FUSED_FOLD")) return std::max<int64_t>(0, std::atoll(e));
    const int64_t per_group = (nrows_pad + g.I - 1) / g.I;  // tiles (= rows at T = 1) of the longest group
    return std::max<int64_t>(16, (int64_t)std::ceil(std::sqrt((double)per_group)));
}

ChainPlan fused_chain_plan(const FusedGeometry& g, int64_t nrows_pad, bool split_schedule) {
    ChainPlan p;
    p.blocks = g.I;
    if (g.variant != 6 || g.I <= 0) return p;
    if (g.K == 1) {
        p.chain_tiles = fused_fold_tiles(g, nrows_pad);
        return p;
    }
    if (!split_schedule) return p;
    // fp32: 2240 tiles (> the 2048 tiles per group of the 64k x 64k headline: one chain there). Wide bf16 tiles: 700
    // (32768 x 150000 voxels, chip-wide T = 4, 1365 tiles per group: one chain measured 1.40x the two-pass error in the
    // bench self-check, segments of 700 / 280 tiles 1.16x / 1.24x, and the XCD-local T = 2 grid in one chain 1.59x)
    int64_t seg = g.cpl == 8 ? 700 : 2240;
    if (const char* e = std::getenv("SART_FUSED_SEG")) seg = std::max<int64_t>(0, std::atoll(e));
    if (seg <= 0) return p;
    seg = (seg + 139) / 140 * 140;
    const int64_t per_group = (nrows_pad / g.K + g.I - 1) / g.I;  // tiles of the longest row group
    if (per_group <= seg) return p;
    p.chain_tiles = seg;
    p.blocks = (int64_t)g.I * g.K * ((per_group + seg - 1) / seg);
    return p;
}

}  // namespace sart

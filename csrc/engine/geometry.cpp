#include "geometry.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace sart {

namespace {

// Variant 6 geometry for a padded width `ld` at T rows per tile and kw lane-vectors per lane: J = ld / slab
// workgroups per row (slab = 1024 kw / T columns: the four compute waves cover T rows x 4 / T sub-slabs of
// 256 kw columns), G = per_xcd / J row groups per XCD (the XCD's remaining per_xcd - G * J CUs stay idle).
// cost = slab / G is the time per matrix row relative to the other candidates (each CU streams slab columns
// of P / (8 G) rows).
struct V6Candidate {
    int T = 0, J = 0, G = 0, kw = 8;
    double cost = 0.0;
};

// kw < 8 streams fewer bytes per pipeline step for the same per-step exchange work: per CU, kw 7 measured
// 26.4 GB/s and kw 6 23.2 GB/s against 26.6 at kw 8 (bench --nvox 200000 / 150000 / 65536,
// profiles/bench_r2_widths_kw.jsonl)
constexpr double narrow_slab_penalty(int kw) { return kw == 8 ? 1.0 : (kw == 7 ? 1.02 : 1.15); }

V6Candidate v6_candidate(int64_t ld, int T, int kw, int per_xcd) {
    V6Candidate c;
    const int64_t slab = 1024 * (int64_t)kw / T;
    if (ld % slab != 0) return c;
    const int64_t J = ld / slab;
    if (J < 1 || J > per_xcd || J * T > 256 /* exchange gather registers */) return c;
    c.T = T, c.J = (int)J, c.G = per_xcd / (int)J, c.kw = kw;
    // T = 2 (schedule 4) measured 4-10 % slower per byte than T = 1 (schedule 5) at equal slab / G
    // (131072 / 106496 columns, profiles/probe_r2_t1_sched5.jsonl); T = 4 and T = 1 tie at 65536
    c.cost = (double)slab / c.G * (T == 2 ? 1.08 : 1.0) * narrow_slab_penalty(kw);
    return c;
}

}  // namespace

int64_t choose_ld(int64_t nvoxel, double max_waste, bool narrow_slabs) {
    // Widths the fused sweep (variant 6) can split into whole slabs, J <= 32 per row group: at each (T, kw) the
    // smallest multiple of the slab covering nvoxel. Take the one with the lowest time per row (ties: less
    // padding, then the larger T and kw, measured fastest at equal cost), if it pads by at most max_waste.
    if (nvoxel >= 1024) {
        constexpr int kPerXcd = 32;  // MI355X: 256 CUs in 8 XCDs
        int64_t best_ld = 0;
        double best_cost = 0.0;
        for (const int kw : {8, 7, 6}) {
            if (kw != 8 && !narrow_slabs) continue;
            for (const int T : {4, 2, 1}) {
                const int64_t slab = 1024 * (int64_t)kw / T;
                const int64_t ld = (nvoxel + slab - 1) / slab * slab;
                const V6Candidate c = v6_candidate(ld, T, kw, kPerXcd);
                if (c.G == 0 || (double)(ld - nvoxel) > max_waste * (double)nvoxel) continue;
                if (best_ld == 0 || c.cost < best_cost || (c.cost == best_cost && ld < best_ld)) {
                    best_ld = ld;
                    best_cost = c.cost;
                }
            }
        }
        if (best_ld) return best_ld;
        // wider than 32 slabs of 8192: a multiple of 8192 keeps the variant 3 fallback (K = 8) available
        const int64_t ld = (nvoxel + 8191) / 8192 * 8192;
        if ((double)(ld - nvoxel) <= max_waste * (double)nvoxel) return ld;
    }
    const int64_t n = std::max<int64_t>(nvoxel, 64);
    return (n + 63) / 64 * 64;
}

FusedGeometry fused_geometry(int64_t ld, int num_cus, int variant, int rows_per_tile, bool narrow_slabs) {
    FusedGeometry g;
    if (rows_per_tile <= 0) {
        const char* e = std::getenv("SART_FUSED_T");
        rows_per_tile = (e && *e) ? std::atoi(e) : 0;
    }
    if (const char* e = std::getenv("SART_FUSED_KW"); e && *e && std::atoi(e) == 8) narrow_slabs = false;
    if (variant == 6 && num_cus % 8 == 0) {
        // Rows per tile and slab: the requested T, else the candidate with the lowest time per row (ties: the
        // larger T and kw; T = 4 at ld = 64k, 2 at 128k, 1 at 256k measured 6.5-6.9 TB/s, against 4.0-4.7 TB/s
        // for variant 3, profiles/probe_r1_fused_T.jsonl). Widths whose J does not divide the XCD's CU count
        // run G = per_xcd / J row groups per XCD and leave the remaining CUs idle.
        V6Candidate best;
        for (const int kw : {8, 7, 6}) {
            if (kw != 8 && !narrow_slabs) continue;
            for (const int T : {4, 2, 1}) {
                if (rows_per_tile > 0 && T != rows_per_tile) continue;
                const V6Candidate c = v6_candidate(ld, T, kw, num_cus / 8);
                if (c.G > 0 && (best.G == 0 || c.cost < best.cost)) best = c;
            }
        }
        if (best.G > 0) {
            g.K = best.T, g.J = best.J, g.I = 8 * best.G, g.grid = g.I * g.J, g.variant = 6, g.T = best.T;
            g.kw = best.kw;
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
    if (num_cus % 8 != 0) return g;
    const int per_xcd = num_cus / 8;
    // T = 4 (slab 4096, schedule 4) or T = 2 (slab 8192, schedule 6: 3-slot ring, lag 3); the lower cost
    // slab / G wins, T = 4 on ties (the deeper lag measured faster at 64k x 64k)
    int64_t best_cost = 0;
    for (const int T : {4, 2}) {
        const int64_t slab = 16384 / T;
        if (ld % slab != 0) continue;
        const int64_t J = ld / slab;
        if (J < 1 || J > per_xcd) continue;
        const int G = per_xcd / (int)J;
        const int64_t cost = slab / G;
        if (g.valid() && cost >= best_cost) continue;
        best_cost = cost;
        g.K = T, g.T = T, g.cpl = 8, g.J = (int)J, g.I = 8 * G, g.grid = g.I * g.J, g.variant = 6;
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
    int64_t seg = 2240;  // > the 2048 tiles per group of the 64k x 64k headline: one chain there
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

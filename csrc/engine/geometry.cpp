#include "geometry.hpp"

#include <algorithm>
#include <cstdlib>

namespace sart {

int64_t choose_ld(int64_t nvoxel, double max_waste) {
    if (nvoxel >= 1024) {
        for (int K = 1; K <= 8; K *= 2) {
            const int64_t wc = 1024 * (int64_t)K;
            const int64_t J = (nvoxel + wc - 1) / wc;
            if (J <= 32 || K == 8) {
                const int64_t ld = J * wc;
                if ((double)(ld - nvoxel) <= max_waste * (double)nvoxel) return ld;
                break;
            }
        }
    }
    const int64_t n = std::max<int64_t>(nvoxel, 64);
    return (n + 63) / 64 * 64;
}

FusedGeometry fused_geometry(int64_t ld, int num_cus, int variant, int rows_per_tile) {
    FusedGeometry g;
    if (rows_per_tile <= 0) {
        const char* e = std::getenv("SART_FUSED_T");
        rows_per_tile = (e && *e) ? std::atoi(e) : 0;
    }
    if (variant == 4 || variant == 6) {
        // Rows per tile: the requested T, else the largest of 4, 2, 1 whose row group fits the XCD (T = 4 at
        // ld = 64k, 2 at 128k, 1 at 256k: 6.5-6.9 TB/s, against 4.0-4.7 TB/s for variant 3 at those widths,
        // profiles/probe_r1_fused_T.jsonl).
        const int per_xcd = num_cus / 8;
        for (const int T : {4, 2, 1}) {
            if (rows_per_tile > 0 && T != rows_per_tile) continue;
            const int64_t slab = 8192 / T;
            if (ld % slab != 0 || ld / slab == 0) continue;
            const int J = (int)(ld / slab);
            if (variant == 6 && num_cus % 8 == 0 && per_xcd % J == 0) {
                g.K = T, g.J = J, g.I = 8 * (per_xcd / J), g.grid = g.I * g.J, g.variant = 6, g.T = T;
                return g;
            }
            if (variant == 4 && J <= std::min(64, num_cus)) {
                g.K = T, g.J = J, g.I = std::max(1, num_cus / J), g.grid = g.I * g.J, g.variant = 4, g.T = T;
                return g;
            }
        }
        variant = 3;
    }
    if (variant == 5) {
        if (ld % 2048 == 0 && ld / 2048 > 0 && ld / 2048 <= std::min(64, num_cus)) {
            g.K = 8, g.J = (int)(ld / 2048), g.I = std::max(1, num_cus / g.J), g.grid = g.I * g.J, g.variant = 5,
            g.T = 4;
            return g;
        }
        variant = 3;
    }
    for (int K = 1; K <= 8; K *= 2) {
        const int64_t wc = 1024 * (int64_t)K;
        if (ld % wc) continue;
        const int64_t J = ld / wc;
        if (J <= 32 || K == 8) {
            const int v = (variant != 2 || K <= 4) ? variant : 3;
            const int T = v == 2 ? 4 / K : 8 / K;
            if (J > num_cus || J * T > 512) return g;
            g.K = K, g.J = (int)J, g.I = std::max(1, num_cus / (int)J), g.grid = g.I * g.J, g.variant = v, g.T = T;
            return g;
        }
    }
    return g;
}

}  // namespace sart

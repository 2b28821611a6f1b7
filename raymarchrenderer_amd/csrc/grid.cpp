// grid.cpp — host construction of the candidate grid (see grid.hpp and rmr_trace.h map_grid_npc).
//
// Per cell C (inflated past the rounding of the kernel's cell index): U = the smallest distance
// upper bound over C of any primitive (box and sphere SDFs are convex: the largest corner value);
// the list = the small primitives whose distance lower bound over C is <= U + margin (margin = 4 x the
// float evaluation error bound of a distance anywhere in the grid), so every unlisted primitive's
// float distance is strictly above the minimum's; the cell's bound = the smallest lower bound of an
// unlisted one, minus that error bound. Exact arithmetic in double.
#include "grid.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>

#include "../../include/rmr_tables.h"

namespace rmr {

bool build_candidate_grid(const std::vector<DPrim>& dp, int n_large, double E, double target, double pad,
                          CandidateGrid& g) {
    const int n = (int)dp.size();
    if (n - n_large < 1 || n > 65535) return false;
    auto half = [&](const DPrim& q, int k) {
        return (double)std::fabs((q.type & 0xff) == RMR_PRIM_SPHERE ? q.r[0] : q.r[k]);
    };
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int i = n_large; i < n; i++)
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], (double)dp[(size_t)i].c[k] - half(dp[(size_t)i], k));
            hi[k] = std::max(hi[k], (double)dp[(size_t)i].c[k] + half(dp[(size_t)i], k));
        }
    // the region: the small primitives' box grown by pad x its largest extent on every side, its lower
    // side clipped to the box of all primitives (large ones included) grown by one cell
    double alo[3] = {1e300, 1e300, 1e300}, ahi[3] = {-1e300, -1e300, -1e300};
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            alo[k] = std::min(alo[k], (double)dp[(size_t)i].c[k] - half(dp[(size_t)i], k));
            ahi[k] = std::max(ahi[k], (double)dp[(size_t)i].c[k] + half(dp[(size_t)i], k));
        }
    const double ext = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    double rlo[3], rhi[3];
    for (int k = 0; k < 3; k++) {
        rlo[k] = lo[k] - pad * ext;
        rhi[k] = hi[k] + pad * ext;
    }
    double cs = std::cbrt(std::max(1e-30, (rhi[0] - rlo[0]) * (rhi[1] - rlo[1]) * (rhi[2] - rlo[2])) / target);
    for (int k = 0; k < 3; k++) rlo[k] = std::max(rlo[k], alo[k] - cs);   // (march points above the scene occur)
    cs = std::cbrt(std::max(1e-30, (rhi[0] - rlo[0]) * (rhi[1] - rlo[1]) * (rhi[2] - rlo[2])) / target);
    for (int k = 0; k < 3; k++) cs = std::max(cs, (rhi[k] - rlo[k]) / 1024.0);
    if (!(cs > 0.0) || !std::isfinite(cs)) return false;
    int dim[3];
    float flo[3];
    double pmax = E;
    for (int k = 0; k < 3; k++) {
        flo[k] = (float)rlo[k];
        dim[k] = std::max(1, (int)std::ceil((rhi[k] - (double)flo[k]) / cs));
        pmax = std::max(pmax, std::max(std::fabs((double)flo[k]), std::fabs((double)flo[k] + dim[k] * cs)));
    }
    const float finv = (float)(1.0 / cs);
    const double csf = 1.0 / (double)finv;   // the cell size the kernel's index arithmetic implies
    const size_t ncell = (size_t)dim[0] * dim[1] * dim[2];
    if (ncell > ((size_t)1 << 24)) return false;
    // float error bound of a box/sphere distance at |p|_inf <= pmax (rmr_trace.h npc_eps, 4x slack)
    const double eps = std::ldexp(pmax + E, -17);
    const double margin = 4.0 * eps;
    const double infl = 1e-4 + std::ldexp(pmax, -16) + 4.0 * std::ldexp(csf, -20);   // cell index rounding
    struct PB { double c[3], h[3], rad; bool box; };
    std::vector<PB> pb((size_t)n);
    for (int i = 0; i < n; i++) {
        const DPrim& q = dp[(size_t)i];
        PB b{};
        b.box = (q.type & 0xff) == RMR_PRIM_BOX;
        for (int k = 0; k < 3; k++) { b.c[k] = q.c[k]; b.h[k] = b.box ? (double)q.r[k] : 0.0; }
        b.rad = b.box ? 0.0 : (double)q.r[0];
        pb[(size_t)i] = b;
    }
    // distance bounds of primitive b over the cell [a0, a1]: lower (Euclidean distance to the box of
    // half-extent |h| minus the radius; -min|h| - rad when they overlap) and upper (the largest corner value)
    auto bounds = [&](const PB& b, const double* a0, const double* a1, double& dmin, double& dmax) {
        double s2 = 0.0, f2 = 0.0, mh = 1e300;
        bool overlap = true;
        for (int k = 0; k < 3; k++) {
            const double h = std::fabs(b.h[k]);
            const double gap = std::max({a0[k] - (b.c[k] + h), (b.c[k] - h) - a1[k], 0.0});
            if (gap > 0.0) overlap = false;
            s2 += gap * gap;
            mh = std::min(mh, h);
        }
        dmin = overlap ? (b.box ? -mh : -b.rad) : std::sqrt(s2) - b.rad;
        dmax = -1e300;
        for (int corner = 0; corner < 8; corner++) {
            double qv[3], mq = -1e300, o2 = 0.0;
            for (int k = 0; k < 3; k++) {
                const double x = (corner >> k) & 1 ? a1[k] : a0[k];
                qv[k] = std::fabs(x - b.c[k]) - b.h[k];
                mq = std::max(mq, qv[k]);
                o2 += std::max(qv[k], 0.0) * std::max(qv[k], 0.0);
            }
            (void)f2;
            dmax = std::max(dmax, std::min(mq, 0.0) + std::sqrt(o2) - b.rad);
        }
    };
    std::vector<std::vector<uint16_t>> lists(ncell);
    std::vector<uint32_t> cnt(ncell);
    std::vector<float> lout(ncell);
    auto work = [&](int z0, int z1) {
        std::vector<double> dmn((size_t)n), dmx((size_t)n);
        for (int z = z0; z < z1; z++)
            for (int y = 0; y < dim[1]; y++)
                for (int x = 0; x < dim[0]; x++) {
                    const int ii[3] = {x, y, z};
                    double a0[3], a1[3];
                    for (int k = 0; k < 3; k++) {
                        a0[k] = (double)flo[k] + ii[k] * csf - infl;
                        a1[k] = (double)flo[k] + (ii[k] + 1) * csf + infl;
                    }
                    double U = 1e300;
                    for (int i = 0; i < n; i++) {
                        bounds(pb[(size_t)i], a0, a1, dmn[(size_t)i], dmx[(size_t)i]);
                        U = std::min(U, dmx[(size_t)i]);
                    }
                    const size_t ci = ((size_t)z * dim[1] + y) * dim[0] + x;
                    double lo_out = 1e300;
                    std::vector<uint16_t>& L = lists[ci];
                    for (int i = n_large; i < n; i++) {
                        if (dmn[(size_t)i] <= U + margin) L.push_back((uint16_t)i);
                        else lo_out = std::min(lo_out, dmn[(size_t)i]);
                    }
                    if (L.size() > 254) { cnt[ci] = 255; L.clear(); }
                    else cnt[ci] = (uint32_t)L.size();
                    float lf = lo_out >= 1e300 ? HUGE_VALF : (float)(lo_out - eps);
                    if ((double)lf > lo_out - eps) lf = std::nextafter(lf, -HUGE_VALF);
                    lout[ci] = lf;
                }
    };
    {
        const int nt = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        const int per = (dim[2] + nt - 1) / nt;
        for (int t = 0; t < nt; t++) {
            const int z0 = t * per, z1 = std::min(dim[2], z0 + per);
            if (z0 < z1) th.emplace_back(work, z0, z1);
        }
        for (auto& t : th) t.join();
    }
    g.cells.assign(2 * ncell, 0u);
    g.list.clear();
    for (size_t i = 0; i < ncell; i++) {
        if (g.list.size() + lists[i].size() >= ((size_t)1 << 24)) return false;
        g.cells[2 * i] = (uint32_t)g.list.size() | (cnt[i] << 24);
        uint32_t lb;
        std::memcpy(&lb, &lout[i], 4);
        g.cells[2 * i + 1] = lb;
        g.list.insert(g.list.end(), lists[i].begin(), lists[i].end());
    }
    for (int k = 0; k < 3; k++) {
        g.lo[k] = flo[k];
        g.dim[k] = dim[k];
        float l = (float)lo[k], h = (float)hi[k];   // the small primitives' box, rounded outward
        if ((double)l > lo[k]) l = std::nextafter(l, -HUGE_VALF);
        if ((double)h < hi[k]) h = std::nextafter(h, HUGE_VALF);
        g.sbox[k] = l;
        g.sbox[3 + k] = h;
    }
    g.inv = finv;
    g.n_large = n_large;
    g.margin = margin;
    g.eps = eps;
    return true;
}

}  // namespace rmr

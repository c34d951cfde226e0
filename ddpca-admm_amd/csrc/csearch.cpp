// Contact search: restatement of CSEARCH::BUCKET_SORT / CONTACT_SEARCH / SEGMENT_INTERSECT
// (CSEARCH.h:205-230, 614-817) -- the producer of the integration points (INTEGRAL_POINT,
// CSEARCH.h:19-32) that MCONTACT::ESTABLISH turns into the interface operators.  Setup-time host
// code: each slave face is intersected with the master faces of the 3 x 3 buckets around it, in
// the reference's order (slave face, bucket row, bucket column, insertion order in the bucket), the
// slave faces spread over OpenMP threads and their points concatenated in order.
//
// Per master/slave face pair (SI_SUB, CSEARCH.h:614-733): the slave corners are projected onto the
// master face (closest point, PROJECT_STM 401-428), the intersection polygon of the two quads is
// clipped in the master's natural coordinates, de-duplicated (1e-10), sorted by angle about its
// vertex mean, and every (centroid, edge) triangle gets the 4-point collapsed Gauss rule
// (TRIANGLE_QUADRATURE, PREP.h); each point is projected onto the slave face along the master
// normal (PROJECT_MTS 232-307) for its slave shape values, basis (master normal and tangents),
// initial gap and weight (MAST_TO_SLAV 430-459, SEGMENT_INTERSECT 735-775).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <omp.h>
#include <string>
#include <vector>

#include "../../include/ddpca_amd.h"
#include "common.hpp"
#include "mcontact.hpp"

using namespace ddpca;

namespace {

struct V3 {
    double x[3];
    double& operator[](int i) { return x[i]; }
    double operator[](int i) const { return x[i]; }
};
struct V2 {
    double x, y;
};

const double kCorn[4][2] = {{-1, -1}, {1, -1}, {1, 1}, {-1, 1}};  // biliQuad.nacoCorn
const double kMiniArea = 1.0e-12;                                  // CSEARCH.h:12

double dot3(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
V3 cross3(const V3& a, const V3& b) {
    return V3{{a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]}};
}
V3 normalized(const V3& a) {
    const double n = std::sqrt(dot3(a, a));
    return V3{{a[0] / n, a[1] / n, a[2] / n}};
}

// 2x2 solve with full pivoting (the reference uses Eigen's fullPivLu on these Newton systems)
void solve2(const double A[2][2], const double b[2], double x[2]) {
    int pr = 0, pc = 0;
    double amax = -1.0;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            if (std::abs(A[i][j]) > amax) amax = std::abs(A[i][j]), pr = i, pc = j;
    const int qr = 1 - pr, qc = 1 - pc;
    if (amax == 0.0) {
        x[0] = x[1] = 0.0;
        return;
    }
    const double l = A[qr][pc] / A[pr][pc];
    const double u = A[qr][qc] - l * A[pr][qc];
    const double y = b[qr] - l * b[pr];
    double xq = u != 0.0 ? y / u : 0.0;
    double xp = (b[pr] - A[pr][qc] * xq) / A[pr][pc];
    x[pc] = xp;
    x[qc] = xq;
}

// bilinear face X(xi, eta) = f0 + f1 xi + f2 eta + f3 xi eta (factMatr of CSEARCH.h:246-255)
void bilinear(const V3 c[4], V3 f[4]) {
    for (int i = 0; i < 3; ++i) {
        f[0][i] = f[1][i] = f[2][i] = f[3][i] = 0.0;
        for (int k = 0; k < 4; ++k) {
            f[0][i] += c[k][i] / 4.0;
            f[1][i] += c[k][i] * kCorn[k][0] / 4.0;
            f[2][i] += c[k][i] * kCorn[k][1] / 4.0;
            f[3][i] += c[k][i] * kCorn[k][0] * kCorn[k][1] / 4.0;
        }
    }
}

// tangents dX/dxi, dX/deta of a face at (xi, eta) (PrmaPxie, CSEARCH.h:237-245)
void tangents(const V3 c[4], double xi, double et, V3& t1, V3& t2) {
    for (int i = 0; i < 3; ++i) {
        t1[i] = t2[i] = 0.0;
        for (int k = 0; k < 4; ++k) {
            t1[i] += c[k][i] * (kCorn[k][0] / 4.0 + kCorn[k][0] * kCorn[k][1] * et / 4.0);
            t2[i] += c[k][i] * (kCorn[k][1] / 4.0 + kCorn[k][0] * kCorn[k][1] * xi / 4.0);
        }
    }
}

// closest point of P on the master face: Newton on the gradient of |X - P|^2 from (xi, eta)
// (PROJECT_STM_SUB, CSEARCH.h:309-398)
void project_stm_sub(const V3 f[4], const V3& P, double& xi, double& et) {
    V3 d;  // f0 - P
    for (int i = 0; i < 3; ++i) d[i] = f[0][i] - P[i];
    const double f11 = dot3(f[1], f[1]), f22 = dot3(f[2], f[2]), f33 = dot3(f[3], f[3]);
    const double f12 = dot3(f[1], f[2]), f13 = dot3(f[1], f[3]), f23 = dot3(f[2], f[3]);
    const double d1 = dot3(d, f[1]), d2 = dot3(d, f[2]), d3 = dot3(d, f[3]);
    // (X - P).dX/dxi = d1 + f11 xi + (f12 + d3) eta + 2 f13 xi eta + f23 eta^2 + f33 xi eta^2, and
    // the same with xi <-> eta, 1 <-> 2
    for (int it = 0; it < 60; ++it) {
        const double r0 = d1 + f11 * xi + (f12 + d3) * et + 2.0 * f13 * xi * et + f23 * et * et + f33 * xi * et * et;
        const double r1 = d2 + f22 * et + (f12 + d3) * xi + 2.0 * f23 * xi * et + f13 * xi * xi + f33 * xi * xi * et;
        const double J[2][2] = {{f11 + 2.0 * f13 * et + f33 * et * et, (f12 + d3) + 2.0 * f13 * xi + 2.0 * f23 * et + 2.0 * f33 * xi * et},
                                {(f12 + d3) + 2.0 * f23 * et + 2.0 * f13 * xi + 2.0 * f33 * xi * et, f22 + 2.0 * f23 * xi + f33 * xi * xi}};
        const double r[2] = {r0, r1};
        double dx[2];
        solve2(J, r, dx);
        dx[0] = -dx[0];
        dx[1] = -dx[1];
        if (std::sqrt(dx[0] * dx[0] + dx[1] * dx[1]) < 1.0e-12 && std::sqrt(r0 * r0 + r1 * r1) < 1.0e-15) break;
        xi += dx[0];
        et += dx[1];
    }
}

// PROJECT_STM (CSEARCH.h:401-428): far points are approached in steps of the face's shortest
// corner distance, each Newton solve starting where the previous one ended
void project_stm(const V3 c[4], const V3& P, double& xi, double& et) {
    V3 f[4];
    bilinear(c, f);
    double diam = 1.0e15;
    V3 cent{{0.0, 0.0, 0.0}};
    for (int i = 0; i < 4; ++i) {
        for (int j = i + 1; j < 4; ++j) {
            V3 e{{c[i][0] - c[j][0], c[i][1] - c[j][1], c[i][2] - c[j][2]}};
            diam = std::min(diam, std::sqrt(dot3(e, e)));
        }
        for (int a = 0; a < 3; ++a) cent[a] += 0.25 * c[i][a];
    }
    xi = et = 0.0;
    V3 dv{{P[0] - cent[0], P[1] - cent[1], P[2] - cent[2]}};
    const double dist = std::sqrt(dot3(dv, dv));
    if (dist > diam) {
        const double steps = dist / diam;
        for (long t = 0; t < steps; ++t) {
            V3 Q{{cent[0] + t * diam * dv[0] / dist, cent[1] + t * diam * dv[1] / dist, cent[2] + t * diam * dv[2] / dist}};
            project_stm_sub(f, Q, xi, et);
        }
    }
    project_stm_sub(f, P, xi, et);
}

// point X_m of the master face projected along... the slave face point whose position satisfies
// (X_s(s) - X_m) . t_k = 0 for the master tangents t_k at the master point (PROJECT_MTS,
// CSEARCH.h:232-307); returns the slave natural coordinates
void project_mts(const V3 mc[4], const V3 sc[4], double xi, double et, const V3& Xm, double s[2]) {
    V3 t1, t2, g[4];
    tangents(mc, xi, et, t1, t2);
    bilinear(sc, g);
    // (g0 - Xm + g1 s0 + g2 s1 + g3 s0 s1) . t_k = 0
    const double e00 = dot3(g[0], t1) - dot3(Xm, t1), e01 = dot3(g[1], t1), e02 = dot3(g[2], t1), e03 = dot3(g[3], t1);
    const double e10 = dot3(g[0], t2) - dot3(Xm, t2), e11 = dot3(g[1], t2), e12 = dot3(g[2], t2), e13 = dot3(g[3], t2);
    s[0] = s[1] = 0.0;
    for (int it = 0; it < 60; ++it) {
        const double r[2] = {e00 + e01 * s[0] + e02 * s[1] + e03 * s[0] * s[1], e10 + e11 * s[0] + e12 * s[1] + e13 * s[0] * s[1]};
        const double J[2][2] = {{e01 + e03 * s[1], e02 + e03 * s[0]}, {e11 + e13 * s[1], e12 + e13 * s[0]}};
        double dx[2];
        solve2(J, r, dx);
        dx[0] = -dx[0];
        dx[1] = -dx[1];
        if (std::sqrt(dx[0] * dx[0] + dx[1] * dx[1]) < 1.0e-14 && std::sqrt(r[0] * r[0] + r[1] * r[1]) < 1.0e-15) break;
        s[0] += dx[0];
        s[1] += dx[1];
    }
}

double tri_area(const V2& a, const V2& b, const V2& c) {
    return std::abs((b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x)) / 2.0;
}

// segment intersection of p0p1 with p2p3 (IS_CROSS_2D / LINE_INTERSECT_2D, CSEARCH.h:495-597)
void segment_cross(V2 p0, V2 p1, V2 p2, V2 p3, std::vector<V2>& out) {
    if (std::max(p0.x, p1.x) < std::min(p2.x, p3.x) || std::max(p0.y, p1.y) < std::min(p2.y, p3.y) ||
        std::min(p0.x, p1.x) > std::max(p2.x, p3.x) || std::min(p0.y, p1.y) > std::max(p2.y, p3.y))
        return;
    const bool straddle =
        ((p2.x - p0.x) * (p2.y - p3.y) - (p2.y - p0.y) * (p2.x - p3.x)) * ((p2.x - p1.x) * (p2.y - p3.y) - (p2.y - p1.y) * (p2.x - p3.x)) <= 0 &&
        ((p0.x - p2.x) * (p0.y - p1.y) - (p0.y - p2.y) * (p0.x - p1.x)) * ((p0.x - p3.x) * (p0.y - p1.y) - (p0.y - p3.y) * (p0.x - p1.x)) <= 0;
    if (!straddle) return;
    const double a2 = tri_area(p2, p0, p1), a3 = tri_area(p3, p0, p1);
    if (std::abs(a2) < kMiniArea && std::abs(a3) < kMiniArea) {  // collinear: the overlap
        const bool byx = std::abs(p0.x - p1.x) > 1.0e-10;
        auto key = [&](const V2& p) { return byx ? p.x : p.y; };
        if (key(p0) > key(p1)) std::swap(p0, p1);
        if (key(p2) > key(p3)) std::swap(p2, p3);
        V2 from = key(p0) < key(p2) ? p2 : p0;
        V2 to = key(p1) > key(p3) ? p3 : p1;
        out.push_back(from);
        if (!(std::abs(from.x - to.x) < 1.0e-10)) out.push_back(to);
    } else if (std::abs(a2) < kMiniArea) {
        out.push_back(p2);
    } else if (std::abs(a3) < kMiniArea) {
        out.push_back(p3);
    } else {
        const double f = a2 / a3;
        out.push_back(V2{(p2.x + f * p3.x) / (1.0 + f), (p2.y + f * p3.y) / (1.0 + f)});
    }
}

bool in_quad(const V2& p, const V2 q[4]) {  // IN_CQUAD_2D (CSEARCH.h:599-612)
    double s = 0.0;
    for (int i = 0; i < 4; ++i) s += tri_area(p, q[i], q[(i + 1) % 4]);
    return s <= (1.0 + 1.0e-12) * (tri_area(q[0], q[1], q[2]) + tri_area(q[2], q[3], q[0]));
}

// the intersection polygon's quadrature points (master natural coordinates) and weights
// (SI_SUB, CSEARCH.h:614-733)
void polygon_points(const V3 mc[4], const V3 sc[4], std::vector<V2>& pts, std::vector<double>& wts) {
    const V2 mp[4] = {{-1, -1}, {1, -1}, {1, 1}, {-1, 1}};
    V2 sp[4];
    for (int i = 0; i < 4; ++i) project_stm(mc, sc[i], sp[i].x, sp[i].y);
    std::vector<V2> p0;
    for (int i = 0; i < 4; ++i) {
        if (in_quad(sp[i], mp)) p0.push_back(sp[i]);
        if (in_quad(mp[i], sp)) p0.push_back(mp[i]);
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) segment_cross(mp[i], mp[(i + 1) % 4], sp[j], sp[(j + 1) % 4], p0);
    if (p0.size() < 3) return;
    std::vector<int> idx(p0.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) {
        if (p0[a].x < p0[b].x - 1.0e-10) return true;
        if (p0[a].x <= p0[b].x + 1.0e-10) return p0[a].y < p0[b].y - 1.0e-10;
        return false;
    });
    std::vector<V2> p1{p0[idx[0]]};
    for (size_t i = 1; i < idx.size(); ++i)
        if (std::abs(p0[idx[i]].x - p0[idx[i - 1]].x) > 1.0e-10 || std::abs(p0[idx[i]].y - p0[idx[i - 1]].y) > 1.0e-10)
            p1.push_back(p0[idx[i]]);
    V2 cm{0.0, 0.0};
    for (const V2& p : p1) cm.x += p.x, cm.y += p.y;
    cm.x /= (double)p1.size();
    cm.y /= (double)p1.size();
    std::vector<double> ang(p1.size());
    for (size_t i = 0; i < p1.size(); ++i) ang[i] = std::atan2(p1[i].y - cm.y, p1[i].x - cm.x);
    idx.resize(p1.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return ang[a] < ang[b]; });
    std::vector<V2> poly(p1.size());
    for (size_t i = 0; i < idx.size(); ++i) poly[i] = p1[idx[i]];
    // area and centroid of the polygon (shoelace)
    const size_t n = poly.size();
    double area = 0.0, cx = 0.0, cy = 0.0;
    for (size_t i = 0; i < n; ++i) {
        const V2& a = poly[i];
        const V2& b = poly[(i + 1) % n];
        const double cr = a.x * b.y - b.x * a.y;
        area += cr;
        cx += (a.x + b.x) * cr;
        cy += (a.y + b.y) * cr;
    }
    area /= 2.0;
    if (std::abs(area) <= kMiniArea) return;
    cx = cx / 6.0 / area;
    cy = cy / 6.0 / area;
    const V2 c{cx, cy};
    const double g = std::sqrt(1.0 / 3.0), gl[2] = {-g, g};
    for (size_t t = 0; t < n; ++t) {  // TRIANGLE_QUADRATURE on (centroid, v_t, v_t+1)
        const V2& v1 = poly[t];
        const V2& v2 = poly[(t + 1) % n];
        const double a = tri_area(c, v1, v2);
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) {
                const double b0 = (1.0 + gl[i]) / 2.0, b1 = (1.0 - gl[i]) * (1.0 + gl[j]) / 4.0, b2 = 1.0 - b0 - b1;
                pts.push_back(V2{b0 * c.x + b1 * v1.x + b2 * v2.x, b0 * c.y + b1 * v1.y + b2 * v2.y});
                wts.push_back(2.0 * a * ((1.0 - gl[i]) / 8.0));
            }
    }
}

// SEGMENT_INTERSECT (CSEARCH.h:735-775) for one master / slave face pair
void segment_intersect(const V3 mc[4], const V3 sc[4], const int64_t mn[4], const int64_t sn[4],
                       std::vector<IntegralPoint>& out) {
    std::vector<V2> pts;
    std::vector<double> wts;
    polygon_points(mc, sc, pts, wts);
    for (size_t q = 0; q < pts.size(); ++q) {
        IntegralPoint p;
        V3 Xm{{0.0, 0.0, 0.0}}, Xs{{0.0, 0.0, 0.0}};
        for (int k = 0; k < 4; ++k) {
            p.node[0][k] = mn[k];
            p.node[1][k] = sn[k];
            p.shap[0][k] = (1.0 + kCorn[k][0] * pts[q].x) * (1.0 + kCorn[k][1] * pts[q].y) / 4.0;
            for (int a = 0; a < 3; ++a) Xm[a] += p.shap[0][k] * mc[k][a];
        }
        double s[2];
        project_mts(mc, sc, pts[q].x, pts[q].y, Xm, s);
        V3 t1, t2;
        tangents(mc, pts[q].x, pts[q].y, t1, t2);
        const V3 nrm = normalized(cross3(t1, t2)), e1 = normalized(t1), e2 = normalized(t2);
        const V3 tc = cross3(t1, t2);
        const double wf = std::sqrt(tc[0] * tc[0] + tc[1] * tc[1] + tc[2] * tc[2]);
        for (int k = 0; k < 4; ++k) {
            p.shap[1][k] = (1.0 + kCorn[k][0] * s[0]) * (1.0 + kCorn[k][1] * s[1]) / 4.0;
            for (int a = 0; a < 3; ++a) Xs[a] += p.shap[1][k] * sc[k][a];
        }
        for (int a = 0; a < 3; ++a) {
            p.basis[0][a] = nrm[a];
            p.basis[1][a] = e1[a];
            p.basis[2][a] = e2[a];
        }
        p.gap = (Xs[0] - Xm[0]) * nrm[0] + (Xs[1] - Xm[1]) * nrm[1] + (Xs[2] - Xm[2]) * nrm[2];
        p.w = wts[q] * wf;
        out.push_back(p);
    }
}

// BUCKET_SORT (CSEARCH.h:205-230) + CONTACT_SEARCH (CSEARCH.h:777-817): every (master, slave) face
// pair of the 3 x 3 buckets around the slave face whose intersection has a point within maxiDist;
// per slave face, in the reference's order
std::vector<std::vector<IntegralPoint>> search(const double* mast_xyz, int64_t mast_nnode, const double* slav_xyz,
                                               int64_t slav_nnode, int64_t nm, const int64_t* mast_segm, const double* mast_2d,
                                               int64_t ns, const int64_t* slav_segm, const double* slav_2d, const int64_t* buck,
                                               double maxiDist) {
    if (!mast_xyz || !slav_xyz || !mast_segm || !slav_segm || !mast_2d || !slav_2d || !buck || nm < 1 || ns < 0)
        throw ApiError(DDPCA_EINVAL, "null argument / no master faces");
    if (buck[0] < 1 || buck[1] < 1) throw ApiError(DDPCA_EINVAL, "bucket counts >= 1");
    for (int64_t i = 0; i < 4 * nm; ++i)
        if (mast_segm[i] < 0 || mast_segm[i] >= mast_nnode) throw ApiError(DDPCA_EINVAL, "master face node out of range");
    for (int64_t i = 0; i < 4 * ns; ++i)
        if (slav_segm[i] < 0 || slav_segm[i] >= slav_nnode) throw ApiError(DDPCA_EINVAL, "slave face node out of range");
    double lo[2], step[2];
    for (int a = 0; a < 2; ++a) {
        double mn = mast_2d[a], mx = mast_2d[a];
        for (int64_t i = 0; i < nm; ++i) mn = std::min(mn, mast_2d[2 * i + a]), mx = std::max(mx, mast_2d[2 * i + a]);
        double inc = (mx - mn) / (double)buck[a];
        if (std::abs(inc) < 1.0e-10) inc = 1.0e-10;
        lo[a] = mn - inc;
        step[a] = ((mx + inc) - lo[a]) / (double)buck[a];
    }
    std::vector<std::vector<int64_t>> bucket(buck[0] * buck[1]);
    for (int64_t i = 0; i < nm; ++i) {
        const long r = (long)((mast_2d[2 * i] - lo[0]) / step[0]), c = (long)((mast_2d[2 * i + 1] - lo[1]) / step[1]);
        bucket[r * buck[1] + c].push_back(i);
    }
    auto corners = [](const double* xyz, const int64_t* seg, V3 c[4]) {
        for (int k = 0; k < 4; ++k)
            for (int a = 0; a < 3; ++a) c[k][a] = xyz[3 * seg[k] + a];
    };
    // CONTACT_SEARCH (CSEARCH.h:777-817): slave faces in order, each over its 3 x 3 buckets
    std::vector<std::vector<IntegralPoint>> per(ns);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t t = 0; t < ns; ++t) {
        const long r = (long)((slav_2d[2 * t] - lo[0]) / step[0]), c = (long)((slav_2d[2 * t + 1] - lo[1]) / step[1]);
        if (r < 0 || r > buck[0] - 1 || c < 0 || c > buck[1] - 1) continue;
        V3 sc[4];
        corners(slav_xyz, slav_segm + 4 * t, sc);
        std::vector<IntegralPoint> e;
        for (long j = std::max(r - 1, 0L); j <= std::min(r + 1, (long)buck[0] - 1); ++j)
            for (long k = std::max(c - 1, 0L); k <= std::min(c + 1, (long)buck[1] - 1); ++k)
                for (int64_t m : bucket[j * buck[1] + k]) {
                    V3 mc[4];
                    corners(mast_xyz, mast_segm + 4 * m, mc);
                    e.clear();
                    segment_intersect(mc, sc, mast_segm + 4 * m, slav_segm + 4 * t, e);
                    bool keep = false;
                    for (const auto& p : e) keep |= p.gap <= maxiDist;
                    if (keep) per[t].insert(per[t].end(), e.begin(), e.end());
                }
    }
    return per;
}

}  // namespace

struct ddpca_ips {
    std::vector<IntegralPoint> ip;
};

extern "C" {

int ddpca_contact_search(const double* mast_xyz, int64_t mast_nnode, const double* slav_xyz, int64_t slav_nnode,
                         int64_t nm, const int64_t* mast_segm, const double* mast_2d, int64_t ns,
                         const int64_t* slav_segm, const double* slav_2d, const int64_t* buck, double maxiDist,
                         ddpca_ips_t* out) {
    return guarded([&] {
        if (!out) throw ApiError(DDPCA_EINVAL, "null argument");
        auto per = search(mast_xyz, mast_nnode, slav_xyz, slav_nnode, nm, mast_segm, mast_2d, ns, slav_segm, slav_2d, buck,
                          maxiDist);
        auto R = std::make_unique<ddpca_ips>();
        size_t total = 0;
        for (const auto& v : per) total += v.size();
        R->ip.reserve(total);
        for (auto& v : per) R->ip.insert(R->ip.end(), v.begin(), v.end());
        *out = R.release();
    });
}

int ddpca_refine_select(const double* mast_xyz, int64_t mast_nnode, const double* slav_xyz, int64_t slav_nnode,
                        int64_t nm, const int64_t* mast_segm, const double* mast_2d, int64_t ns, const int64_t* slav_segm,
                        const double* slav_2d, const int64_t* buck, double distCrit, int64_t ne_m, const int64_t* mast_elem,
                        int64_t ne_s, const int64_t* slav_elem, uint8_t* mast_split, uint8_t* slav_split) {
    int any = 0;
    const int rc = guarded([&] {
        if ((ne_m > 0 && (!mast_elem || !mast_split)) || (ne_s > 0 && (!slav_elem || !slav_split)) || ne_m < 0 || ne_s < 0)
            throw ApiError(DDPCA_EINVAL, "null argument");
        // the face pairs whose intersection comes within distCrit (ADAPTIVE_REFINE's miniNgap <=
        // distCrit is CONTACT_SEARCH's keep rule): every node of their points is a split node
        const auto per = search(mast_xyz, mast_nnode, slav_xyz, slav_nnode, nm, mast_segm, mast_2d, ns, slav_segm, slav_2d,
                                buck, distCrit);
        std::vector<uint8_t> split[2] = {std::vector<uint8_t>(mast_nnode, 0), std::vector<uint8_t>(slav_nnode, 0)};
        for (const auto& v : per)
            for (const auto& p : v)
                for (int s = 0; s < 2; ++s)
                    for (int k = 0; k < 4; ++k) {
                        split[s][p.node[s][k]] = 1;
                        any = 1;
                    }
        // candidate elements with a split corner node are refined (CSEARCH.h:927-952)
        const int64_t ne[2] = {ne_m, ne_s};
        const int64_t* el[2] = {mast_elem, slav_elem};
        uint8_t* fl[2] = {mast_split, slav_split};
        const int64_t nn[2] = {mast_nnode, slav_nnode};
        for (int s = 0; s < 2; ++s)
            for (int64_t e = 0; e < ne[s]; ++e) {
                uint8_t f = 0;
                for (int k = 0; k < 8; ++k) {
                    const int64_t n = el[s][8 * e + k];
                    if (n < 0 || n >= nn[s]) throw ApiError(DDPCA_EINVAL, "element corner node out of range");
                    f |= split[s][n];
                }
                fl[s][e] = f;
            }
    });
    return rc != 0 ? rc : any;
}

int64_t ddpca_ips_count(ddpca_ips_t h) { return h ? (int64_t)h->ip.size() : -1; }

int ddpca_ips_get(ddpca_ips_t h, int64_t* node, double* shap, double* basis, double* gap, double* w) {
    return guarded([&] {
        if (!h) throw ApiError(DDPCA_EINVAL, "null handle");
        const int64_t n = (int64_t)h->ip.size();
        for (int64_t q = 0; q < n; ++q) {
            const IntegralPoint& p = h->ip[q];
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    if (node) node[8 * q + 4 * s + k] = p.node[s][k];
                    if (shap) shap[8 * q + 4 * s + k] = p.shap[s][k];
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b)
                    if (basis) basis[9 * q + 3 * a + b] = p.basis[a][b];
            if (gap) gap[q] = p.gap;
            if (w) w[q] = p.w;
        }
    });
}

int ddpca_ips_destroy(ddpca_ips_t h) {
    delete h;
    return DDPCA_OK;
}

}  // extern "C"

// Host restatement of MCONTACT::LAGRANGE (MCONTACT.h:2847-3701): dual mortar basis, nodal
// normal/tangent frames, normal-tangential mortar coupling, static condensation of the
// non-mortar dofs and the semi-smooth Newton active-set loop (stick / slip / open).  Every
// Newton step's condensed system (and, for precType 1, the MGPIS hierarchy the reference builds
// for it, MCONTACT.h:3419-3561) goes to the `solve` callback -- the device BiCGSTAB in
// capi_lagrange.hip.  The sparse algebra follows the reference's operation order on CSR
// (csr_ops.hpp); the reference's std::map iteration orders are kept, so unknown numbering,
// condensed-dof choice and the Newton decisions are the reference's.
#include "lagrange.hpp"

#include <cmath>
#include <set>
#include <stdexcept>
#include <string>

#include "csr_ops.hpp"

namespace ddpca {

namespace {

using Key = std::array<int64_t, 2>;  // {body, node}: the reference's std::vector<long> key
using csr::Trip;

constexpr double kSeneScale = 210.0e9;  // the semi-smooth Newton constant (MCONTACT.h:3647, 3673)

// general 4x4 / 3x3 inverse by Gauss-Jordan with partial pivoting (Eigen inverse(), row-major)
template <int N>
std::array<double, N * N> inverse(std::array<double, N * N> a) {
    std::array<double, N * N> r{};
    for (int i = 0; i < N; ++i) r[i * N + i] = 1.0;
    for (int c = 0; c < N; ++c) {
        int p = c;
        for (int i = c + 1; i < N; ++i)
            if (std::fabs(a[i * N + c]) > std::fabs(a[p * N + c])) p = i;
        if (a[p * N + c] == 0.0) throw std::runtime_error("LAGRANGE: singular block");
        if (p != c)
            for (int j = 0; j < N; ++j) {
                std::swap(a[p * N + j], a[c * N + j]);
                std::swap(r[p * N + j], r[c * N + j]);
            }
        const double d = 1.0 / a[c * N + c];
        for (int j = 0; j < N; ++j) {
            a[c * N + j] *= d;
            r[c * N + j] *= d;
        }
        for (int i = 0; i < N; ++i) {
            if (i == c) continue;
            const double f = a[i * N + c];
            if (f == 0.0) continue;
            for (int j = 0; j < N; ++j) {
                a[i * N + j] -= f * a[c * N + j];
                r[i * N + j] -= f * r[c * N + j];
            }
        }
    }
    return r;
}

// nodal frame from the averaged normal (MCONTACT.h:2990-3037): columns n, t1, t2
std::array<double, 9> frame(const double n[3]) {
    std::array<double, 9> f{};  // row-major f[3 * row + col]
    for (int a = 0; a < 3; ++a) f[3 * a] = n[a];
    const double d1x = n[0], d1y = n[1], d1z = n[2], e = 1.0e-14;
    if (std::fabs(d1y) < e) {
        f[3 * 1 + 1] = 1.0;
        if (std::fabs(d1x) < e) {
            f[3 * 0 + 2] = 1.0;
        } else if (std::fabs(d1z) < e) {
            f[3 * 2 + 2] = 1.0;
        } else {
            const double s = std::sqrt(d1z * d1z + d1x * d1x);
            f[3 * 0 + 2] = d1z / s;
            f[3 * 2 + 2] = -d1x / s;
        }
    } else if (std::fabs(d1z) < e) {
        f[3 * 2 + 1] = 1.0;
        if (std::fabs(d1x) < e) {
            f[3 * 0 + 2] = 1.0;
        } else {
            const double s = std::sqrt(d1y * d1y + d1x * d1x);
            f[3 * 0 + 2] = d1y / s;
            f[3 * 1 + 2] = -d1x / s;
        }
    } else {
        const double b2c2 = d1y * d1y + d1z * d1z;
        f[3 * 1 + 1] = d1z / std::sqrt(b2c2);
        f[3 * 2 + 1] = -d1y / std::sqrt(b2c2);
        const double abc = std::sqrt(b2c2 * b2c2 + (d1x * d1y) * (d1x * d1y) + (d1x * d1z) * (d1x * d1z));
        f[3 * 0 + 2] = b2c2 / abc;
        f[3 * 1 + 2] = (-d1x * d1y) / abc;
        f[3 * 2 + 2] = (-d1x * d1z) / abc;
    }
    const double c0[3] = {f[0], f[3], f[6]}, c1[3] = {f[1], f[4], f[7]}, c2[3] = {f[2], f[5], f[8]};
    const double x[3] = {c0[1] * c1[2] - c0[2] * c1[1], c0[2] * c1[0] - c0[0] * c1[2], c0[0] * c1[1] - c0[1] * c1[0]};
    if (x[0] * c2[0] + x[1] * c2[1] + x[2] * c2[2] < 0.0)
        for (int a = 0; a < 3; ++a) f[3 * a + 2] = -f[3 * a + 2];
    return f;
}

std::vector<double> segment(const std::vector<double>& v, int64_t o, int64_t n) {
    return std::vector<double>(v.begin() + o, v.begin() + o + n);
}

void axpy(std::vector<double>& y, double a, const std::vector<double>& x) {
    for (size_t i = 0; i < y.size(); ++i) y[i] += a * x[i];
}

}  // namespace

LagrangeResult run_lagrange(std::vector<LagrangeSub>& subs, std::vector<LagrangeItf>& itfs, int64_t max_newton,
                            const LagrangeSolve& solve) {
    const int64_t nsub = (int64_t)subs.size(), nint = (int64_t)itfs.size();
    if (nsub < 1) throw std::invalid_argument("LAGRANGE: no subdomains");
    const int nlev = subs[0].nlev;
    for (const auto& s : subs)
        if (s.nlev != nlev) throw std::invalid_argument("LAGRANGE: every subdomain needs the same number of levels");
    const int L = nlev - 1;
    for (const auto& f : itfs)
        for (int s = 0; s < 2; ++s)
            if (f.body[s] < 0 || f.body[s] >= nsub) throw std::invalid_argument("LAGRANGE: contact body out of range");
    // condensed offsets (baseReco, MCONTACT.h:2861-2868)
    std::vector<int64_t> base(nsub + 1, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) base[tv + 1] = base[tv] + subs[tv].nfree[L];
    const int64_t baseN = base[nsub];

    // ---- non-mortar side may not hold hanging nodes (MCONTACT.h:2870-2893)
    for (auto& f : itfs) {
        const LagrangeSub& g = subs[f.body[0]];
        std::vector<LagrangeIp> keep;
        for (const auto& q : f.ips) {
            bool ok = true;
            for (int k = 0; k < 4; ++k) {
                const int64_t n = q.node[0][k];
                if (n < 0 || n >= g.nall) throw std::invalid_argument("LAGRANGE: integration point node out of range");
                if (!g.hanging.empty() && g.hanging[n]) ok = false;
            }
            if (ok) keep.push_back(q);
        }
        f.ips.swap(keep);
    }
    // ---- dual basis, boundary-consistent (MCONTACT.h:2894-2947)
    for (auto& f : itfs) {
        std::map<std::array<int64_t, 4>, std::vector<int64_t>> segm;
        for (int64_t i = 0; i < (int64_t)f.ips.size(); ++i) {
            const auto& n = f.ips[i].node[0];
            segm[{n[0], n[1], n[2], n[3]}].push_back(i);
        }
        for (const auto& s : segm) {
            std::array<double, 16> D{}, M{};
            for (int64_t i : s.second) {
                const LagrangeIp& q = f.ips[i];
                for (int a = 0; a < 4; ++a) {
                    D[5 * a] += q.w * q.shap[0][a];
                    for (int b = 0; b < 4; ++b) M[4 * a + b] += q.w * (q.shap[0][a] * q.shap[0][b]);
                }
            }
            const auto Mi = inverse<4>(M);
            std::array<double, 16> A{};
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) A[4 * a + b] = D[5 * a] * Mi[4 * a + b];
            for (int64_t i : s.second) {
                LagrangeIp& q = f.ips[i];
                for (int a = 0; a < 4; ++a) {
                    double v = 0.0;
                    for (int b = 0; b < 4; ++b) v += A[4 * a + b] * q.shap[0][b];
                    q.dual[a] = v;
                }
            }
        }
    }
    // ---- non-mortar nodes: status and number (MCONTACT.h:2950-2967)
    std::vector<std::map<Key, int64_t>> stat(nint), numb(nint);
    for (int64_t ts = 0; ts < nint; ++ts) {
        const int64_t st = itfs[ts].fric == 0.0 ? 1 : 2;
        for (const auto& q : itfs[ts].ips)
            for (int k = 0; k < 4; ++k) {
                const Key key{itfs[ts].body[0], q.node[0][k]};
                stat[ts].emplace(key, st);
                const int64_t sz = (int64_t)numb[ts].size();
                numb[ts].emplace(key, sz);
            }
    }
    // ---- nodal frames over all interfaces (MCONTACT.h:2968-3038)
    std::map<Key, std::array<double, 9>> nota;
    {
        std::map<Key, std::array<double, 4>> acc;  // weighted normal sum, weight
        for (int64_t ts = 0; ts < nint; ++ts)
            for (const auto& kv : numb[ts]) acc.emplace(kv.first, std::array<double, 4>{0, 0, 0, 0});
        for (int64_t ts = 0; ts < nint; ++ts)
            for (const auto& q : itfs[ts].ips)
                for (int k = 0; k < 4; ++k) {
                    auto& a = acc[{itfs[ts].body[0], q.node[0][k]}];
                    for (int c = 0; c < 3; ++c) a[c] = a[c] + q.w * q.basis[0][c];
                    a[3] += q.w;
                }
        for (const auto& kv : acc) {
            const double n[3] = {kv.second[0] / kv.second[3], kv.second[1] / kv.second[3], kv.second[2] / kv.second[3]};
            nota[kv.first] = frame(n);
        }
    }
    // ---- normal-tangential mortar coupling notaMoco[ts][tv] (MCONTACT.h:3040-3109)
    std::vector<std::array<Csr, 2>> moco(nint);
    for (int64_t ts = 0; ts < nint; ++ts) {
        const LagrangeItf& f = itfs[ts];
        const int64_t nr = 3 * (int64_t)numb[ts].size();
        for (int tv = 0; tv < 2; ++tv) {
            const LagrangeSub& g = subs[f.body[tv]];
            std::vector<Trip> t;
            for (const auto& q : f.ips)
                for (int tj = 0; tj < 4; ++tj) {
                    const int64_t num = numb[ts].at({f.body[0], q.node[0][tj]});
                    for (int tk = 0; tk < 3; ++tk)
                        for (int tm = 0; tm < 4; ++tm) {
                            const int64_t nd = q.node[tv][tm];
                            if (nd < 0 || nd >= g.nall) throw std::invalid_argument("LAGRANGE: integration point node out of range");
                            for (int tn = 0; tn < 3; ++tn) {
                                if (tv == 0 && 3 * tj + tk != 3 * tm + tn) continue;
                                const double v = tk == tn ? q.w * q.dual[tj] * q.shap[tv][tm] : 0.0;
                                t.push_back({3 * num + tk, 3 * nd + tn, v});
                            }
                        }
                }
            Csr m = csr::from_triplets(nr, 3 * g.nall, t);
            m = csr::multiply(m, g.G);
            if (tv == 1) m = csr::scale(m, -1.0);
            std::vector<Trip> nt;
            for (const auto& kv : numb[ts]) {
                const auto& F = nota.at(kv.first);
                for (int tj = 0; tj < 3; ++tj)
                    for (int tk = 0; tk < 3; ++tk) nt.push_back({3 * kv.second + tj, 3 * kv.second + tk, F[3 * tk + tj]});
            }
            moco[ts][tv] = csr::multiply(csr::from_triplets(nr, nr, nt), m);
        }
    }
    // ---- initial gap (MCONTACT.h:3111-3124)
    std::vector<std::vector<double>> gap0(nint);
    for (int64_t ts = 0; ts < nint; ++ts) {
        gap0[ts].assign(3 * numb[ts].size(), 0.0);
        for (const auto& q : itfs[ts].ips)
            for (int tj = 0; tj < 4; ++tj)
                gap0[ts][3 * numb[ts].at({itfs[ts].body[0], q.node[0][tj]})] += q.w * q.dual[tj] * q.gap;
    }
    // ---- the saddle-point system [K B^T; B 0] (MCONTACT.h:3126-3178)
    std::vector<int64_t> acin(nint + 1, 0);
    for (int64_t ts = 0; ts < nint; ++ts) acin[ts + 1] = acin[ts] + (int64_t)numb[ts].size();
    const int64_t origN = baseN + 3 * acin[nint];
    std::vector<Trip> orig;
    for (int64_t tv = 0; tv < nsub; ++tv) csr::append(orig, subs[tv].K[L], base[tv], base[tv]);
    for (int64_t ts = 0; ts < nint; ++ts)
        for (int tv = 0; tv < 2; ++tv) {
            const Csr& m = moco[ts][tv];
            const int64_t rb = baseN + 3 * acin[ts], cb = base[itfs[ts].body[tv]];
            for (int64_t r = 0; r < m.nrow; ++r)
                for (int64_t k = m.ptr[r]; k < m.ptr[r + 1]; ++k) {
                    orig.push_back({rb + r, cb + m.col[k], m.val[k]});
                    orig.push_back({cb + m.col[k], rb + r, m.val[k]});
                }
        }
    std::vector<double> origF(origN, 0.0);
    for (int64_t tv = 0; tv < nsub; ++tv) std::copy(subs[tv].consForc.begin(), subs[tv].consForc.end(), origF.begin() + base[tv]);
    for (int64_t ts = 0; ts < nint; ++ts) std::copy(gap0[ts].begin(), gap0[ts].end(), origF.begin() + baseN + 3 * acin[ts]);

    // ---- semi-smooth Newton (MCONTACT.h:3180-3699)
    LagrangeResult res;
    std::vector<std::vector<double>> wedi(nint), lagr(nint);
    std::vector<std::map<Key, int64_t>> hist = stat;
    for (int64_t tc = 0;; ++tc) {
        if (tc >= max_newton) break;
        // SlidCoup: Coulomb terms of sliding nodes (MCONTACT.h:3186-3240)
        std::vector<Trip> slid = orig;
        for (int64_t ts = 0; ts < nint; ++ts) {
            const double mu = itfs[ts].fric;
            if (mu <= 0.0) continue;
            const int64_t nr = 3 * (int64_t)numb[ts].size();
            std::vector<Trip> t;
            for (const auto& kv : numb[ts]) {
                if (stat[ts].at(kv.first) != 1) continue;
                const int64_t h = hist[ts].at(kv.first);
                const int64_t n = kv.second;
                double c0, c1;
                if (h == 1 || h == 0) {
                    c0 = wedi[ts][3 * n + 1];
                    c1 = wedi[ts][3 * n + 2];
                } else {
                    c0 = lagr[ts][3 * n + 1];
                    c1 = lagr[ts][3 * n + 2];
                }
                const double tt = std::sqrt(c0 * c0 + c1 * c1);
                t.push_back({3 * n, 3 * n + 1, c0 / tt});
                t.push_back({3 * n, 3 * n + 2, c1 / tt});
            }
            const Csr S = csr::scale(csr::from_triplets(nr, nr, t), mu);
            for (int tv = 0; tv < 2; ++tv) {
                const Csr m = csr::multiply(S, moco[ts][tv]);
                const int64_t rb = baseN + 3 * acin[ts], cb = base[itfs[ts].body[tv]];
                for (int64_t r = 0; r < m.nrow; ++r)
                    for (int64_t k = m.ptr[r]; k < m.ptr[r + 1]; ++k) slid.push_back({cb + m.col[k], rb + r, m.val[k]});
            }
        }
        const Csr slidCoup = csr::from_triplets(origN, origN, slid);
        slid.clear();
        // RealCoup: active multiplier components (MCONTACT.h:3242-3279)
        std::vector<Trip> rl;
        for (int64_t i = 0; i < baseN; ++i) rl.push_back({i, i, 1.0});
        int64_t cons = 0;
        for (int64_t ts = 0; ts < nint; ++ts) {
            const int64_t tb = baseN + 3 * acin[ts];
            for (const auto& kv : numb[ts]) {
                const int64_t s = stat[ts].at(kv.first);
                if (s == 1) rl.push_back({baseN + cons++, tb + 3 * kv.second, 1.0});
                else if (s == 2)
                    for (int d = 0; d < 3; ++d) rl.push_back({baseN + cons++, tb + 3 * kv.second + d, 1.0});
            }
        }
        const int64_t totN = baseN + cons;
        const Csr R = csr::from_triplets(totN, origN, rl);
        const Csr Rt = csr::transpose(R);
        const Csr realCoup = csr::multiply(csr::multiply(R, slidCoup), Rt);
        const std::vector<double> realF = csr::apply(R, origF);
        // SoluCoup: condensed non-mortar dofs (MCONTACT.h:3281-3349)
        std::vector<std::vector<std::set<int64_t>>> cond(nint);
        cons = 0;
        for (int64_t ts = 0; ts < nint; ++ts) {
            cond[ts].resize(numb[ts].size());
            const int64_t lo = base[itfs[ts].body[0]], hi = base[itfs[ts].body[0] + 1];
            for (const auto& kv : numb[ts]) {
                const int64_t s = stat[ts].at(kv.first);
                if (s == 1) {
                    const int64_t row = baseN + cons;
                    double mx = -1.0;
                    int64_t pick = -1;
                    for (int64_t k = realCoup.ptr[row]; k < realCoup.ptr[row + 1]; ++k)
                        if (lo <= realCoup.col[k] && realCoup.col[k] < hi && std::fabs(realCoup.val[k]) > mx) {
                            mx = std::fabs(realCoup.val[k]);
                            pick = realCoup.col[k];
                        }
                    if (pick < 0) throw std::runtime_error("LAGRANGE: a sliding node has no non-mortar dof (ERROR 1, MCONTACT.h:3305)");
                    cond[ts][kv.second].insert(pick);
                    ++cons;
                } else if (s == 2) {
                    for (int d = 0; d < 3; ++d) {
                        const int64_t row = baseN + cons;
                        for (int64_t k = realCoup.ptr[row]; k < realCoup.ptr[row + 1]; ++k)
                            if (lo <= realCoup.col[k] && realCoup.col[k] < hi) cond[ts][kv.second].insert(realCoup.col[k]);
                        ++cons;
                    }
                    if (cond[ts][kv.second].size() != 3)
                        throw std::runtime_error("LAGRANGE: a sticking node does not couple to exactly 3 non-mortar dofs (ERROR 2, MCONTACT.h:3320)");
                }
            }
        }
        std::vector<Trip> sl;
        std::vector<uint8_t> condFlag(totN, 0);
        cons = 0;
        for (int64_t ts = 0; ts < nint; ++ts)
            for (const auto& kv : numb[ts])
                for (int64_t d : cond[ts][kv.second]) {
                    sl.push_back({d, cons++, 1.0});
                    condFlag[d] = 1;
                }
        for (int64_t i = 0; i < totN; ++i)
            if (!condFlag[i]) sl.push_back({i, cons++, 1.0});
        const Csr S = csr::from_triplets(totN, totN, sl);
        const Csr St = csr::transpose(S);
        const Csr soluCoup = csr::multiply(csr::multiply(St, realCoup), S);
        const std::vector<double> soluF = csr::apply(St, realF);
        // block elimination (MCONTACT.h:3351-3416)
        const int64_t n0 = totN - baseN, n1 = totN - 2 * n0;
        const Csr K00 = csr::block(soluCoup, 0, 0, n0, n0), K01 = csr::block(soluCoup, 0, n0, n0, n1);
        const Csr K10 = csr::block(soluCoup, n0, 0, n1, n0), K11 = csr::block(soluCoup, n0, n0, n1, n1);
        const Csr T0 = csr::block(soluCoup, baseN, 0, n0, n0), T1 = csr::block(soluCoup, baseN, n0, n0, n1);
        const Csr T0f = csr::block(soluCoup, 0, baseN, n0, n0), T1f = csr::block(soluCoup, n0, baseN, n1, n0);
        const std::vector<double> F0 = segment(soluF, 0, n0), F1 = segment(soluF, n0, baseN - n0), g0 = segment(soluF, baseN, n0);
        std::vector<Trip> i0, i1;
        cons = 0;
        for (int64_t ts = 0; ts < nint; ++ts)
            for (const auto& kv : numb[ts]) {
                const int64_t s = stat[ts].at(kv.first);
                if (s == 1) {
                    i0.push_back({cons, cons, 1.0 / csr::coeff(T0, cons, cons)});
                    i1.push_back({cons, cons, 1.0 / csr::coeff(T0f, cons, cons)});
                    ++cons;
                } else if (s == 2) {
                    std::array<double, 9> a{}, b{};
                    for (int r = 0; r < 3; ++r)
                        for (int c = 0; c < 3; ++c) {
                            a[3 * r + c] = csr::coeff(T0, cons + r, cons + c);
                            b[3 * r + c] = csr::coeff(T0f, cons + r, cons + c);
                        }
                    const auto ai = inverse<3>(a), bi = inverse<3>(b);
                    for (int r = 0; r < 3; ++r)
                        for (int c = 0; c < 3; ++c) {
                            i0.push_back({cons + r, cons + c, ai[3 * r + c]});
                            i1.push_back({cons + r, cons + c, bi[3 * r + c]});
                        }
                    cons += 3;
                }
            }
        const Csr iT0 = csr::from_triplets(n0, n0, i0), iT0f = csr::from_triplets(n0, n0, i1);
        const Csr iT0_T1 = csr::multiply(iT0, T1);                      // inveT_0 T_1
        const Csr T1f_iT0f = csr::multiply(T1f, iT0f);                  // T_1f inveT_0f
        const Csr K10_iT0 = csr::multiply(K10, iT0);
        const Csr T1f_iT0f_K00 = csr::multiply(T1f_iT0f, K00);
        const Csr T1f_iT0f_K00_iT0 = csr::multiply(T1f_iT0f_K00, iT0);
        Csr K = csr::add(K11, csr::multiply(K10_iT0, T1), 1.0, -1.0);
        K = csr::add(K, csr::multiply(T1f_iT0f, K01), 1.0, -1.0);
        K = csr::add(K, csr::multiply(T1f_iT0f_K00_iT0, T1));
        std::vector<double> F = F1;
        axpy(F, -1.0, csr::apply(K10_iT0, g0));
        axpy(F, -1.0, csr::apply(T1f_iT0f, F0));
        axpy(F, 1.0, csr::apply(T1f_iT0f_K00_iT0, g0));
        // the hierarchy of the condensed system (precType 1, MCONTACT.h:3419-3561)
        LagrangeSystem sys;
        sys.K.assign(nlev, Csr());
        sys.dofs.assign(nlev, {});
        for (int l = 0; l < nlev; ++l)
            for (int64_t tv = 0; tv < nsub; ++tv)
                for (int64_t ti = 0; ti < subs[tv].nfree[l]; ++ti)
                    if (!condFlag[base[tv] + ti]) sys.dofs[l].push_back({(int32_t)tv, (int32_t)ti});
        if ((int64_t)sys.dofs[L].size() != n1) throw std::logic_error("LAGRANGE: condensed dof count");
        sys.K[L] = K;
        if (nlev > 1) {
            std::vector<Csr> origProl(L);
            for (int tl = 0; tl < L; ++tl) {
                std::vector<Trip> t;
                int64_t ro = 0, co = 0;
                for (int64_t tv = 0; tv < nsub; ++tv) {
                    csr::append(t, subs[tv].P[tl], ro, co);
                    ro += subs[tv].P[tl].nrow;
                    co += subs[tv].P[tl].ncol;
                }
                origProl[tl] = csr::from_triplets(ro, co, t);
            }
            const Csr reseMaxi = csr::block(St, n0, 0, baseN - n0, baseN);
            std::vector<Csr> condProl(nlev);
            condProl[L] = csr::multiply(csr::block(S, 0, 0, baseN, n0), csr::scale(csr::multiply(iT0_T1, reseMaxi), -1.0));
            for (int tl = L - 1; tl >= 0; --tl) condProl[tl] = csr::multiply(condProl[tl + 1], origProl[tl]);
            sys.P.assign(L, Csr());
            for (int tl = L - 1; tl >= 0; --tl) {
                // reseProl[tl]: condensed coarse dofs replaced by their condProl rows
                std::vector<Trip> t;
                int64_t co = 0;
                for (int64_t tv = 0; tv < nsub; ++tv) {
                    for (int64_t ti = 0; ti < subs[tv].nfree[tl]; ++ti) {
                        const int64_t real = base[tv] + ti;
                        if (!condFlag[real]) {
                            t.push_back({co + ti, co + ti, 1.0});
                        } else {
                            const Csr& C = condProl[tl];
                            for (int64_t k = C.ptr[real]; k < C.ptr[real + 1]; ++k) t.push_back({co + ti, C.col[k], C.val[k]});
                        }
                    }
                    co += subs[tv].nfree[tl];
                }
                const Csr rese = csr::from_triplets(co, co, t);
                const Csr P0 = csr::multiply(origProl[tl], rese);
                std::vector<int64_t> br(P0.nrow, -1), bc(P0.ncol, -1);
                int64_t nr = 0, nc = 0, ro = 0, cc = 0;
                for (int64_t tv = 0; tv < nsub; ++tv) {
                    const Csr& Pt = subs[tv].P[tl];
                    for (int64_t ti = 0; ti < Pt.nrow; ++ti)
                        if (!condFlag[base[tv] + ti]) {
                            br[ro + ti] = nr++;
                            if (ti < Pt.ncol) bc[cc + ti] = nc++;
                        }
                    ro += Pt.nrow;
                    cc += Pt.ncol;
                }
                std::vector<Trip> pt;
                for (int64_t r = 0; r < P0.nrow; ++r) {
                    if (br[r] < 0) continue;
                    for (int64_t k = P0.ptr[r]; k < P0.ptr[r + 1]; ++k)
                        if (bc[P0.col[k]] >= 0) pt.push_back({br[r], bc[P0.col[k]], P0.val[k]});
                }
                sys.P[tl] = csr::from_triplets(nr, nc, pt);
            }
            for (int tl = L - 1; tl >= 0; --tl)
                sys.K[tl] = csr::multiply(csr::multiply(csr::transpose(sys.P[tl]), sys.K[tl + 1]), sys.P[tl]);
        }
        sys.F = F;
        std::vector<double> U1;
        res.solver_iters.push_back(solve(sys, U1));
        if ((int64_t)U1.size() != n1) throw std::logic_error("LAGRANGE: solver returned a wrong-sized vector");
        // recover U_0 and the multipliers (MCONTACT.h:3580-3589)
        std::vector<double> U0 = csr::apply(iT0, g0);
        axpy(U0, -1.0, csr::apply(iT0_T1, U1));
        const Csr iT0f_K00 = csr::multiply(iT0f, K00);
        const Csr iT0f_K00_iT0 = csr::multiply(iT0f_K00, iT0);
        std::vector<double> lamb = csr::apply(iT0f, F0);
        axpy(lamb, -1.0, csr::apply(iT0f_K00_iT0, g0));
        axpy(lamb, -1.0, csr::apply(csr::multiply(iT0f, K01), U1));
        axpy(lamb, 1.0, csr::apply(csr::multiply(iT0f_K00_iT0, T1), U1));
        std::vector<double> sd(totN, 0.0);
        std::copy(U0.begin(), U0.end(), sd.begin());
        std::copy(U1.begin(), U1.end(), sd.begin() + n0);
        std::copy(lamb.begin(), lamb.end(), sd.begin() + baseN);
        const std::vector<double> slidDisp = csr::apply(Rt, csr::apply(S, sd));
        for (int64_t ts = 0; ts < nint; ++ts) {
            wedi[ts] = gap0[ts];
            for (double& v : wedi[ts]) v = -v;
            for (int tv = 0; tv < 2; ++tv) {
                const int64_t b = itfs[ts].body[tv];
                axpy(wedi[ts], 1.0, csr::apply(moco[ts][tv], segment(slidDisp, base[b], base[b + 1] - base[b])));
            }
            lagr[ts] = segment(slidDisp, baseN + 3 * acin[ts], 3 * (acin[ts + 1] - acin[ts]));
        }
        res.u.assign(nsub, {});
        for (int64_t tv = 0; tv < nsub; ++tv) res.u[tv] = segment(slidDisp, base[tv], base[tv + 1] - base[tv]);
        res.node.assign(nint, {});
        res.status.assign(nint, {});
        res.lambda.assign(nint, {});
        res.wedi.assign(nint, {});
        for (int64_t ts = 0; ts < nint; ++ts)
            for (const auto& kv : numb[ts]) {
                res.node[ts].push_back(kv.first[1]);
                res.status[ts].push_back(stat[ts].at(kv.first));
                for (int d = 0; d < 3; ++d) {
                    res.lambda[ts].push_back(lagr[ts][3 * kv.second + d]);
                    res.wedi[ts].push_back(wedi[ts][3 * kv.second + d]);
                }
            }
        res.newton = tc;
        // active-set update (MCONTACT.h:3637-3698)
        hist = stat;
        int64_t changes = 0;
        for (int64_t ts = 0; ts < nint; ++ts) {
            const double mu = itfs[ts].fric;
            if (mu < 0.0) continue;
            for (const auto& kv : numb[ts]) {
                int64_t& s = stat[ts].at(kv.first);
                const int64_t n = kv.second;
                const double sn = lagr[ts][3 * n] + kSeneScale * wedi[ts][3 * n];
                if (sn <= 0.0) {
                    if (s != 0) ++changes;
                    s = 0;
                    continue;
                }
                if (mu == 0.0) {
                    if (s != 1) ++changes;
                    s = 1;
                    continue;
                }
                double st;
                if (s == 2) {
                    st = std::sqrt(lagr[ts][3 * n + 1] * lagr[ts][3 * n + 1] + lagr[ts][3 * n + 2] * lagr[ts][3 * n + 2]);
                } else {
                    st = mu * lagr[ts][3 * n] +
                         kSeneScale * std::sqrt(wedi[ts][3 * n + 1] * wedi[ts][3 * n + 1] + wedi[ts][3 * n + 2] * wedi[ts][3 * n + 2]);
                }
                const int64_t ns = st >= mu * sn ? 1 : 2;
                if (s != ns) ++changes;
                s = ns;
            }
        }
        res.changes.push_back(changes);
        if (changes == 0) {
            res.converged = true;
            break;
        }
    }
    return res;
}

}  // namespace ddpca

// Host restatement of MCONTACT::ESTABLISH operator assembly (see mcontact.hpp).
#include "mcontact.hpp"

#include <algorithm>
#include <cmath>
#include <map>
#include <stdexcept>
#include <unordered_map>

namespace ddpca {

namespace {

struct Trip {
    int64_t r, c;
    double v;
};

// Triplets -> CSR, duplicates summed (Eigen setFromTriplets semantics).
Csr from_triplets(int64_t nrow, int64_t ncol, std::vector<Trip>& t) {
    std::stable_sort(t.begin(), t.end(), [](const Trip& a, const Trip& b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
    Csr m;
    m.nrow = nrow;
    m.ncol = ncol;
    m.ptr.assign(nrow + 1, 0);
    for (size_t i = 0; i < t.size();) {
        size_t j = i;
        double s = 0.0;
        while (j < t.size() && t[j].r == t[i].r && t[j].c == t[i].c) s += t[j++].v;
        m.col.push_back((int32_t)t[i].c);
        m.val.push_back(s);
        m.ptr[t[i].r + 1]++;
        i = j;
    }
    for (int64_t r = 0; r < nrow; ++r) m.ptr[r + 1] += m.ptr[r];
    return m;
}

}  // namespace

void Interface::BUILD(const MULTIGRID& g0, const MULTIGRID& g1) {
    const int C = comp();
    const int64_t nip = (int64_t)ip.size();
    const MULTIGRID* g[2] = {&g0, &g1};
    const double pen[3] = {penN, penF, penF};
    for (int s = 0; s < 2; ++s) {
        std::unordered_map<int64_t, int64_t> nc;
        nodeCont[s].clear();
        for (const auto& p : ip)
            for (int k = 0; k < 4; ++k)
                if (nc.emplace(p.node[s][k], (int64_t)nc.size()).second) nodeCont[s].push_back(p.node[s][k]);
        const int64_t nn = g[s]->numNodes();
        const int64_t mc = C * (int64_t)nodeCont[s].size();
        std::vector<Trip> tM, tT, tTp, tI, tIp, tL, tD, tII;
        for (int64_t q = 0; q < nip; ++q) {
            const IntegralPoint& p = ip[q];
            const double* M = p.shap[s];
            // T: rows n, t1, t2 (C == 3); n only (C == 1)
            double T[3][3];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) T[a][b] = p.basis[a][b];
            // G = T^T T, GP = T^T P T, GPi = T^T P^-1 T (3x3 nodal-space couplings)
            double G[3][3], GP[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double a = 0, b = 0;
                    for (int m = 0; m < C; ++m) {
                        a += T[m][i] * T[m][j];
                        b += T[m][i] * pen[m] * T[m][j];
                    }
                    G[i][j] = a;
                    GP[i][j] = b;
                }
            for (int a = 0; a < 4; ++a) {
                const int64_t na = p.node[s][a], ca = nc.at(na);
                for (int b = 0; b < 4; ++b) {
                    const int64_t nb = p.node[s][b], cb = nc.at(nb);
                    const double mm = p.w * M[a] * M[b];
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j) tM.push_back({3 * na + i, 3 * nb + j, mm * GP[i][j]});
                    if (C == 1) {
                        for (int i = 0; i < 3; ++i) {
                            tT.push_back({3 * na + i, cb, p.w * M[a] * T[0][i] * M[b]});
                            tTp.push_back({3 * na + i, cb, penN * (p.w * M[a] * T[0][i] * M[b])});
                        }
                        tI.push_back({ca, cb, mm});
                        tIp.push_back({ca, cb, mm * penN});
                    } else {
                        for (int i = 0; i < 3; ++i)
                            for (int j = 0; j < 3; ++j) {
                                tT.push_back({3 * na + i, 3 * cb + j, mm * G[i][j]});
                                tTp.push_back({3 * na + i, 3 * cb + j, mm * GP[i][j]});
                                tI.push_back({3 * ca + i, 3 * cb + j, mm * G[i][j]});
                                tIp.push_back({3 * ca + i, 3 * cb + j, mm * GP[i][j]});
                            }
                    }
                }
                // inpoLagr, inpoDisp (rows: ip components), inteInpo (rows: contact dofs)
                const double sgn = (s == 0) ? -1.0 : 1.0;
                for (int m = 0; m < C; ++m)
                    for (int k = 0; k < 3; ++k) {
                        if (C == 1) {
                            tD.push_back({q, 3 * na + k, T[0][k] * M[a]});
                        } else {
                            tL.push_back({3 * q + m, 3 * ca + k, T[m][k] * M[a]});
                            tD.push_back({3 * q + m, 3 * na + k, T[m][k] * M[a]});
                            tII.push_back({3 * ca + k, 3 * q + m, sgn * (p.w * M[a] * T[m][k])});
                        }
                    }
                if (C == 1) {
                    tL.push_back({q, ca, M[a]});
                    tII.push_back({ca, q, sgn * (p.w * M[a])});
                }
            }
        }
        systMass[s] = from_triplets(3 * nn, 3 * nn, tM);
        systTran[s] = from_triplets(3 * nn, mc, tT);
        systTran_pena[s] = from_triplets(3 * nn, mc, tTp);
        inteMass[s] = from_triplets(mc, mc, tI);
        inteMass_pena[s] = from_triplets(mc, mc, tIp);
        inpoLagr[s] = from_triplets(C * nip, mc, tL);
        inpoDisp[s] = from_triplets(C * nip, 3 * nn, tD);
        inteInpo[s] = from_triplets(mc, C * nip, tII);
    }
    inpoNgap.assign(C * nip, 0.0);
    pemaDiag.assign(C * nip, 0.0);
    for (int64_t q = 0; q < nip; ++q) {
        inpoNgap[C * q] = ip[q].gap;
        for (int m = 0; m < C; ++m) pemaDiag[C * q + m] = pen[m];
    }
    for (int s = 0; s < 2; ++s) {
        pemaInpo_r[s] = inpoDisp[s];
        for (int64_t r = 0; r < pemaInpo_r[s].nrow; ++r)
            for (int64_t k = pemaInpo_r[s].ptr[r]; k < pemaInpo_r[s].ptr[r + 1]; ++k) pemaInpo_r[s].val[k] *= pemaDiag[r];
    }
}

void MCONTACT::ESTABLISH() {
    for (auto& itf : searCont) itf.BUILD(multGrid[itf.body[0]], multGrid[itf.body[1]]);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tv = 0; tv < (int64_t)multGrid.size(); ++tv) {
        MULTIGRID& g = multGrid[tv];
        g.TRANSFER();
        g.STIF_MATR();
        for (const auto& itf : searCont)
            for (int s = 0; s < 2; ++s)
                if (itf.body[s] == tv) g.ADD_NODAL(itf.systMass[s]);
        g.CONSTRAINT();
    }
}

double MCONTACT::GET_CHAR_LENG() const {
    double v = 0.0;
    for (const auto& g : multGrid) v += g.GET_VOLUME();
    v /= (double)multGrid.size();
    return std::pow(v, 0.333333333333333333);
}

// ------------------------------------------------------------------------------------------
void conforming_face_ips(const MULTIGRID& gm, const int64_t mast[4], const MULTIGRID& gs,
                         const int64_t slav[4], std::vector<IntegralPoint>& out) {
    static const double nacoCorn[4][2] = {{-1, -1}, {1, -1}, {1, 1}, {-1, 1}};
    double X[4][3], Y[4][3];
    for (int k = 0; k < 4; ++k)
        for (int a = 0; a < 3; ++a) {
            X[k][a] = gm.nodeCoor[mast[k]][a];
            Y[k][a] = gs.nodeCoor[slav[k]][a];
        }
    // slave corners in master natural coordinates (coincident faces: match by position)
    double sxi[4][2];
    for (int k = 0; k < 4; ++k) {
        int hit = -1;
        for (int m = 0; m < 4; ++m) {
            double d = 0;
            for (int a = 0; a < 3; ++a) d += (Y[k][a] - X[m][a]) * (Y[k][a] - X[m][a]);
            if (d < 1e-20) hit = m;
        }
        if (hit < 0) throw std::runtime_error("conforming_face_ips: faces do not coincide");
        sxi[k][0] = nacoCorn[hit][0];
        sxi[k][1] = nacoCorn[hit][1];
    }
    // polygon = master square, vertices sorted by angle about the centroid: (-1,-1),(1,-1),(1,1),(-1,1)
    const double poly[4][2] = {{-1, -1}, {1, -1}, {1, 1}, {-1, 1}};
    const double g = std::sqrt(1.0 / 3.0);
    const double gl[2] = {-g, g};
    for (int t = 0; t < 4; ++t) {
        const double* v1 = poly[t];
        const double* v2 = poly[(t + 1) % 4];
        const double area = std::abs((v1[0] - 0.0) * (v2[1] - 0.0) - (v1[1] - 0.0) * (v2[0] - 0.0)) / 2.0;
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) {
                // PREP.h:336-361 triangle rule, CSEARCH.h:468-483
                const double b0 = (1.0 + gl[i]) / 2.0;
                const double b1 = (1.0 - gl[i]) * (1.0 + gl[j]) / 4.0;
                const double b2 = 1.0 - b0 - b1;
                const double wq = (1.0 - gl[i]) / 8.0;
                const double xi = b0 * 0.0 + b1 * v1[0] + b2 * v2[0];
                const double et = b0 * 0.0 + b1 * v1[1] + b2 * v2[1];
                IntegralPoint p;
                double dx[3] = {0, 0, 0}, de[3] = {0, 0, 0};
                for (int k = 0; k < 4; ++k) {
                    p.node[0][k] = mast[k];
                    p.node[1][k] = slav[k];
                    p.shap[0][k] = (1.0 + nacoCorn[k][0] * xi) * (1.0 + nacoCorn[k][1] * et) / 4.0;
                    for (int a = 0; a < 3; ++a) {
                        dx[a] += X[k][a] * (nacoCorn[k][0] / 4.0 + nacoCorn[k][0] * nacoCorn[k][1] * et / 4.0);
                        de[a] += X[k][a] * (nacoCorn[k][1] / 4.0 + nacoCorn[k][0] * nacoCorn[k][1] * xi / 4.0);
                    }
                }
                // slave shape functions: the projected point coincides with the master point,
                // so slave corner k (sitting on master corner m) carries master weight m
                for (int k = 0; k < 4; ++k) {
                    int m = 0;
                    for (; m < 4; ++m)
                        if (nacoCorn[m][0] == sxi[k][0] && nacoCorn[m][1] == sxi[k][1]) break;
                    p.shap[1][k] = p.shap[0][m];
                }
                double n[3] = {dx[1] * de[2] - dx[2] * de[1], dx[2] * de[0] - dx[0] * de[2], dx[0] * de[1] - dx[1] * de[0]};
                const double jac = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                const double lx = std::sqrt(dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2]);
                const double le = std::sqrt(de[0] * de[0] + de[1] * de[1] + de[2] * de[2]);
                for (int a = 0; a < 3; ++a) {
                    p.basis[0][a] = n[a] / jac;
                    p.basis[1][a] = dx[a] / lx;
                    p.basis[2][a] = de[a] / le;
                }
                p.gap = 0.0;
                p.w = 2.0 * area * wq * jac;
                out.push_back(p);
            }
    }
}

}  // namespace ddpca

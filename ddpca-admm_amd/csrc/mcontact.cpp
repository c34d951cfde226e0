// Host restatement of MCONTACT::ESTABLISH operator assembly (see mcontact.hpp).
#include "mcontact.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <numeric>
#include <stdexcept>
#include <unordered_map>

namespace ddpca {


void Interface::BUILD(const MULTIGRID& g0, const MULTIGRID& g1) {
    const int C = comp();
    const int64_t nip = (int64_t)ip.size();
    const MULTIGRID* g[2] = {&g0, &g1};
    const double pen[3] = {penN, penF, penF};
#pragma omp parallel for schedule(static, 1) num_threads(2)
    for (int s = 0; s < 2; ++s) {
        std::unordered_map<int64_t, int64_t> nc;
        nodeCont[s].clear();
        for (const auto& p : ip)
            for (int k = 0; k < 4; ++k)
                if (nc.emplace(p.node[s][k], (int64_t)nc.size()).second) nodeCont[s].push_back(p.node[s][k]);
        const int64_t nn = g[s]->numNodes();
        const int64_t ncn = (int64_t)nodeCont[s].size();
        const int64_t mc = C * ncn;
        // ---- contact-node pairs coupled by an integration point (node-block sparsity)
        std::vector<int32_t> ipc(4 * nip);
        std::vector<std::vector<int32_t>> part(ncn);
        for (int64_t q = 0; q < nip; ++q)
            for (int a = 0; a < 4; ++a) ipc[4 * q + a] = (int32_t)nc.at(ip[q].node[s][a]);
        for (int64_t q = 0; q < nip; ++q)
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) part[ipc[4 * q + a]].push_back(ipc[4 * q + b]);
        std::vector<int64_t> pptr(ncn + 1, 0);
        for (int64_t a = 0; a < ncn; ++a) {
            std::sort(part[a].begin(), part[a].end());
            part[a].erase(std::unique(part[a].begin(), part[a].end()), part[a].end());
            pptr[a + 1] = pptr[a] + (int64_t)part[a].size();
        }
        // per pair: sum_q w M_a M_b (T^T P T), sum_q w M_a M_b (T^T T) [C = 3] or
        // sum_q w M_a M_b n (3) and sum_q w M_a M_b [C = 1]   (MCONTACT.h:241-568)
        std::vector<double> aGP(9 * pptr[ncn], 0.0), aG(9 * pptr[ncn], 0.0), aN(3 * pptr[ncn], 0.0),
            aM(pptr[ncn], 0.0);
        for (int64_t q = 0; q < nip; ++q) {
            const IntegralPoint& p = ip[q];
            const double* M = p.shap[s];
            double GP[3][3], G[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double x = 0, y = 0;
                    for (int m = 0; m < C; ++m) {
                        x += p.basis[m][i] * p.basis[m][j];
                        y += p.basis[m][i] * pen[m] * p.basis[m][j];
                    }
                    G[i][j] = x;
                    GP[i][j] = y;
                }
            for (int a = 0; a < 4; ++a) {
                const int32_t ca = ipc[4 * q + a];
                for (int b = 0; b < 4; ++b) {
                    const int32_t cb = ipc[4 * q + b];
                    const int64_t k = pptr[ca] + (std::lower_bound(part[ca].begin(), part[ca].end(), cb) - part[ca].begin());
                    const double mm = p.w * M[a] * M[b];
                    for (int t = 0; t < 9; ++t) {
                        aGP[9 * k + t] += mm * GP[t / 3][t % 3];
                        aG[9 * k + t] += mm * G[t / 3][t % 3];
                    }
                    for (int i = 0; i < 3; ++i) aN[3 * k + i] += mm * p.basis[0][i];
                    aM[k] += mm;
                }
            }
        }
        // partners ordered by body node id (rows/cols of nodal-space operators)
        std::vector<std::vector<int32_t>> bypos(ncn);
        for (int64_t a = 0; a < ncn; ++a) {
            bypos[a].resize(part[a].size());
            std::iota(bypos[a].begin(), bypos[a].end(), 0);
            std::sort(bypos[a].begin(), bypos[a].end(),
                      [&](int32_t x, int32_t y) { return nodeCont[s][part[a][x]] < nodeCont[s][part[a][y]]; });
        }
        std::vector<int64_t> rowc(nn, -1);  // body node -> contact index
        for (int64_t a = 0; a < ncn; ++a) rowc[nodeCont[s][a]] = a;
        // nodal-space rows (3 nn): systMass (cols 3 nn), systTran(_pena) (cols mc)
        auto emit_nodal = [&](bool mass, bool pena) {
            Csr m;
            m.nrow = 3 * nn;
            m.ncol = mass ? 3 * nn : mc;
            m.ptr.assign(3 * nn + 1, 0);
            for (int64_t n = 0; n < nn; ++n) {
                const int64_t a = rowc[n];
                const int64_t per = a < 0 ? 0 : (int64_t)part[a].size() * ((mass || C == 3) ? 3 : 1);
                for (int i = 0; i < 3; ++i) m.ptr[3 * n + i + 1] = per;
            }
            for (int64_t r = 0; r < 3 * nn; ++r) m.ptr[r + 1] += m.ptr[r];
            m.col.resize(m.ptr[3 * nn]);
            m.val.resize(m.ptr[3 * nn]);
            for (int64_t a = 0; a < ncn; ++a) {
                const int64_t n = nodeCont[s][a];
                for (int i = 0; i < 3; ++i) {
                    int64_t w = m.ptr[3 * n + i];
                    for (size_t t = 0; t < part[a].size(); ++t) {
                        const int64_t kk = mass ? bypos[a][t] : (int64_t)t;
                        const int64_t k = pptr[a] + kk;
                        const int64_t cb = part[a][kk];
                        if (mass) {
                            const int64_t nb = nodeCont[s][cb];
                            for (int j = 0; j < 3; ++j) { m.col[w] = (int32_t)(3 * nb + j); m.val[w++] = aGP[9 * k + 3 * i + j]; }
                        } else if (C == 3) {
                            for (int j = 0; j < 3; ++j) {
                                m.col[w] = (int32_t)(3 * cb + j);
                                m.val[w++] = pena ? aGP[9 * k + 3 * i + j] : aG[9 * k + 3 * i + j];
                            }
                        } else {
                            m.col[w] = (int32_t)cb;
                            m.val[w++] = pena ? penN * aN[3 * k + i] : aN[3 * k + i];
                        }
                    }
                }
            }
            return m;
        };
        // contact-space rows (mc): inteMass(_pena)
        auto emit_contact = [&](bool pena) {
            Csr m;
            m.nrow = m.ncol = mc;
            m.ptr.assign(mc + 1, 0);
            for (int64_t a = 0; a < ncn; ++a)
                for (int i = 0; i < C; ++i) m.ptr[C * a + i + 1] = (int64_t)part[a].size() * C;
            for (int64_t r = 0; r < mc; ++r) m.ptr[r + 1] += m.ptr[r];
            m.col.resize(m.ptr[mc]);
            m.val.resize(m.ptr[mc]);
            for (int64_t a = 0; a < ncn; ++a)
                for (int i = 0; i < C; ++i) {
                    int64_t w = m.ptr[C * a + i];
                    for (size_t t = 0; t < part[a].size(); ++t) {
                        const int64_t k = pptr[a] + (int64_t)t, cb = part[a][t];
                        for (int j = 0; j < C; ++j) {
                            m.col[w] = (int32_t)(C * cb + j);
                            m.val[w++] = C == 3 ? (pena ? aGP[9 * k + 3 * i + j] : aG[9 * k + 3 * i + j])
                                                : (pena ? aM[k] * penN : aM[k]);
                        }
                    }
                }
            return m;
        };
        systMass[s] = emit_nodal(true, false);
        systTran[s] = emit_nodal(false, false);
        systTran_pena[s] = emit_nodal(false, true);
        inteMass[s] = emit_contact(false);
        inteMass_pena[s] = emit_contact(true);
        // per-ip operators: inpoLagr (C nip x mc), inpoDisp (C nip x 3 nn), inteInpo (mc x C nip)
        const double sgn = (s == 0) ? -1.0 : 1.0;
        Csr& L = inpoLagr[s];
        Csr& Dd = inpoDisp[s];
        L.nrow = Dd.nrow = C * nip;
        L.ncol = mc;
        Dd.ncol = 3 * nn;
        L.ptr.assign(C * nip + 1, 0);
        Dd.ptr.assign(C * nip + 1, 0);
        for (int64_t r = 0; r < C * nip; ++r) {
            L.ptr[r + 1] = L.ptr[r] + 4 * C;
            Dd.ptr[r + 1] = Dd.ptr[r] + 12;
        }
        L.col.resize(L.ptr.back());
        L.val.resize(L.ptr.back());
        Dd.col.resize(Dd.ptr.back());
        Dd.val.resize(Dd.ptr.back());
        Csr& Ii = inteInpo[s];
        Ii.nrow = mc;
        Ii.ncol = C * nip;
        Ii.ptr.assign(mc + 1, 0);
        for (int64_t q = 0; q < nip; ++q)
            for (int a = 0; a < 4; ++a)
                for (int k = 0; k < C; ++k) Ii.ptr[C * ipc[4 * q + a] + k + 1] += C;
        for (int64_t r = 0; r < mc; ++r) Ii.ptr[r + 1] += Ii.ptr[r];
        Ii.col.resize(Ii.ptr[mc]);
        Ii.val.resize(Ii.ptr[mc]);
        std::vector<int64_t> ifill(Ii.ptr.begin(), Ii.ptr.end() - 1);
        for (int64_t q = 0; q < nip; ++q) {
            const IntegralPoint& p = ip[q];
            const double* M = p.shap[s];
            int ord_c[4] = {0, 1, 2, 3}, ord_n[4] = {0, 1, 2, 3};
            std::sort(ord_c, ord_c + 4, [&](int x, int y) { return ipc[4 * q + x] < ipc[4 * q + y]; });
            std::sort(ord_n, ord_n + 4, [&](int x, int y) { return p.node[s][x] < p.node[s][y]; });
            for (int m = 0; m < C; ++m) {
                const int64_t r = C * q + m;
                int64_t wl = L.ptr[r], wd = Dd.ptr[r];
                for (int t = 0; t < 4; ++t) {
                    const int a = ord_c[t];
                    if (C == 1) {
                        L.col[wl] = ipc[4 * q + a];
                        L.val[wl++] = M[a];
                    } else {
                        for (int k = 0; k < 3; ++k) {
                            L.col[wl] = 3 * ipc[4 * q + a] + k;
                            L.val[wl++] = p.basis[m][k] * M[a];
                        }
                    }
                    const int an = ord_n[t];
                    for (int k = 0; k < 3; ++k) {
                        Dd.col[wd] = (int32_t)(3 * p.node[s][an] + k);
                        Dd.val[wd++] = p.basis[C == 1 ? 0 : m][k] * M[an];
                    }
                }
            }
            for (int a = 0; a < 4; ++a)
                for (int k = 0; k < C; ++k) {
                    const int64_t row = C * ipc[4 * q + a] + k;
                    for (int m = 0; m < C; ++m) {
                        const int64_t w = ifill[row]++;
                        Ii.col[w] = (int32_t)(C * q + m);
                        Ii.val[w] = sgn * (p.w * M[a] * (C == 1 ? 1.0 : p.basis[m][k]));
                    }
                }
        }
    }
    // CONT_ROTA (MCONTACT.h:157-179) on the operators that map to or from a body's nodal vectors in
    // its rotated frames: R^T on the rows of systTran(_pena) (349-350, 392-393, 415), R on the
    // columns of inpoDisp (656-660, 693-697); systMass stays global (CONSTRAINT rotates it with the
    // stiffness, MULTIGRID.h:1105-1124).  A side with rotated contact nodes leaves the factored
    // per-ip form (its rows are no longer outer products of the shape values and the basis).
    factored = true;
    for (int s = 0; s < 2; ++s) {
        const auto& rot = g[s]->nodeRota;
        if (rot.empty()) continue;
        bool any = false;
        for (int64_t n : nodeCont[s]) any = any || rot.count(n);
        if (!any) continue;
        factored = false;
        for (Csr* M : {&systTran[s], &systTran_pena[s]})
            for (int64_t n : nodeCont[s]) {
                const auto it = rot.find(n);
                if (it == rot.end()) continue;
                const double* R = it->second.data();
                const int64_t len = M->ptr[3 * n + 1] - M->ptr[3 * n];
                double* v[3] = {&M->val[M->ptr[3 * n]], &M->val[M->ptr[3 * n + 1]], &M->val[M->ptr[3 * n + 2]]};
                for (int64_t k = 0; k < len; ++k) {
                    const double o[3] = {v[0][k], v[1][k], v[2][k]};
                    for (int a = 0; a < 3; ++a) v[a][k] = R[a] * o[0] + R[3 + a] * o[1] + R[6 + a] * o[2];
                }
            }
        Csr& Dd = inpoDisp[s];
        for (int64_t r = 0; r < Dd.nrow; ++r)
            for (int64_t k = Dd.ptr[r]; k < Dd.ptr[r + 1]; k += 3) {  // one node's three columns, 3 n + 0..2
                const auto it = rot.find(Dd.col[k] / 3);
                if (it == rot.end()) continue;
                const double* R = it->second.data();
                const double o[3] = {Dd.val[k], Dd.val[k + 1], Dd.val[k + 2]};
                for (int b = 0; b < 3; ++b) Dd.val[k + b] = o[0] * R[b] + o[1] * R[3 + b] + o[2] * R[6 + b];
            }
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

void MCONTACT::ESTABLISH(const std::vector<uint8_t>* owned) {
    auto mine = [&](int64_t tv) { return !owned || (*owned)[tv] != 0; };
    const int64_t nsub = (int64_t)multGrid.size(), nint = (int64_t)searCont.size();
    // ---- TRANSFER first: a general tree (local refinement -> hanging level, coupled nodes) is
    // renumbered to the reference's positions (MULTIGRID.h:884-910, earlTran), and the integration
    // points of its interfaces follow the numbering before the mortar operators are built; on a
    // uniform tree node ids already are positions.  Transferred: the owned subdomains, the mates of
    // their interfaces, and with a coarse space every subdomain (MULTISCALE reads all of them).
    std::vector<uint8_t> need(nsub, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) need[tv] = mine(tv) || (muscSett & 3) ? 1 : 0;
    for (const auto& itf : searCont)
        if (mine(itf.body[0]) || mine(itf.body[1])) need[itf.body[0]] = need[itf.body[1]] = 1;
    std::vector<uint8_t> renumbered(nsub, 0);
    std::vector<double> t_transfer(nsub, 0.0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tv = 0; tv < nsub; ++tv) {
        MULTIGRID& g = multGrid[tv];
        if (!need[tv] || !g.scalProl.empty()) continue;
        const auto t0 = std::chrono::steady_clock::now();
        g.TRANSFER();
        t_transfer[tv] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        renumbered[tv] = g.general ? 1 : 0;
    }
    for (int64_t ts = 0; ts < nint; ++ts)
        for (int s = 0; s < 2; ++s) {
            const int64_t b = searCont[ts].body[s];
            if (!renumbered[b]) continue;
            const MULTIGRID& g = multGrid[b];
            std::vector<int64_t> pos(g.posiNode.size());
            for (int64_t p = 0; p < (int64_t)g.posiNode.size(); ++p) pos[g.posiNode[p]] = p;
            for (auto& ip : searCont[ts].ip)
                for (int k = 0; k < 4; ++k) ip.node[s][k] = pos.at(ip.node[s][k]);
        }
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t ts = 0; ts < nint; ++ts) {
        Interface& itf = searCont[ts];
        if (mine(itf.body[0]) || mine(itf.body[1])) itf.BUILD(multGrid[itf.body[0]], multGrid[itf.body[1]]);
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tv = 0; tv < nsub; ++tv) {
        if (!mine(tv)) continue;
        MULTIGRID& g = multGrid[tv];
        const bool verbose = std::getenv("DDPCA_VERBOSE") != nullptr;
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto t1 = now();
        g.STIF_MATR();
        auto t2 = now();
        for (const auto& itf : searCont)
            for (int s = 0; s < 2; ++s)
                if (itf.body[s] == tv) g.ADD_NODAL(itf.systMass[s]);
        auto t3 = now();
        g.CONSTRAINT();
        // the hanging level's rows of prolOper[maxiLeve] (OUTP_SUB1, MULTIGRID.h:1279), read by the
        // device (op_hang) as for an operator-level subdomain (ddpca_problem_set_hanging)
        if (g.nodeAll) g.hangProl = g.hangRows();
        auto t4 = now();
        if (verbose) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::fprintf(stderr, "[ddpca] establish sd %ld: transfer %.0f ms, stif %.0f ms, systMass %.0f ms, constraint %.0f ms\n",
                         (long)tv, t_transfer[tv], ms(t1, t2), ms(t2, t3), ms(t3, t4));
        }
    }
    // ---- coarse space (MCONTACT.h:858-863)
    if ((muscSett & 3) == 3)
        throw std::invalid_argument("muscSett: choose one coarse space (1 = MULTISCALE, 2 = MULTISCALE_1)");
    if (muscSett & 1) {
        // the dof bookkeeping and prolongation chains of every subdomain (baseReco, the coarse
        // contact unknowns of every interface's side 0)
        for (int64_t tv = 0; tv < (int64_t)multGrid.size(); ++tv) {
            if (mine(tv)) continue;
            MULTIGRID& g = multGrid[tv];
            if (g.scalProl.empty()) g.TRANSFER();
            g.FLAGS();
            g.PROL_OPER();
        }
        MULTISCALE(owned);
    }
    if (muscSett & 2) {
        // the dof bookkeeping of every subdomain (baseReco) and the transfer stencils of the
        // mates of owned interface sides (their restriction chains)
        for (int64_t tv = 0; tv < (int64_t)multGrid.size(); ++tv) {
            if (mine(tv)) continue;
            MULTIGRID& g = multGrid[tv];
            if (g.scalProl.empty()) g.TRANSFER();
            g.FLAGS();
            g.PROL_OPER();
        }
        MULTISCALE_1(owned);
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
                         const int64_t slav[4], std::vector<IntegralPoint>& out, int sub) {
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
    // polygons = the sub x sub cells of the master square (sub = 1: the square itself, the
    // intersection with a coincident slave face; sub = 2^k: what SEGMENT_INTERSECT clips against a
    // slave face mesh 2^k times finer), vertices sorted by angle about the cell centroid, each
    // triangulated from that centroid (CSEARCH.h:614-775)
    // one integration point at master natural coordinates (xi, et) with weight factor wgt
    auto emit = [&](double xi, double et, double wgt) {
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
        p.w = wgt * jac;
        out.push_back(p);
    };
    const double g = std::sqrt(1.0 / 3.0);
    const double gl[2] = {-g, g};
    const double hc = 2.0 / sub;
    for (int cy = 0; cy < sub; ++cy)
        for (int cx = 0; cx < sub; ++cx) {
            const double x0 = -1.0 + cx * hc, y0 = -1.0 + cy * hc;
            const double poly[4][2] = {{x0, y0}, {x0 + hc, y0}, {x0 + hc, y0 + hc}, {x0, y0 + hc}};
            const double c0 = x0 + 0.5 * hc, c1 = y0 + 0.5 * hc;  // sub = 1: the origin
            for (int t = 0; t < 4; ++t) {
                const double* v1 = poly[t];
                const double* v2 = poly[(t + 1) % 4];
                const double area = std::abs((v1[0] - c0) * (v2[1] - c1) - (v1[1] - c1) * (v2[0] - c0)) / 2.0;
                for (int i = 0; i < 2; ++i)
                    for (int j = 0; j < 2; ++j) {
                        // PREP.h:336-361 triangle rule, CSEARCH.h:468-483
                        const double b0 = (1.0 + gl[i]) / 2.0;
                        const double b1 = (1.0 - gl[i]) * (1.0 + gl[j]) / 4.0;
                        const double b2 = 1.0 - b0 - b1;
                        const double wq = (1.0 - gl[i]) / 8.0;
                        emit(b0 * c0 + b1 * v1[0] + b2 * v2[0], b0 * c1 + b1 * v1[1] + b2 * v2[1], 2.0 * area * wq);
                    }
            }
        }
}

}  // namespace ddpca

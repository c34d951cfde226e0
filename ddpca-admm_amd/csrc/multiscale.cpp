// Host restatement of the two coarse spaces of the reference's ADMM loop on any octree -- the
// interface-eliminated one, MCONTACT::MULTISCALE_1 (MCONTACT.h:1672-2301), and the LATIN-type one,
// MCONTACT::MULTISCALE (898-1536) -- and of accuProl (864-872).  Setup only: the per-iteration
// correction runs on the GPU (device_mcontact.hip, MCONTACT.h:2539-2624).
//
// Numbering: positions (MULTIGRID.h:884-910); the library renumbers a general tree at TRANSFER, so
// the reference's earlTran is the identity here and the nodal interface operators already act on
// positions (incl. the hanging level past maxiLeve).  Notation for body b: L = maxiLeve,
// d = doleMcsc[b], C_l = consOper[l] (free-dof selection), R = the nodal rotations (CONT_ROTA,
// MCONTACT.h:157-179: nodeRota's 3x3 block on a rotated node, I elsewhere),
//   P_l  = prolOper[l] (MULTIGRID.h:1141-1181: scalar stencil entries, w R_off^T / w R_par blocks
//          where exactly one end is rotated), P_L = prolOper[maxiLeve] (the hanging level: identity
//          on the level-L positions, the hanging nodes' parents below),
//   Q    = P_L P_{L-1} ... P_d   (positions incl. the hanging level <- level-d nodes; one composite
//          stencil with 3x3 block entries where a rotation enters),
//   H    = P_L C_L^T             (positions <- free fine dofs: the hanging fold),
//   Rc   = realProl[d]^T ... realProl[L-1]^T, realProl[l] = C_{l+1} P_l C_l^T (the condensed
//          chain, masked at every level; MULTIGRID.h:1246-1249).
// The reference uses Q inside globCoup_1 / globCoup and accuProl, H and Rc for every right-hand-side
// operator (MCONTACT.h:1808-1819, 2010-2019, 2113-2118, 2266-2271).  On a uniformly refined tree
// without rotations H = C_L^T and Q is one scalar stencil with <= 8 parents per node.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <stdexcept>
#include <string>
#include <unordered_map>

#include "mcontact.hpp"

namespace ddpca {

namespace {

struct Trip {
    int64_t r, c;
    double v;
};

// CSR from triplets, duplicates summed in insertion order, columns sorted (Eigen setFromTriplets).
// The sort is stable: an entry's sum then depends only on the order its own contributions were
// appended, not on what else the array holds -- a rank-local build (ESTABLISH(owner, rank)) gives
// the full build's rows bit for bit, and the multi-rank runs stay the single-rank run's arithmetic
Csr from_triplets(int64_t nrow, int64_t ncol, std::vector<Trip>& t) {
    std::stable_sort(t.begin(), t.end(), [](const Trip& a, const Trip& b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
    Csr m;
    m.nrow = nrow;
    m.ncol = ncol;
    m.ptr.assign(nrow + 1, 0);
    for (size_t k = 0; k < t.size();) {
        size_t e = k;
        double v = 0.0;
        while (e < t.size() && t[e].r == t[k].r && t[e].c == t[k].c) v += t[e++].v;
        if (t[k].r < 0 || t[k].r >= nrow || t[k].c < 0 || t[k].c >= ncol)
            throw std::logic_error("MULTISCALE: triplet out of range");
        m.col.push_back((int32_t)t[k].c);
        m.val.push_back(v);
        m.ptr[t[k].r + 1]++;
        k = e;
    }
    for (int64_t r = 0; r < nrow; ++r) m.ptr[r + 1] += m.ptr[r];
    return m;
}

void append(std::vector<Trip>& t, const Csr& A, int64_t roff, int64_t coff, double scale = 1.0) {
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) t.push_back({roff + r, coff + A.col[k], scale * A.val[k]});
}

Csr transpose_csr(const Csr& A) {
    std::vector<Trip> t;
    t.reserve(A.nnz());
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) t.push_back({A.col[k], r, A.val[k]});
    return from_triplets(A.ncol, A.nrow, t);
}

// A * B, both CSR
Csr spgemm(const Csr& A, const Csr& B) {
    if (A.ncol != B.nrow) throw std::logic_error("MULTISCALE: spgemm shape");
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t i = A.col[k];
            for (int64_t q = B.ptr[i]; q < B.ptr[i + 1]; ++q) t.push_back({r, B.col[q], A.val[k] * B.val[q]});
        }
    return from_triplets(A.nrow, B.ncol, t);
}

// free index -> nodal dof (all levels: the level-ordered numbering makes level l's free dofs a
// prefix of the fine level's)
std::vector<int64_t> free_to_dof(const MULTIGRID& g) {
    std::vector<int64_t> f(g.freeCount.back());
    for (int64_t d = 0; d < (int64_t)g.freeIndex.size(); ++d)
        if (g.freeIndex[d] >= 0) f[g.freeIndex[d]] = d;
    return f;
}

std::vector<int64_t> block_of(const Stencil& S) {
    std::vector<int64_t> b(S.col.size(), -1);
    for (size_t q = 0; q < S.bent.size(); ++q) b[S.bent[q]] = (int64_t)q;
    return b;
}

// The composite prolongation Q from level d to the positions [0, nrow), nrow = leveCount[L] or,
// with `hanging`, every position (the hanging level's rows of P_L).  `rotated`: the prolOper chain
// (block entries of the nodal rotations), else the scalar chain scalProl (MULTISCALE's ficoCotr,
// MCONTACT.h:910-914).  Rows are built in position order: a node's parents sit at lower positions.
Stencil composite(const MULTIGRID& g, int64_t d, bool hanging, bool rotated) {
    const int64_t L = g.maxiLeve, NL = g.leveCount.at(L), nd = g.leveCount.at(d);
    const bool hang = hanging && g.nodeAll > NL;
    const int64_t nrow = hang ? g.nodeAll : NL;
    const std::vector<Stencil>& P = rotated && !g.prolOper.empty() ? g.prolOper : g.scalProl;
    const Stencil& Hs = rotated && g.prolHang.nf ? g.prolHang : g.hangStencil;
    if ((int64_t)P.size() < L) throw std::logic_error("MULTISCALE: transfer stencils missing (TRANSFER)");
    if ((int64_t)g.nodeLevel.size() < NL) throw std::logic_error("MULTISCALE: node levels missing (TRANSFER)");
    std::vector<std::vector<int64_t>> bof(L);
    for (int64_t l = d; l < L; ++l) bof[l] = block_of(P[l]);
    const std::vector<int64_t> hof = hang ? block_of(Hs) : std::vector<int64_t>();
    Stencil Q;
    Q.nf = nrow;
    Q.nc = nd;
    Q.ptr.assign(1, 0);
    std::vector<int64_t> qb;  // per entry: its block in Q.bval, or -1
    struct Acc {
        int32_t c;
        bool blk;
        double v[9];
    };
    std::vector<Acc> acc;
    auto add = [&](int32_t c, bool blk, const double* m, double s) {
        Acc* a = nullptr;
        for (auto& e : acc)
            if (e.c == c) a = &e;
        if (!a) {
            acc.push_back(Acc{c, false, {0, 0, 0, 0, 0, 0, 0, 0, 0}});
            a = &acc.back();
        }
        if (blk && !a->blk) {  // scalar so far -> s I
            const double s0 = a->v[0];
            for (int q = 0; q < 9; ++q) a->v[q] = q % 4 == 0 ? s0 : 0.0;
            a->blk = true;
        }
        if (a->blk) {
            for (int q = 0; q < 9; ++q) a->v[q] += blk ? m[q] : (q % 4 == 0 ? s : 0.0);
        } else {
            a->v[0] += s;
        }
    };
    for (int64_t n = 0; n < nrow; ++n) {
        if (n < nd) {
            Q.col.push_back((int32_t)n);
            Q.w.push_back(1.0);
            qb.push_back(-1);
            Q.ptr.push_back((int64_t)Q.col.size());
            continue;
        }
        const Stencil* S;
        const std::vector<int64_t>* bo;
        if (n < NL) {
            const int lv = g.nodeLevel[n];  // created on level lv: parents on level lv - 1
            if (lv < 1 || lv - 1 < d || lv > L) throw std::logic_error("MULTISCALE: node level inconsistent with leveCount");
            S = &P[lv - 1];
            bo = &bof[lv - 1];
        } else {
            S = &Hs;
            bo = &hof;
        }
        acc.clear();
        for (int64_t k = S->ptr[n]; k < S->ptr[n + 1]; ++k) {
            const int64_t c = S->col[k];
            const double* E = (*bo)[k] >= 0 ? &S->bval[9 * (*bo)[k]] : nullptr;
            const double w = S->w[k];
            for (int64_t q = Q.ptr[c]; q < Q.ptr[c + 1]; ++q) {
                const double* F = qb[q] >= 0 ? &Q.bval[9 * qb[q]] : nullptr;
                if (!E && !F) {
                    add(Q.col[q], false, nullptr, w * Q.w[q]);
                    continue;
                }
                double A[9], B[9], M[9];
                for (int t = 0; t < 9; ++t) {
                    A[t] = E ? E[t] : (t % 4 == 0 ? w : 0.0);
                    B[t] = F ? F[t] : (t % 4 == 0 ? Q.w[q] : 0.0);
                }
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) M[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
                add(Q.col[q], true, M, 0.0);
            }
        }
        std::sort(acc.begin(), acc.end(), [](const Acc& a, const Acc& b) { return a.c < b.c; });
        for (const auto& e : acc) {
            Q.col.push_back(e.c);
            if (e.blk) {
                Q.w.push_back(0.0);
                qb.push_back((int64_t)Q.bval.size() / 9);
                Q.bval.insert(Q.bval.end(), e.v, e.v + 9);
            } else {
                Q.w.push_back(e.v[0]);
                qb.push_back(-1);
            }
        }
        Q.ptr.push_back((int64_t)Q.col.size());
    }
    for (int64_t k = 0; k < (int64_t)qb.size(); ++k)
        if (qb[k] >= 0) Q.bent.push_back(k);
    return Q;
}

// Q (x) I3 (block entries as they are) C_d^T as nodal rows 3 n + a of the nodes n < nrow selected
// by sel (others empty); columns = free dofs of level d (MCONTACT.h:1812-1819, 866-871)
Csr nodal_prolong(const MULTIGRID& g, const Stencil& Q, int64_t d, const std::vector<uint8_t>* sel, int64_t nrow = -1) {
    if (nrow < 0) nrow = Q.nf;
    const std::vector<int64_t> bo = block_of(Q);
    std::vector<Trip> t;
    for (int64_t n = 0; n < nrow; ++n) {
        if (sel && !(*sel)[n]) continue;
        for (int a = 0; a < 3; ++a)
            for (int64_t k = Q.ptr[n]; k < Q.ptr[n + 1]; ++k) {
                const int64_t c = Q.col[k];
                if (bo[k] >= 0) {
                    for (int b = 0; b < 3; ++b) {
                        const int32_t f = g.freeIndex[3 * c + b];
                        if (f >= 0) t.push_back({3 * n + a, f, Q.bval[9 * bo[k] + 3 * a + b]});
                    }
                } else {
                    const int32_t f = g.freeIndex[3 * c + a];
                    if (f >= 0) t.push_back({3 * n + a, f, Q.w[k]});
                }
            }
    }
    return from_triplets(3 * nrow, g.freeCount[d], t);
}

// CONT_ROTA (MCONTACT.h:157-179) on assembled nodal operators: R^T A (rows) and A R (columns);
// R's block on node n is nodeRota[n] (positions), I elsewhere
const double* rota(const MULTIGRID& g, int64_t node) {
    const auto it = g.nodeRota.find(node);
    return it == g.nodeRota.end() ? nullptr : it->second.data();
}

Csr rot_rows(const MULTIGRID& g, const Csr& A) {
    if (g.nodeRota.empty()) return A;
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow; ++r) {
        const double* R = rota(g, r / 3);
        const int b = (int)(r % 3);
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            if (!R) {
                t.push_back({r, A.col[k], A.val[k]});
                continue;
            }
            for (int a = 0; a < 3; ++a) t.push_back({r - b + a, A.col[k], R[3 * b + a] * A.val[k]});  // (R^T)_ab = R_ba
        }
    }
    return from_triplets(A.nrow, A.ncol, t);
}

Csr rot_cols(const MULTIGRID& g, const Csr& A) {
    if (g.nodeRota.empty()) return A;
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t c = A.col[k];
            const double* R = rota(g, c / 3);
            const int a = (int)(c % 3);
            if (!R) {
                t.push_back({r, c, A.val[k]});
                continue;
            }
            for (int b = 0; b < 3; ++b) t.push_back({r, c - a + b, A.val[k] * R[3 * a + b]});
        }
    return from_triplets(A.nrow, A.ncol, t);
}

void rot_vec(const MULTIGRID& g, std::vector<double>& v) {
    for (const auto& kv : g.nodeRota) {
        const int64_t n = kv.first;
        if (3 * n + 2 >= (int64_t)v.size()) continue;
        const double* R = kv.second.data();
        double o[3];
        for (int a = 0; a < 3; ++a) o[a] = R[a] * v[3 * n] + R[3 + a] * v[3 * n + 1] + R[6 + a] * v[3 * n + 2];
        for (int a = 0; a < 3; ++a) v[3 * n + a] = o[a];
    }
}

// H^T A: nodal rows (positions incl. the hanging level) -> free rows of the fine level
Csr fold_rows(const Csr& H, int64_t nfree, const Csr& A) {
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow && r < H.nrow; ++r) {
        if (A.ptr[r] == A.ptr[r + 1]) continue;
        for (int64_t h = H.ptr[r]; h < H.ptr[r + 1]; ++h)
            for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) t.push_back({H.col[h], A.col[k], H.val[h] * A.val[k]});
    }
    return from_triplets(nfree, A.ncol, t);
}

// A H with the free fine columns moved back to their nodal dofs (neceTran, MCONTACT.h:1874-1880:
// the level-L positions' free dofs; a hanging column folds into its parents)
Csr fold_cols(const Csr& H, const std::vector<int64_t>& f2d, const Csr& A) {
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t c = A.col[k];
            if (c >= H.nrow) continue;
            for (int64_t h = H.ptr[c]; h < H.ptr[c + 1]; ++h) t.push_back({r, f2d[H.col[h]], A.val[k] * H.val[h]});
        }
    return from_triplets(A.nrow, A.ncol, t);
}

// Rc A = realProl[d]^T ... realProl[L-1]^T A for A with rows = free dofs of level L
// (MCONTACT.h:1883-1885, 2017-2019, 2116-2118, 2269-2271), touching only A's nonempty rows (surface
// operators); prolOper's block entries as 3x3 blocks.  Gather form: every coarse row lists its
// (fine row, weight) children in the order the scatter form appended them (fine row ascending,
// stencil entry, block row) and sums w * A[r, :] into a dense accumulator in that order -- per entry
// the same additions in the same order as from_triplets over the scattered triplets, so the same
// bits, without the triplet array (≈ 3.4 triplets per stored entry of A: 8 GB and a stable sort
// for a 1.2M-dof subdomain's consStif, the full globTran_D_1 of the tests), rows in parallel.
Csr restrict_chain(const MULTIGRID& g, int64_t d, const std::vector<int64_t>& f2d, Csr A) {
    const std::vector<Stencil>& P = !g.prolOper.empty() ? g.prolOper : g.scalProl;
    for (int64_t l = g.maxiLeve - 1; l >= d; --l) {
        const Stencil& S = P[l];
        const std::vector<int64_t> bo = block_of(S);
        const int64_t nc = g.freeCount[l];
        // the children of every coarse row, in the scatter form's order
        auto visit = [&](auto&& emit) {
            for (int64_t r = 0; r < A.nrow; ++r) {
                if (A.ptr[r] == A.ptr[r + 1]) continue;
                const int64_t dof = f2d[r];  // free row r of level l+1 -> nodal dof
                const int64_t n = dof / 3, a = dof % 3;
                for (int64_t s = S.ptr[n]; s < S.ptr[n + 1]; ++s) {
                    const int64_t cn = S.col[s];
                    if (bo[s] >= 0) {
                        for (int b = 0; b < 3; ++b) {
                            const int32_t c = g.freeIndex[3 * cn + b];
                            const double w = S.bval[9 * bo[s] + 3 * a + b];
                            if (c < 0 || w == 0.0) continue;
                            emit(c, r, w);
                        }
                    } else {
                        const int32_t c = g.freeIndex[3 * cn + a];
                        if (c < 0) continue;  // realProl keeps free coarse columns only
                        emit(c, r, S.w[s]);
                    }
                }
            }
        };
        std::vector<int64_t> start(nc + 1, 0);
        visit([&](int64_t c, int64_t, double) {
            if (c >= nc) throw std::logic_error("MULTISCALE: restriction row out of range");
            ++start[c + 1];
        });
        for (int64_t c = 0; c < nc; ++c) start[c + 1] += start[c];
        std::vector<int64_t> cr(start[nc]);
        std::vector<double> cw(start[nc]);
        {
            std::vector<int64_t> pos(start.begin(), start.end() - 1);
            visit([&](int64_t c, int64_t r, double w) {
                cr[pos[c]] = r;
                cw[pos[c]++] = w;
            });
        }
        std::vector<std::vector<int32_t>> rcol(nc);
        std::vector<std::vector<double>> rval(nc);
        // (called inside the subdomain-parallel loops too, where this region runs on one thread:
        // the accumulator is per thread and kept across calls, its marks cleared row by row)
#pragma omp parallel
        {
            thread_local std::vector<double> acc;
            thread_local std::vector<uint8_t> mark;
            if ((int64_t)acc.size() < A.ncol) {
                acc.resize(A.ncol, 0.0);
                mark.resize(A.ncol, 0);
            }
            std::vector<int32_t> touched;
#pragma omp for schedule(dynamic, 64)
            for (int64_t c = 0; c < nc; ++c) {
                touched.clear();
                for (int64_t q = start[c]; q < start[c + 1]; ++q) {
                    const int64_t r = cr[q];
                    const double w = cw[q];
                    for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
                        const int32_t j = A.col[k];
                        const double t = w * A.val[k];  // rounded on its own, as the triplet's value
                        if (!mark[j]) {
                            mark[j] = 1;
                            acc[j] = 0.0;
                            touched.push_back(j);
                        }
                        acc[j] += t;
                    }
                }
                std::sort(touched.begin(), touched.end());
                rcol[c].assign(touched.begin(), touched.end());
                rval[c].resize(touched.size());
                for (size_t i = 0; i < touched.size(); ++i) {
                    rval[c][i] = acc[touched[i]];
                    mark[touched[i]] = 0;
                }
            }
        }
        Csr R;
        R.nrow = nc;
        R.ncol = A.ncol;
        R.ptr.assign(nc + 1, 0);
        for (int64_t c = 0; c < nc; ++c) R.ptr[c + 1] = R.ptr[c] + (int64_t)rcol[c].size();
        R.col.resize(R.ptr[nc]);
        R.val.resize(R.ptr[nc]);
#pragma omp parallel for schedule(static)
        for (int64_t c = 0; c < nc; ++c) {
            std::copy(rcol[c].begin(), rcol[c].end(), R.col.begin() + R.ptr[c]);
            std::copy(rval[c].begin(), rval[c].end(), R.val.begin() + R.ptr[c]);
        }
        A = std::move(R);
    }
    return A;
}

Csr dense_vector_csr(const std::vector<double>& v) {
    Csr m;
    m.nrow = (int64_t)v.size();
    m.ncol = 1;
    m.ptr.assign(m.nrow + 1, 0);
    for (int64_t i = 0; i < m.nrow; ++i) {
        if (v[i] != 0.0) {
            m.col.push_back(0);
            m.val.push_back(v[i]);
        }
        m.ptr[i + 1] = (int64_t)m.col.size();
    }
    return m;
}

// rows of the fine level's free dofs of a nodal-row operator whose rows lie on the level-L
// positions (C_L A)
Csr rows_to_free(const MULTIGRID& g, const Csr& A) {
    std::vector<Trip> t;
    for (int64_t r = 0; r < A.nrow; ++r) {
        const int32_t fr = r < (int64_t)g.freeIndex.size() ? g.freeIndex[r] : -1;
        if (fr < 0) continue;
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) t.push_back({fr, A.col[k], A.val[k]});
    }
    return from_triplets(g.freeCount.back(), A.ncol, t);
}

// the first `rows` rows of a stencil (the level-L positions of a composite with hanging rows)
Stencil stencil_prefix(const Stencil& Q, int64_t rows) {
    Stencil P;
    P.nf = rows;
    P.nc = Q.nc;
    P.ptr.assign(Q.ptr.begin(), Q.ptr.begin() + rows + 1);
    P.col.assign(Q.col.begin(), Q.col.begin() + P.ptr.back());
    P.w.assign(Q.w.begin(), Q.w.begin() + P.ptr.back());
    for (size_t q = 0; q < Q.bent.size(); ++q)
        if (Q.bent[q] < P.ptr.back()) {
            P.bent.push_back(Q.bent[q]);
            P.bval.insert(P.bval.end(), Q.bval.begin() + 9 * q, Q.bval.begin() + 9 * q + 9);
        }
    return P;
}

// accuProl[tv] = C_L P_{L-1} ... P_d C_d^T (MCONTACT.h:864-872), free_L x free_d
Csr accu_prol(const MULTIGRID& g, const Stencil& Qfine, int64_t d) {
    return rows_to_free(g, nodal_prolong(g, Qfine, d, nullptr));
}

}  // namespace

// Composite nodal prolongation from level d to the fine level (scalar chain, no masks).
Stencil accumulated_stencil(const MULTIGRID& g, int64_t d) { return composite(g, d, false, false); }

void MCONTACT::MULTISCALE_1(const std::vector<uint8_t>* owned) {
    const int64_t nsub = (int64_t)multGrid.size(), nint = (int64_t)searCont.size();
    auto mine = [&](int64_t tv) { return !owned || (*owned)[tv] != 0; };
    if ((int64_t)doleMcsc.size() != nsub) doleMcsc.assign(nsub, 0);  // MCONTACT.h:185-187
    CoarseSpace& C = coarse;
    C = CoarseSpace();
    const bool verbose = std::getenv("DDPCA_VERBOSE") != nullptr;
    auto t_start = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!verbose) return;
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ddpca] MULTISCALE_1 %s: %.0f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t_start).count());
        t_start = now;
    };
    C.built.assign(nsub, 0);
    // bodies whose restriction chain / nodal prolongation is needed here: owned ones and the
    // mates of their interface sides
    std::vector<uint8_t> need(nsub, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) need[tv] = mine(tv);
    for (const auto& itf : searCont)
        if (mine(itf.body[0]) || mine(itf.body[1])) need[itf.body[0]] = need[itf.body[1]] = 1;
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const MULTIGRID& g = multGrid[tv];
        if (need[tv] && g.freeCount.empty()) throw std::logic_error("MULTISCALE_1: grid flags missing");
        if (doleMcsc[tv] < 0 || doleMcsc[tv] > g.maxiLeve) throw std::invalid_argument("doleMcsc out of range");
    }
    // baseReco (MCONTACT.h:849-857): every rank knows every subdomain's level-d size
    C.baseReco.assign(nsub + 1, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const MULTIGRID& g = multGrid[tv];
        int64_t nd = 0;
        if (!g.freeCount.empty()) nd = g.freeCount[doleMcsc[tv]];
        else throw std::logic_error("MULTISCALE_1: every subdomain needs its dof flags (FLAGS)");
        C.baseReco[tv + 1] = C.baseReco[tv] + nd;
    }
    C.n = C.baseReco[nsub];
    std::vector<std::vector<int64_t>> f2d(nsub);
    std::vector<Stencil> Qall(nsub);  // Q with the hanging level's rows
    std::vector<Csr> Hf(nsub);        // H = P_L C_L^T
    C.accuQ.assign(nsub, Stencil());
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tv = 0; tv < nsub; ++tv) {
        if (!need[tv]) continue;
        const MULTIGRID& g = multGrid[tv];
        f2d[tv] = free_to_dof(g);
        Qall[tv] = composite(g, doleMcsc[tv], true, true);
        Hf[tv] = nodal_prolong(g, composite(g, g.maxiLeve, true, true), g.maxiLeve, nullptr);
        if (mine(tv)) C.accuQ[tv] = stencil_prefix(Qall[tv], g.leveCount[g.maxiLeve]);
    }
    for (int64_t tv = 0; tv < nsub; ++tv) C.built[tv] = mine(tv);
    lap("accumulated stencils");
    auto Rc = [&](int64_t tv, const Csr& A_free) { return restrict_chain(multGrid[tv], doleMcsc[tv], f2d[tv], A_free); };
    auto QI = [&](int64_t tv, const std::vector<uint8_t>& sel) {
        return nodal_prolong(multGrid[tv], Qall[tv], doleMcsc[tv], &sel);
    };
    auto HT = [&](int64_t tv, const Csr& A) { return fold_rows(Hf[tv], multGrid[tv].freeCount.back(), A); };
    // ---- per interface side: nodal surface operators from the integration points
    //      (MCONTACT.h:1699-1841, 1906-2047, 2078-2119, 2130-2297)
    std::vector<Trip> coup;                       // globCoup_1 (owned rows)
    std::vector<std::vector<Trip>> tranS(nsub);   // globTran_S[tv]
    std::vector<double> forc(C.n, 0.0);
    C.globTran_1.assign(nint, {});
    // one task per owned interface side, run in parallel; results merged in task order
    struct SideOut {
        std::vector<Trip> coup, tran;     // globCoup_1 rows e, globTran_D_1[e] interface part
        std::vector<std::pair<int64_t, double>> forc;
    };
    std::vector<std::pair<int64_t, int>> tasks;
    for (int64_t ts = 0; ts < nint; ++ts)
        for (int s = 0; s < 2; ++s)
            if (mine(searCont[ts].body[s])) tasks.push_back({ts, s});
    std::vector<SideOut> outs(tasks.size());
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t task = 0; task < (int64_t)tasks.size(); ++task) {
        const int64_t ts = tasks[task].first;
        const int s = tasks[task].second;
        std::vector<Trip>& coup_t = outs[task].coup;
        std::vector<Trip>& tran_t = outs[task].tran;
        auto& forc_t = outs[task].forc;
        const Interface& itf = searCont[ts];
        const int Cc = itf.comp();
        const double pen[3] = {itf.penN, itf.penF, itf.penF};
        const int64_t e = itf.body[s], m = itf.body[1 - s];
        const MULTIGRID& ge = multGrid[e];
        const MULTIGRID& gm = multGrid[m];
        const int64_t Ne = ge.nodalCount(), Nm = gm.nodalCount();
        // self operators are the interface mass / transfer of ESTABLISH up to -1/2 and CONT_ROTA:
        //   sum_ip -1/2 w R^T N_e^T T^T P T N_e R = -1/2 R^T systMass[s] R   (MCONTACT.h:1734-1749)
        //   sum_ip -1/2 w R^T N_e^T T^T [T] M_e  = -1/2 systTran[s]          (MCONTACT.h:2170-2212; BUILD rotates systTran)
        Csr S = rot_rows(ge, rot_cols(ge, itf.systMass[s])), Ts = itf.systTran[s];
        for (auto& v : S.val) v *= -0.5;
        for (auto& v : Ts.val) v *= -0.5;
        // cross (self node a, mate node b) blocks: sum_ip w Me_a Mm_b {T^T P T, T^T T, n}
        std::vector<int64_t> cidx(Ne, -1), midx(Nm, -1);
        for (size_t k = 0; k < itf.nodeCont[s].size(); ++k) cidx[itf.nodeCont[s][k]] = (int64_t)k;
        for (size_t k = 0; k < itf.nodeCont[1 - s].size(); ++k) midx[itf.nodeCont[1 - s][k]] = (int64_t)k;
        const int64_t nce = (int64_t)itf.nodeCont[s].size();
        std::vector<std::vector<int64_t>> part(nce);     // mate contact nodes per self contact node
        std::vector<std::vector<double>> blk(nce);       // 9 GP + 9 G + 3 n per partner
        std::vector<double> gap(3 * Ne, 0.0);
        std::vector<uint8_t> sel_e(Ne, 0), sel_m(Nm, 0);
        for (const auto& p : itf.ip) {
            double G[9], GP[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double x = 0, y = 0;
                    for (int c = 0; c < Cc; ++c) {
                        x += p.basis[c][i] * p.basis[c][j];
                        y += p.basis[c][i] * pen[c] * p.basis[c][j];
                    }
                    G[3 * i + j] = x;
                    GP[3 * i + j] = y;
                }
            const double* Me = p.shap[s];
            const double* Mm = p.shap[1 - s];
            for (int a = 0; a < 4; ++a) {
                const int64_t na = p.node[s][a], ca = cidx[na];
                sel_e[na] = 1;
                sel_m[p.node[1 - s][a]] = 1;
                for (int b = 0; b < 4; ++b) {
                    const int64_t cb = midx[p.node[1 - s][b]];
                    auto& pl = part[ca];
                    size_t k = std::find(pl.begin(), pl.end(), cb) - pl.begin();
                    if (k == pl.size()) {
                        pl.push_back(cb);
                        blk[ca].resize(21 * pl.size(), 0.0);
                    }
                    double* q = &blk[ca][21 * k];
                    const double ww = p.w * Me[a] * Mm[b];
                    for (int t = 0; t < 9; ++t) {
                        q[t] += ww * GP[t];
                        q[9 + t] += ww * G[t];
                    }
                    for (int t = 0; t < 3; ++t) q[18 + t] += ww * p.basis[0][t];
                }
                // initial-gap force, normal only (MCONTACT.h:2081-2108), side 1 negated
                const double gsc = (s == 1 ? -0.5 : 0.5) * p.w * itf.penN * p.gap * Me[a];
                for (int i = 0; i < 3; ++i) gap[3 * na + i] += gsc * p.basis[0][i];
            }
        }
        std::vector<Trip> tM, tTm;
        for (int64_t ca = 0; ca < nce; ++ca) {
            const int64_t na = itf.nodeCont[s][ca];
            for (size_t k = 0; k < part[ca].size(); ++k) {
                const int64_t mb = itf.nodeCont[1 - s][part[ca][k]];
                const double* q = &blk[ca][21 * k];
                for (int i = 0; i < 3; ++i) {
                    for (int j = 0; j < 3; ++j) tM.push_back({3 * na + i, 3 * mb + j, -0.5 * q[3 * i + j]});
                    // globTran_1 mate: +1/2 w N_m^T T^T [T] N_e, row = mate dof, col = self contact dof
                    if (Cc == 1) tTm.push_back({3 * mb + i, ca, 0.5 * q[18 + i]});
                    else
                        for (int j = 0; j < 3; ++j) tTm.push_back({3 * mb + i, 3 * ca + j, 0.5 * q[9 + 3 * j + i]});
                }
            }
        }
        // -1/2 w R_e^T N_e^T T^T P T N_m R_m (MCONTACT.h:1765-1780), and its transpose, the mate
        // rows of globTran_D_1 (1967-1982)
        const Csr Mx = rot_rows(ge, rot_cols(gm, from_triplets(3 * Ne, 3 * Nm, tM)));
        const Csr MT = transpose_csr(Mx);
        const Csr Tm = rot_rows(gm, from_triplets(3 * Nm, itf.mside(s), tTm));  // (MCONTACT.h:2177-2179, 2213-2215)
        rot_vec(ge, gap);                                                           // (2096-2098)
        // globCoup_1 += inteCoup[ts][s] (MCONTACT.h:1797-1841): Q-based Galerkin blocks
        {
            const Csr Qe = QI(e, sel_e), Qm = QI(m, sel_m);
            const Csr QeT = transpose_csr(Qe);
            append(coup_t, spgemm(QeT, spgemm(S, Qe)), C.baseReco[e], C.baseReco[e]);
            append(coup_t, spgemm(QeT, spgemm(Mx, Qm)), C.baseReco[e], C.baseReco[m]);
        }
        // globTran_D_1 interface part (MCONTACT.h:1999-2052): rows e and rows m (H^T, Rc),
        // columns = u_e through H (the level-L free dofs)
        append(tran_t, Rc(e, HT(e, fold_cols(Hf[e], f2d[e], S))), C.baseReco[e], 0);
        append(tran_t, Rc(m, HT(m, fold_cols(Hf[e], f2d[e], MT))), C.baseReco[m], 0);
        // globForc_1 gap part (MCONTACT.h:2110-2119)
        {
            const Csr gc = Rc(e, HT(e, dense_vector_csr(gap)));
            for (int64_t r = 0; r < gc.nrow; ++r)
                for (int64_t k = gc.ptr[r]; k < gc.ptr[r + 1]; ++k) forc_t.push_back({C.baseReco[e] + r, gc.val[k]});
        }
        // globTran_1[ts][s] (MCONTACT.h:2246-2297)
        {
            std::vector<Trip> t;
            append(t, Rc(e, HT(e, Ts)), C.baseReco[e], 0);
            append(t, Rc(m, HT(m, Tm)), C.baseReco[m], 0);
            C.globTran_1[ts][s] = from_triplets(C.n, itf.mside(s), t);
        }
    }
    for (size_t task = 0; task < tasks.size(); ++task) {
        const int64_t e = searCont[tasks[task].first].body[tasks[task].second];
        coup.insert(coup.end(), outs[task].coup.begin(), outs[task].coup.end());
        tranS[e].insert(tranS[e].end(), outs[task].tran.begin(), outs[task].tran.end());
        for (const auto& rv : outs[task].forc) forc[rv.first] += rv.second;
        outs[task] = SideOut();
    }
    lap("interface operators");
    // ---- subdomain blocks: consStif[d] (MCONTACT.h:1675-1693) and Rc consForc (2058-2067)
    for (int64_t tv = 0; tv < nsub; ++tv) {
        if (!mine(tv)) continue;
        const MULTIGRID& g = multGrid[tv];
        append(coup, g.consStif(doleMcsc[tv]), C.baseReco[tv], C.baseReco[tv]);
        const Csr fc = Rc(tv, dense_vector_csr(g.consForc));
        for (int64_t r = 0; r < fc.nrow; ++r)
            for (int64_t k = fc.ptr[r]; k < fc.ptr[r + 1]; ++k) forc[C.baseReco[tv] + r] += fc.val[k];
    }
    C.globCoup_1 = from_triplets(C.n, C.n, coup);
    C.globForc_1 = std::move(forc);
    C.globTran_S.assign(nsub, Csr());
    for (int64_t tv = 0; tv < nsub; ++tv)
        if (mine(tv)) C.globTran_S[tv] = from_triplets(C.n, 3 * multGrid[tv].nodalCount(), tranS[tv]);
    lap("subdomain blocks");
    C.ready = true;
}

// Full globTran_D_1[tv] = Rc consStif[L] neceTran + interface part (tests; the device applies the
// stiffness part as an SpMV followed by the restriction chain instead); columns = nodal dofs
// (positions), the level-L positions' free dofs only (MCONTACT.h:1868-1895)
Csr MCONTACT::globTran_D_1(int64_t tv) const {
    const MULTIGRID& g = multGrid.at(tv);
    const std::vector<int64_t> f2d = free_to_dof(g);
    Csr K = g.consStif(g.maxiLeve);
    for (auto& c : K.col) c = (int32_t)f2d[c];
    K.ncol = 3 * g.nodalCount();
    Csr R = restrict_chain(g, doleMcsc.at(tv), f2d, K);
    std::vector<Trip> t;
    append(t, R, coarse.baseReco[tv], 0);
    append(t, coarse.globTran_S.at(tv), 0, 0);
    return from_triplets(coarse.n, 3 * g.nodalCount(), t);
}

// accuProl[tv] = C_L P_{L-1} ... P_d C_d^T (MCONTACT.h:864-872), free_L x free_d
Csr MCONTACT::accuProl(int64_t tv) const {
    if (coarse.assembled) return coarse.accuProl_full.at(tv);
    const MULTIGRID& g = multGrid.at(tv);
    return accu_prol(g, coarse.accuQ.at(tv), doleMcsc.at(tv));
}

}  // namespace ddpca

namespace ddpca {

// Host restatement of the LATIN-type coarse space, MCONTACT::MULTISCALE (MCONTACT.h:898-1536,
// muscSett bit 0, CYLINDER.h:42) on any octree.  Side 0 of every interface carries the coarse
// contact unknowns: ficoCotr = the scalar chain scalProl[L..d] (hanging level included, no
// rotations: MCONTACT.h:910-914) restricted to side 0's contact nodes, one unknown per level-d node
// it touches (x3 with friction).  dispUnba takes R^T on its rows and Q^T (MCONTACT.h:1033-1035,
// 1069-1074), globTran_D R on its columns (1430-1432).  Output in the assembled LATIN form the device
// consumes (CoarseSpace::latin; the same fields ddpca_problem_set_coarse_latin fills from a caller).
void MCONTACT::MULTISCALE(const std::vector<uint8_t>* owned) {
    const int64_t nsub = (int64_t)multGrid.size(), nint = (int64_t)searCont.size();
    auto mine = [&](int64_t tv) { return !owned || (*owned)[tv] != 0; };
    if ((int64_t)doleMcsc.size() != nsub) doleMcsc.assign(nsub, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const MULTIGRID& g = multGrid[tv];
        if (g.freeCount.empty()) throw std::logic_error("MULTISCALE: every subdomain needs its dof flags (FLAGS)");
        if (mine(tv) && g.levelStif.empty()) throw std::logic_error("MULTISCALE: owned subdomain not established");
        if (doleMcsc[tv] < 0 || doleMcsc[tv] > g.maxiLeve) throw std::invalid_argument("doleMcsc out of range");
    }
    CoarseSpace C;
    C.assembled = true;
    C.latin = true;
    C.rank_local = owned != nullptr;
    C.built.assign(nsub, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) C.built[tv] = mine(tv);
    C.baseReco.assign(nsub + 1, 0);
    for (int64_t tv = 0; tv < nsub; ++tv) C.baseReco[tv + 1] = C.baseReco[tv] + multGrid[tv].freeCount[doleMcsc[tv]];
    const int64_t N = C.baseReco[nsub];
    // prolongation chains: the scalar one (hanging level included) of side 0 of every interface (its
    // coarse contact unknowns number every rank's columns, so each rank derives all of them), the
    // rotated one of the owned bodies
    std::vector<uint8_t> need0(nsub, 0);
    for (const auto& itf : searCont) need0[itf.body[0]] = 1;
    std::vector<Stencil> Qs(nsub), Qr(nsub);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tv = 0; tv < nsub; ++tv) {
        if (need0[tv]) Qs[tv] = composite(multGrid[tv], doleMcsc[tv], true, false);
        if (mine(tv)) Qr[tv] = composite(multGrid[tv], doleMcsc[tv], true, true);
    }
    // side-0 contact nodes of interfaces this rank did not build (Interface::BUILD's order)
    std::vector<std::vector<int64_t>> nc0(nint);
    for (int64_t ts = 0; ts < nint; ++ts) {
        const Interface& itf = searCont[ts];
        if (!itf.nodeCont[0].empty() || itf.ip.empty()) {
            nc0[ts] = itf.nodeCont[0];
            continue;
        }
        std::unordered_map<int64_t, int64_t> seen;
        for (const auto& p : itf.ip)
            for (int k = 0; k < 4; ++k)
                if (seen.emplace(p.node[0][k], (int64_t)seen.size()).second) nc0[ts].push_back(p.node[0][k]);
    }
    // ---- ficoCotr[ts] (side 0): contact index -> selected level-d nodes (MCONTACT.h:900-959)
    std::vector<Csr> fico(nint);
    std::vector<int64_t> contReco(nint + 1, 0);
    C.coarNode.assign(nint, {});
    for (int64_t ts = 0; ts < nint; ++ts) {
        const Interface& itf = searCont[ts];
        const Stencil& Q0 = Qs[itf.body[0]];
        const auto& nc0t = nc0[ts];
        std::vector<int64_t> newc(Q0.nc, -1);
        for (int64_t k = 0; k < (int64_t)nc0t.size(); ++k)
            for (int64_t q = Q0.ptr[nc0t[k]]; q < Q0.ptr[nc0t[k] + 1]; ++q) newc[Q0.col[q]] = 0;
        int64_t ncc = 0;
        for (int64_t c = 0; c < Q0.nc; ++c)
            if (newc[c] == 0) newc[c] = ncc++;
        const int comp = itf.comp();
        std::vector<Trip> t;
        for (int64_t k = 0; k < (int64_t)nc0t.size(); ++k)
            for (int64_t q = Q0.ptr[nc0t[k]]; q < Q0.ptr[nc0t[k] + 1]; ++q)
                for (int j = 0; j < comp; ++j) t.push_back({comp * k + j, comp * newc[Q0.col[q]] + j, Q0.w[q]});
        fico[ts] = from_triplets(comp * (int64_t)nc0t.size(), comp * ncc, t);
        contReco[ts + 1] = contReco[ts] + comp * ncc;
        for (int64_t c = 0; c < Q0.nc; ++c)
            if (newc[c] >= 0) C.coarNode[ts].push_back(c);
    }
    const int64_t n = N + contReco[nint];
    C.n = n;
    std::vector<Trip> coup;
    for (int64_t tv = 0; tv < nsub; ++tv)
        if (mine(tv)) append(coup, multGrid[tv].consStif(doleMcsc[tv]), C.baseReco[tv], C.baseReco[tv]);
    C.globTran_L.assign(nint, {});
    C.globTran_pena_L.assign(nint, {});
    C.globTran_D_L.assign(nint, {});
    std::vector<std::vector<Trip>> coup_side(2 * nint);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t task = 0; task < 2 * nint; ++task) {
        const int64_t ts = task / 2;
        const int tv = (int)(task % 2);
        const Interface& itf = searCont[ts];
        const int64_t b = itf.body[tv];
        if (!mine(b)) continue;  // the side's owner assembles it (the device sums the ranks)
        const MULTIGRID& g = multGrid[b];
        const int comp = itf.comp();
        const int64_t N3 = 3 * g.nodalCount();
        const int64_t m0 = itf.mside(0), mv = itf.mside(tv);
        std::vector<int64_t> c0(multGrid[itf.body[0]].nodalCount(), -1), cv(g.nodalCount(), -1);
        for (size_t k = 0; k < itf.nodeCont[0].size(); ++k) c0[itf.nodeCont[0][k]] = (int64_t)k;
        for (size_t k = 0; k < itf.nodeCont[tv].size(); ++k) cv[itf.nodeCont[tv][k]] = (int64_t)k;
        std::vector<Trip> disp, unba, tran, tranp, tranD;
        for (const auto& p : itf.ip) {
            const double* Me = p.shap[tv];
            const double* M0 = p.shap[0];
            const double* nv = p.basis[0];
            double G[9], GP[9];  // T^T T, T^T P T (T rows = basiVect, P = diag(penN, penF, penF))
            const double pen[3] = {itf.penN, itf.penF, itf.penF};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double x = 0.0, y = 0.0;
                    for (int c = 0; c < 3; ++c) {
                        x += p.basis[c][i] * p.basis[c][j];
                        y += p.basis[c][i] * pen[c] * p.basis[c][j];
                    }
                    G[3 * i + j] = x;
                    GP[3 * i + j] = y;
                }
            for (int a = 0; a < 4; ++a) {
                const int64_t node_a = p.node[tv][a], ca0 = c0[p.node[0][a]];
                for (int bb = 0; bb < 4; ++bb) {
                    const int64_t cb0 = c0[p.node[0][bb]], cbv = cv[p.node[tv][bb]];
                    if (comp == 1) {
                        // inteCoup: w pn N_e^T n^T M_0e (MCONTACT.h:1010-1044), unbaMatr w pn M_0e^T M_0e
                        for (int k = 0; k < 3; ++k)
                            disp.push_back({3 * node_a + k, cb0, p.w * itf.penN * Me[a] * nv[k] * M0[bb]});
                        unba.push_back({ca0, cb0, p.w * itf.penN * M0[a] * M0[bb]});
                        // globTran: w M_0e^T M_e (MCONTACT.h:1249-1268); globTran_D: w pn M_0e^T n N_e
                        tran.push_back({ca0, cbv, p.w * M0[a] * Me[bb]});
                        for (int k = 0; k < 3; ++k)
                            tranD.push_back({ca0, 3 * p.node[tv][bb] + k, p.w * itf.penN * M0[a] * nv[k] * Me[bb]});
                    } else {
                        for (int i = 0; i < 3; ++i)
                            for (int j = 0; j < 3; ++j) {
                                disp.push_back({3 * node_a + i, 3 * cb0 + j, p.w * Me[a] * M0[bb] * GP[3 * i + j]});
                                unba.push_back({3 * ca0 + i, 3 * cb0 + j, p.w * M0[a] * M0[bb] * GP[3 * i + j]});
                                tran.push_back({3 * ca0 + i, 3 * cbv + j, p.w * M0[a] * Me[bb] * G[3 * i + j]});
                                tranp.push_back({3 * ca0 + i, 3 * cbv + j, p.w * M0[a] * Me[bb] * GP[3 * i + j]});
                                tranD.push_back({3 * ca0 + i, 3 * p.node[tv][bb] + j, p.w * M0[a] * Me[bb] * GP[3 * i + j]});
                            }
                    }
                }
            }
        }
        const Csr& F = fico[ts];
        const Csr FT = transpose_csr(F);
        // dispUnba -> level-d free rows: C_d Q^T R^T (MCONTACT.h:1033-1035, 1068-1074)
        const Csr QI = nodal_prolong(g, Qr[b], doleMcsc[b], nullptr);
        const Csr D = spgemm(transpose_csr(QI), spgemm(rot_rows(g, from_triplets(N3, m0, disp)), F));
        std::vector<Trip>& out = coup_side[task];
        const int64_t cr = N + contReco[ts];
        for (int64_t r = 0; r < D.nrow; ++r)
            for (int64_t k = D.ptr[r]; k < D.ptr[r + 1]; ++k) {
                out.push_back({C.baseReco[b] + r, cr + D.col[k], -D.val[k]});
                out.push_back({cr + D.col[k], C.baseReco[b] + r, -D.val[k]});
            }
        append(out, spgemm(FT, spgemm(from_triplets(m0, m0, unba), F)), cr, cr);
        // globTran / globTran_pena / globTran_D (MCONTACT.h:1235-1534): rows N + contReco[ts] + i
        auto place = [&](const Csr& A, int64_t ncol) {
            std::vector<Trip> t;
            append(t, spgemm(FT, A), cr, 0);
            return from_triplets(n, ncol, t);
        };
        C.globTran_L[ts][tv] = place(from_triplets(m0, mv, tran), mv);
        if (comp == 1) {
            C.globTran_pena_L[ts][tv] = C.globTran_L[ts][tv];
            for (auto& v : C.globTran_pena_L[ts][tv].val) v *= itf.penN;
        } else
            C.globTran_pena_L[ts][tv] = place(from_triplets(m0, mv, tranp), mv);
        C.globTran_D_L[ts][tv] = place(rot_cols(g, from_triplets(m0, N3, tranD)), N3);
    }
    for (auto& t : coup_side) coup.insert(coup.end(), t.begin(), t.end());
    C.globCoup_1 = from_triplets(n, n, coup);
    C.globForc_1.assign(n, 0.0);
    // accuProl[tv] = C_L P_{L-1} ... P_d C_d^T (MCONTACT.h:864-872)
    for (int64_t tv = 0; tv < nsub; ++tv)
        C.accuProl_full.push_back(mine(tv) ? accu_prol(multGrid[tv], Qr[tv], doleMcsc[tv]) : Csr());
    C.ready = true;
    coarse = std::move(C);
}

}  // namespace ddpca

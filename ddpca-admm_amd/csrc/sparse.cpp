// Host sparse kernels for operator setup (not on the per-iteration path).
#include "sparse.hpp"

#include <algorithm>
#include <numeric>
#include <omp.h>
#include <stdexcept>

namespace ddpca {

void Bsr3::apply(const double* x, double* y) const {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nb; ++i) {
        double a0 = 0, a1 = 0, a2 = 0;
        for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
            const double* b = &val[9 * k];
            const double* xj = x + 3 * (int64_t)col[k];
            a0 += b[0] * xj[0] + b[1] * xj[1] + b[2] * xj[2];
            a1 += b[3] * xj[0] + b[4] * xj[1] + b[5] * xj[2];
            a2 += b[6] * xj[0] + b[7] * xj[1] + b[8] * xj[2];
        }
        y[3 * i] = a0;
        y[3 * i + 1] = a1;
        y[3 * i + 2] = a2;
    }
}

namespace {
// C = P^T A P with P = S (x) I3 plus S's 3x3 block entries (rotated nodes): per coarse node, the
// blocks B1^T A_f1f2 B2 over the entries (f1 -> c1) and (f2 -> c2), a scalar entry being w I
Bsr3 galerkin_rap_blocks(const Bsr3& A, const Stencil& S) {
    const int64_t nc = S.nc;
    std::vector<int64_t> blk_of(S.col.size(), -1);
    for (size_t q = 0; q < S.bent.size(); ++q) blk_of[S.bent[q]] = (int64_t)q;
    std::vector<int64_t> tptr(nc + 1, 0);
    for (int64_t f = 0; f < S.nf; ++f)
        for (int64_t k = S.ptr[f]; k < S.ptr[f + 1]; ++k) tptr[S.col[k] + 1]++;
    for (int64_t c = 0; c < nc; ++c) tptr[c + 1] += tptr[c];
    std::vector<int64_t> tent(tptr[nc]);  // S^T: coarse node -> entry index
    std::vector<int32_t> tfine(tptr[nc]);
    {
        std::vector<int64_t> fill(tptr.begin(), tptr.end() - 1);
        for (int64_t f = 0; f < S.nf; ++f)
            for (int64_t k = S.ptr[f]; k < S.ptr[f + 1]; ++k) {
                const int64_t p = fill[S.col[k]]++;
                tent[p] = k;
                tfine[p] = (int32_t)f;
            }
    }
    auto block = [&](int64_t k, double B[9]) {
        if (blk_of[k] >= 0) std::copy(&S.bval[9 * blk_of[k]], &S.bval[9 * blk_of[k]] + 9, B);
        else
            for (int q = 0; q < 9; ++q) B[q] = q % 4 == 0 ? S.w[k] : 0.0;
    };
    std::vector<std::vector<int32_t>> rcol(nc);
    std::vector<std::vector<double>> rval(nc);
#pragma omp parallel
    {
        std::vector<int32_t> mark(nc, -1);
        std::vector<int32_t> cols;
        std::vector<double> acc;
#pragma omp for schedule(dynamic, 64)
        for (int64_t c1 = 0; c1 < nc; ++c1) {
            cols.clear();
            acc.clear();
            for (int64_t t = tptr[c1]; t < tptr[c1 + 1]; ++t) {
                const int64_t f1 = tfine[t];
                double B1[9];
                block(tent[t], B1);
                for (int64_t k = A.ptr[f1]; k < A.ptr[f1 + 1]; ++k) {
                    const int64_t f2 = A.col[k];
                    const double* Ak = A.block(k);
                    double T[9];  // B1^T A_f1f2
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b)
                            T[3 * a + b] = B1[a] * Ak[b] + B1[3 + a] * Ak[3 + b] + B1[6 + a] * Ak[6 + b];
                    for (int64_t s = S.ptr[f2]; s < S.ptr[f2 + 1]; ++s) {
                        const int32_t c2 = S.col[s];
                        double B2[9];
                        block(s, B2);
                        int32_t pos = mark[c2];
                        if (pos < 0) {
                            pos = (int32_t)cols.size();
                            mark[c2] = pos;
                            cols.push_back(c2);
                            acc.resize(acc.size() + 9, 0.0);
                        }
                        double* o = &acc[9 * (size_t)pos];
                        for (int a = 0; a < 3; ++a)
                            for (int b = 0; b < 3; ++b)
                                o[3 * a + b] += T[3 * a] * B2[b] + T[3 * a + 1] * B2[3 + b] + T[3 * a + 2] * B2[6 + b];
                    }
                }
            }
            std::vector<int32_t> order(cols.size());
            std::iota(order.begin(), order.end(), 0);
            std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return cols[a] < cols[b]; });
            rcol[c1].resize(cols.size());
            rval[c1].resize(9 * cols.size());
            for (size_t q = 0; q < order.size(); ++q) {
                rcol[c1][q] = cols[order[q]];
                std::copy(&acc[9 * (size_t)order[q]], &acc[9 * (size_t)order[q]] + 9, &rval[c1][9 * q]);
            }
            for (int32_t c2 : cols) mark[c2] = -1;
        }
    }
    Bsr3 C;
    C.nb = C.mb = nc;
    C.ptr.assign(nc + 1, 0);
    for (int64_t c = 0; c < nc; ++c) C.ptr[c + 1] = C.ptr[c] + (int64_t)rcol[c].size();
    C.col.resize(C.ptr[nc]);
    C.val.resize(9 * C.ptr[nc]);
    for (int64_t c = 0; c < nc; ++c) {
        std::copy(rcol[c].begin(), rcol[c].end(), C.col.begin() + C.ptr[c]);
        std::copy(rval[c].begin(), rval[c].end(), C.val.begin() + 9 * C.ptr[c]);
    }
    return C;
}
}  // namespace

Bsr3 galerkin_rap(const Bsr3& A, const Stencil& S) {
    if (!S.bent.empty()) return galerkin_rap_blocks(A, S);
    const int64_t nc = S.nc;
    // S^T: coarse node -> list of (fine node, weight)
    std::vector<int64_t> tptr(nc + 1, 0);
    for (int64_t f = 0; f < S.nf; ++f)
        for (int64_t k = S.ptr[f]; k < S.ptr[f + 1]; ++k) tptr[S.col[k] + 1]++;
    for (int64_t c = 0; c < nc; ++c) tptr[c + 1] += tptr[c];
    std::vector<int32_t> tcol(tptr[nc]);
    std::vector<double> tw(tptr[nc]);
    {
        std::vector<int64_t> fill(tptr.begin(), tptr.end() - 1);
        for (int64_t f = 0; f < S.nf; ++f)
            for (int64_t k = S.ptr[f]; k < S.ptr[f + 1]; ++k) {
                int64_t p = fill[S.col[k]]++;
                tcol[p] = (int32_t)f;
                tw[p] = S.w[k];
            }
    }
    std::vector<std::vector<int32_t>> rcol(nc);
    std::vector<std::vector<double>> rval(nc);
#pragma omp parallel
    {
        std::vector<int32_t> mark(nc, -1);
        std::vector<int32_t> cols;
        std::vector<double> acc;
#pragma omp for schedule(dynamic, 64)
        for (int64_t c1 = 0; c1 < nc; ++c1) {
            cols.clear();
            acc.clear();
            for (int64_t t = tptr[c1]; t < tptr[c1 + 1]; ++t) {
                const int64_t f1 = tcol[t];
                const double w1 = tw[t];
                for (int64_t k = A.ptr[f1]; k < A.ptr[f1 + 1]; ++k) {
                    const int64_t f2 = A.col[k];
                    const double* blk = A.block(k);
                    for (int64_t s = S.ptr[f2]; s < S.ptr[f2 + 1]; ++s) {
                        const int32_t c2 = S.col[s];
                        const double ww = w1 * S.w[s];
                        int32_t pos = mark[c2];
                        if (pos < 0) {
                            pos = (int32_t)cols.size();
                            mark[c2] = pos;
                            cols.push_back(c2);
                            acc.resize(acc.size() + 9, 0.0);
                        }
                        double* a = &acc[9 * (size_t)pos];
                        for (int q = 0; q < 9; ++q) a[q] += ww * blk[q];
                    }
                }
            }
            std::vector<int32_t> order(cols.size());
            std::iota(order.begin(), order.end(), 0);
            std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return cols[a] < cols[b]; });
            rcol[c1].resize(cols.size());
            rval[c1].resize(9 * cols.size());
            for (size_t q = 0; q < order.size(); ++q) {
                rcol[c1][q] = cols[order[q]];
                std::copy(&acc[9 * (size_t)order[q]], &acc[9 * (size_t)order[q]] + 9, &rval[c1][9 * q]);
            }
            for (int32_t c2 : cols) mark[c2] = -1;
        }
    }
    Bsr3 C;
    C.nb = C.mb = nc;
    C.ptr.assign(nc + 1, 0);
    for (int64_t c = 0; c < nc; ++c) C.ptr[c + 1] = C.ptr[c] + (int64_t)rcol[c].size();
    C.col.resize(C.ptr[nc]);
    C.val.resize(9 * C.ptr[nc]);
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < nc; ++c) {
        std::copy(rcol[c].begin(), rcol[c].end(), C.col.begin() + C.ptr[c]);
        std::copy(rval[c].begin(), rval[c].end(), C.val.begin() + 9 * C.ptr[c]);
    }
    return C;
}

Csr condense(const Bsr3& A, const std::vector<int32_t>& free_index, int64_t nfree) {
    Csr C;
    C.nrow = C.ncol = nfree;
    C.ptr.assign(nfree + 1, 0);
    // row counts
    for (int64_t i = 0; i < A.nb; ++i)
        for (int a = 0; a < 3; ++a) {
            const int32_t r = free_index[3 * i + a];
            if (r < 0) continue;
            int64_t cnt = 0;
            for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
                for (int b = 0; b < 3; ++b) cnt += free_index[3 * (int64_t)A.col[k] + b] >= 0;
            C.ptr[r + 1] = cnt;
        }
    for (int64_t r = 0; r < nfree; ++r) C.ptr[r + 1] += C.ptr[r];
    C.col.resize(C.ptr[nfree]);
    C.val.resize(C.ptr[nfree]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A.nb; ++i)
        for (int a = 0; a < 3; ++a) {
            const int32_t r = free_index[3 * i + a];
            if (r < 0) continue;
            int64_t p = C.ptr[r];
            for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
                for (int b = 0; b < 3; ++b) {
                    const int32_t c = free_index[3 * (int64_t)A.col[k] + b];
                    if (c < 0) continue;
                    C.col[p] = c;
                    C.val[p] = A.val[9 * k + 3 * a + b];
                    ++p;
                }
        }
    return C;
}

}  // namespace ddpca

namespace ddpca {

Bsr3 condensed_to_bsr3(int64_t nn, int64_t nfree, const int32_t* free_dof, const int64_t* ptr, const int32_t* col,
                       const double* val) {
    std::vector<std::vector<int32_t>> bcols(nn);
    for (int64_t r = 0; r < nfree; ++r) {
        const int32_t dr = free_dof[r];
        if (dr < 0 || dr >= 3 * nn) throw std::invalid_argument("free dof out of range");
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) {
            if (col[k] < 0 || col[k] >= nfree) throw std::invalid_argument("column out of range");
            bcols[dr / 3].push_back(free_dof[col[k]] / 3);
        }
    }
    Bsr3 B;
    B.nb = B.mb = nn;
    B.ptr.assign(nn + 1, 0);
    for (int64_t i = 0; i < nn; ++i) {
        bcols[i].push_back((int32_t)i);
        std::sort(bcols[i].begin(), bcols[i].end());
        bcols[i].erase(std::unique(bcols[i].begin(), bcols[i].end()), bcols[i].end());
        B.ptr[i + 1] = B.ptr[i] + (int64_t)bcols[i].size();
    }
    B.col.resize(B.ptr[nn]);
    B.val.assign(9 * B.ptr[nn], 0.0);
    for (int64_t i = 0; i < nn; ++i) std::copy(bcols[i].begin(), bcols[i].end(), B.col.begin() + B.ptr[i]);
    for (int64_t r = 0; r < nfree; ++r) {
        const int32_t dr = free_dof[r];
        const int64_t i = dr / 3;
        const int32_t* cb = &B.col[B.ptr[i]];
        const int64_t len = B.ptr[i + 1] - B.ptr[i];
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) {
            const int32_t dc = free_dof[col[k]];
            const int64_t pos = B.ptr[i] + (std::lower_bound(cb, cb + len, dc / 3) - cb);
            B.val[9 * pos + 3 * (dr % 3) + dc % 3] += val[k];
        }
    }
    return B;
}

Stencil make_stencil(int64_t nf, int64_t nc, const int64_t* ptr, const int32_t* col, const double* w) {
    Stencil S;
    S.nf = nf;
    S.nc = nc;
    S.ptr.assign(ptr, ptr + nf + 1);
    S.col.assign(col, col + ptr[nf]);
    S.w.assign(w, w + ptr[nf]);
    for (int32_t c : S.col)
        if (c < 0 || c >= nc) throw std::invalid_argument("stencil column out of range");
    return S;
}

Stencil prol_to_stencil(int64_t nf, int64_t nc, int64_t nfree_f, const int32_t* free_f, const int32_t* free_c,
                        const int64_t* ptr, const int32_t* col, const double* val) {
    // blocks per fine node, keyed by coarse node; fm/cm: which rows/columns of the block are free
    struct Blk {
        int32_t p;
        double b[9];
        uint8_t fm, cm;
    };
    std::vector<std::vector<Blk>> rows(nf);
    std::vector<uint8_t> fmask(nf, 0);
    for (int64_t r = 0; r < nfree_f; ++r) {
        const int32_t fd = free_f[r];
        if (fd < 0 || fd >= 3 * nf) throw std::invalid_argument("realProl: fine free dof out of range");
        const int64_t i = fd / 3;
        const int a = fd % 3;
        fmask[i] |= (uint8_t)(1u << a);
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) {
            const int32_t cd = free_c[col[k]];
            if (cd < 0 || cd >= 3 * nc) throw std::invalid_argument("realProl: coarse free dof out of range");
            const int32_t p = cd / 3;
            const int b = cd % 3;
            auto& v = rows[i];
            auto it = std::find_if(v.begin(), v.end(), [p](const Blk& x) { return x.p == p; });
            if (it == v.end()) {
                v.push_back(Blk{p, {0, 0, 0, 0, 0, 0, 0, 0, 0}, 0, 0});
                it = v.end() - 1;
            }
            it->b[3 * a + b] += val[k];
            it->cm |= (uint8_t)(1u << b);
        }
    }
    Stencil S;
    S.nf = nf;
    S.nc = nc;
    S.ptr.assign(nf + 1, 0);
    for (int64_t i = 0; i < nf; ++i) {
        auto& v = rows[i];
        if (i < nc) {  // identity rows (MULTIGRID.h:1144-1146): the node itself, weight 1
            // realProl = consOper_f·prolOper·consOper_cᵀ (MULTIGRID.h:1248): a constrained dof has
            // no row (fine side) or no column (coarse side), so only free×free entries are checked
            for (const Blk& x : v)
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b)
                        if ((fmask[i] >> a & 1) && (x.cm >> b & 1) &&
                            x.b[3 * a + b] != ((x.p == i && a == b) ? 1.0 : 0.0))
                            throw std::invalid_argument("realProl: coarse node row is not the identity");
            S.col.push_back((int32_t)i);
            S.w.push_back(1.0);
        } else {
            std::sort(v.begin(), v.end(), [](const Blk& x, const Blk& y) { return x.p < y.p; });
            for (const Blk& x : v) {
                // scalar iff the free part is w*I (the free diagonal entries equal, the rest 0)
                double w = 0.0;
                bool have = false, scalar = true;
                for (int a = 0; a < 3; ++a)
                    if ((fmask[i] >> a & 1) && (x.cm >> a & 1)) {
                        if (!have) w = x.b[4 * a], have = true;
                        else if (x.b[4 * a] != w) scalar = false;
                    }
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b)
                        if (a != b && x.b[3 * a + b] != 0.0) scalar = false;
                if (!scalar) {
                    S.bent.push_back((int64_t)S.col.size());
                    S.bval.insert(S.bval.end(), x.b, x.b + 9);
                    w = 0.0;
                }
                S.col.push_back(x.p);
                S.w.push_back(w);
            }
        }
        S.ptr[i + 1] = (int64_t)S.col.size();
    }
    return S;
}

}  // namespace ddpca

// Scalar CSR algebra for the host-side assembly of the LAGRANGE path (lagrange.cpp): the few
// Eigen::SparseMatrix operations MCONTACT::LAGRANGE composes (setFromTriplets, products,
// transposes, sums, blocks).  Structure is symbolic as Eigen's: products keep every structurally
// nonzero entry (numerical cancellations and explicit zeros stay stored), since LAGRANGE reads
// the stored pattern (the condensed-dof choice, MCONTACT.h:3289-3323).
#pragma once
#include <algorithm>
#include <stdexcept>
#include <vector>

#include "sparse.hpp"

namespace ddpca {
namespace csr {

struct Trip {
    int64_t r, c;
    double v;
};

// setFromTriplets: duplicates summed, columns sorted, explicit zeros kept
inline Csr from_triplets(int64_t nrow, int64_t ncol, std::vector<Trip>& t) {
    for (const Trip& x : t)
        if (x.r < 0 || x.r >= nrow || x.c < 0 || x.c >= ncol) throw std::logic_error("csr::from_triplets: index out of range");
    std::stable_sort(t.begin(), t.end(), [](const Trip& a, const Trip& b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
    Csr m;
    m.nrow = nrow;
    m.ncol = ncol;
    m.ptr.assign(nrow + 1, 0);
    for (size_t k = 0; k < t.size();) {
        size_t e = k;
        double v = 0.0;
        while (e < t.size() && t[e].r == t[k].r && t[e].c == t[k].c) v += t[e++].v;
        m.col.push_back((int32_t)t[k].c);
        m.val.push_back(v);
        m.ptr[t[k].r + 1]++;
        k = e;
    }
    for (int64_t r = 0; r < nrow; ++r) m.ptr[r + 1] += m.ptr[r];
    return m;
}

inline void append(std::vector<Trip>& t, const Csr& A, int64_t roff, int64_t coff, double s = 1.0) {
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) t.push_back({roff + r, coff + A.col[k], s * A.val[k]});
}

inline Csr transpose(const Csr& A) {
    Csr T;
    T.nrow = A.ncol;
    T.ncol = A.nrow;
    T.ptr.assign(A.ncol + 1, 0);
    for (int32_t c : A.col) T.ptr[c + 1]++;
    for (int64_t r = 0; r < A.ncol; ++r) T.ptr[r + 1] += T.ptr[r];
    T.col.resize(A.col.size());
    T.val.resize(A.val.size());
    std::vector<int64_t> pos(T.ptr.begin(), T.ptr.end() - 1);
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t q = pos[A.col[k]]++;
            T.col[q] = (int32_t)r;
            T.val[q] = A.val[k];
        }
    return T;
}

// A * B (Gustavson, symbolic pattern)
inline Csr multiply(const Csr& A, const Csr& B) {
    if (A.ncol != B.nrow) throw std::logic_error("csr::multiply: shape");
    Csr C;
    C.nrow = A.nrow;
    C.ncol = B.ncol;
    C.ptr.assign(A.nrow + 1, 0);
    std::vector<int64_t> mark(B.ncol, -1);
    std::vector<double> acc(B.ncol, 0.0);
    std::vector<int32_t> cols;
    for (int64_t r = 0; r < A.nrow; ++r) {
        cols.clear();
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t i = A.col[k];
            const double a = A.val[k];
            for (int64_t q = B.ptr[i]; q < B.ptr[i + 1]; ++q) {
                const int32_t c = B.col[q];
                if (mark[c] != r) {
                    mark[c] = r;
                    acc[c] = 0.0;
                    cols.push_back(c);
                }
                acc[c] += a * B.val[q];
            }
        }
        std::sort(cols.begin(), cols.end());
        for (int32_t c : cols) {
            C.col.push_back(c);
            C.val.push_back(acc[c]);
        }
        C.ptr[r + 1] = (int64_t)C.col.size();
    }
    return C;
}

// a A + b B (union pattern)
inline Csr add(const Csr& A, const Csr& B, double a = 1.0, double b = 1.0) {
    if (A.nrow != B.nrow || A.ncol != B.ncol) throw std::logic_error("csr::add: shape");
    std::vector<Trip> t;
    t.reserve(A.col.size() + B.col.size());
    append(t, A, 0, 0, a);
    append(t, B, 0, 0, b);
    return from_triplets(A.nrow, A.ncol, t);
}

inline Csr scale(Csr A, double s) {
    for (double& v : A.val) v *= s;
    return A;
}

// rows [r0, r0 + nr) x columns [c0, c0 + nc) (Eigen .block)
inline Csr block(const Csr& A, int64_t r0, int64_t c0, int64_t nr, int64_t nc) {
    Csr B;
    B.nrow = nr;
    B.ncol = nc;
    B.ptr.assign(nr + 1, 0);
    for (int64_t r = 0; r < nr; ++r) {
        for (int64_t k = A.ptr[r0 + r]; k < A.ptr[r0 + r + 1]; ++k)
            if (A.col[k] >= c0 && A.col[k] < c0 + nc) {
                B.col.push_back((int32_t)(A.col[k] - c0));
                B.val.push_back(A.val[k]);
            }
        B.ptr[r + 1] = (int64_t)B.col.size();
    }
    return B;
}

// y = A x
inline std::vector<double> apply(const Csr& A, const std::vector<double>& x) {
    if ((int64_t)x.size() != A.ncol) throw std::logic_error("csr::apply: shape");
    std::vector<double> y(A.nrow, 0.0);
    for (int64_t r = 0; r < A.nrow; ++r) {
        double s = 0.0;
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) s += A.val[k] * x[A.col[k]];
        y[r] = s;
    }
    return y;
}

// the stored value at (r, c), 0 when not stored (Eigen .coeff)
inline double coeff(const Csr& A, int64_t r, int64_t c) {
    const int32_t* b = A.col.data() + A.ptr[r];
    const int32_t* e = A.col.data() + A.ptr[r + 1];
    const int32_t* it = std::lower_bound(b, e, (int32_t)c);
    return (it != e && *it == c) ? A.val[it - A.col.data()] : 0.0;
}

}  // namespace csr
}  // namespace ddpca

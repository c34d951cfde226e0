// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// CPU restatement of the reference's MGPIS (MGPIS.h) on its own data layout (condensed scalar
// CSR per level, realProl[l] CSR), used only by tests/ and bench.py's cpu_baseline leg as the
// checker.  Pinned against the reference's golden vectors (tests/test_oracle.py): one SGS
// V-cycle application (vcycle_z), CG_SOLV(1) / CG_SOLV(0) solutions and iteration counts.
//   orc_mult_vcyc   MGPIS::MULT_VCYC  MGPIS.h:55-128  (symmetric Gauss-Seidel V(1,1))
//   orc_cg_solv     MGPIS::CG_SOLV    MGPIS.h:163-225 (x0 = 0, rtol on the recursive residual)
// The coarse solve is a dense Cholesky (the reference's SimplicialLDLT, PREP.h:107, agrees to
// rounding).  SpMV is OpenMP-parallel over rows like Eigen's row-major product
// (SparseDenseProduct.h:47-57); the SGS sweeps are sequential as in the reference.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <omp.h>
#include <vector>

namespace {

struct Csr {
    int64_t n = 0, m = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> col;
    std::vector<double> val;
    void spmv(const double* x, double* y) const {
#pragma omp parallel for schedule(static) if (ptr.back() > 20000)
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) s += val[k] * x[col[k]];
            y[i] = s;
        }
    }
    void spmv_t(const double* x, double* y) const {  // y = A^T x (m)
        std::fill(y, y + m, 0.0);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) y[col[k]] += val[k] * x[i];
    }
};

struct Level {
    Csr K, Lo, Up;  // strict lower / strict upper parts (consLowe / consUppe, MGPIS.h:45,50)
    std::vector<double> D;
};

struct Mgpis {
    std::vector<Level> lev;
    std::vector<Csr> P;       // realProl[l]: n_{l+1} x n_l
    std::vector<double> chol;  // dense Cholesky factor of consStif[0]
    int64_t n0 = 0;

    void coarse_solve(const double* b, double* x) const {
        std::vector<double> y(b, b + n0);
        for (int64_t i = 0; i < n0; ++i) {
            double s = y[i];
            for (int64_t k = 0; k < i; ++k) s -= chol[i * n0 + k] * y[k];
            y[i] = s / chol[i * n0 + i];
        }
        for (int64_t i = n0 - 1; i >= 0; --i) {
            double s = y[i];
            for (int64_t k = i + 1; k < n0; ++k) s -= chol[k * n0 + i] * y[k];
            y[i] = s / chol[i * n0 + i];
        }
        std::copy(y.begin(), y.end(), x);
    }

    // MGPIS.h:61-77 / 102-114: one forward + one backward Gauss-Seidel sweep; returns p_1.
    void sgs(const Level& L, const double* rhs, std::vector<double>& x, std::vector<double>& p1) const {
        const int64_t n = L.K.n;
        std::vector<double> p0(n), bpp0(n);
        L.Up.spmv(x.data(), p0.data());
        for (int64_t i = 0; i < n; ++i) {
            p0[i] = -p0[i];
            bpp0[i] = rhs[i] + p0[i];
        }
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = L.Lo.ptr[i]; k < L.Lo.ptr[i + 1]; ++k) s += L.Lo.val[k] * x[L.Lo.col[k]];
            x[i] = (bpp0[i] - s) / L.D[i];
        }
        p1.resize(n);
        for (int64_t i = 0; i < n; ++i) p1[i] = L.D[i] * x[i] - p0[i];
        for (int64_t i = n - 1; i >= 0; --i) {
            double s = 0.0;
            for (int64_t k = L.Up.ptr[i]; k < L.Up.ptr[i + 1]; ++k) s += L.Up.val[k] * x[L.Up.col[k]];
            x[i] = (p1[i] - s) / L.D[i];
        }
    }

    void vcycle(int l, const double* rhs, std::vector<double>& x) const {
        if (l == 0) {
            coarse_solve(rhs, x.data());
            return;
        }
        const Level& L = lev[l];
        const int64_t n = L.K.n;
        std::vector<double> p1;
        sgs(L, rhs, x, p1);
        std::vector<double> lx(n), res(n);
        L.Lo.spmv(x.data(), lx.data());
        for (int64_t i = 0; i < n; ++i) res[i] = rhs[i] - (p1[i] + lx[i]);
        std::vector<double> rc(P[l - 1].m), xc(P[l - 1].m, 0.0), corr(n);
        P[l - 1].spmv_t(res.data(), rc.data());
        vcycle(l - 1, rc.data(), xc);
        P[l - 1].spmv(xc.data(), corr.data());
        for (int64_t i = 0; i < n; ++i) x[i] = x[i] + corr[i];
        std::vector<double> p1b;
        sgs(L, rhs, x, p1b);
    }
};

double dot(const std::vector<double>& a, const std::vector<double>& b) {
    double s = 0.0;
    for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
    return s;
}

}  // namespace

extern "C" {

void* orc_mgpis_create(int nlev, const int64_t* n, const int64_t* const* kp, const int32_t* const* kc,
                       const double* const* kv, const int64_t* const* pp, const int32_t* const* pc,
                       const double* const* pv) {
    auto* M = new Mgpis();
    M->lev.resize(nlev);
    for (int l = 0; l < nlev; ++l) {
        Level& L = M->lev[l];
        const int64_t nl = n[l];
        L.K.n = L.K.m = nl;
        L.K.ptr.assign(kp[l], kp[l] + nl + 1);
        L.K.col.assign(kc[l], kc[l] + kp[l][nl]);
        L.K.val.assign(kv[l], kv[l] + kp[l][nl]);
        L.D.assign(nl, 0.0);
        for (Csr* T : {&L.Lo, &L.Up}) {
            T->n = T->m = nl;
            T->ptr.assign(1, 0);
        }
        for (int64_t i = 0; i < nl; ++i) {
            for (int64_t k = L.K.ptr[i]; k < L.K.ptr[i + 1]; ++k) {
                const int32_t c = L.K.col[k];
                if (c < i) { L.Lo.col.push_back(c); L.Lo.val.push_back(L.K.val[k]); }
                else if (c > i) { L.Up.col.push_back(c); L.Up.val.push_back(L.K.val[k]); }
                else L.D[i] = L.K.val[k];
            }
            L.Lo.ptr.push_back((int64_t)L.Lo.col.size());
            L.Up.ptr.push_back((int64_t)L.Up.col.size());
        }
    }
    M->P.resize(nlev > 0 ? nlev - 1 : 0);
    for (int l = 0; l + 1 < nlev; ++l) {
        Csr& P = M->P[l];
        P.n = n[l + 1];
        P.m = n[l];
        P.ptr.assign(pp[l], pp[l] + P.n + 1);
        P.col.assign(pc[l], pc[l] + pp[l][P.n]);
        P.val.assign(pv[l], pv[l] + pp[l][P.n]);
    }
    // dense Cholesky of the coarsest operator
    const Csr& K0 = M->lev[0].K;
    const int64_t n0 = K0.n;
    M->n0 = n0;
    M->chol.assign(n0 * n0, 0.0);
    for (int64_t i = 0; i < n0; ++i)
        for (int64_t k = K0.ptr[i]; k < K0.ptr[i + 1]; ++k) M->chol[i * n0 + K0.col[k]] = K0.val[k];
    std::vector<double>& A = M->chol;
    for (int64_t j = 0; j < n0; ++j) {
        double d = A[j * n0 + j];
        for (int64_t k = 0; k < j; ++k) d -= A[j * n0 + k] * A[j * n0 + k];
        const double ljj = std::sqrt(d);
        A[j * n0 + j] = ljj;
#pragma omp parallel for schedule(static) if (n0 - j > 512)
        for (int64_t i = j + 1; i < n0; ++i) {
            double s = A[i * n0 + j];
            for (int64_t k = 0; k < j; ++k) s -= A[i * n0 + k] * A[j * n0 + k];
            A[i * n0 + j] = s / ljj;
        }
    }
    return M;
}

void orc_mgpis_destroy(void* h) { delete static_cast<Mgpis*>(h); }

void orc_mult_vcyc(void* h, const double* r, double* z) {
    const Mgpis& M = *static_cast<Mgpis*>(h);
    const int L = (int)M.lev.size() - 1;
    std::vector<double> x(M.lev[L].K.n, 0.0);
    M.vcycle(L, r, x);
    std::copy(x.begin(), x.end(), z);
}

void orc_spmv(void* h, int level, const double* x, double* y) {
    static_cast<Mgpis*>(h)->lev[level].K.spmv(x, y);
}

// MGPIS::CG_SOLV (MGPIS.h:163-225).  prec 0: diagonal, 1: SGS V-cycle.  Returns iterNumb.
int64_t orc_cg_solv(void* h, int prec, const double* b, double* xout, double rtol, int64_t maxit, double* relres) {
    const Mgpis& M = *static_cast<Mgpis*>(h);
    const int L = (int)M.lev.size() - 1;
    const Level& F = M.lev[L];
    const int64_t n = F.K.n;
    std::vector<double> x(n, 0.0), r(b, b + n), p(n, 0.0), q(n), z(n);
    double bn = 0.0;
    for (int64_t i = 0; i < n; ++i) bn += b[i] * b[i];
    bn = std::sqrt(bn);
    const double tol = rtol * bn;
    auto precond = [&](const std::vector<double>& rr, std::vector<double>& out) {
        if (prec == 0)
            for (int64_t i = 0; i < n; ++i) out[i] = (1.0 / F.D[i]) * rr[i];
        else {
            std::fill(out.begin(), out.end(), 0.0);
            M.vcycle(L, rr.data(), out);
        }
    };
    precond(r, p);
    double delta = dot(r, p);
    int64_t it = 0;
    while (it < maxit && std::sqrt(dot(r, r)) > tol) {
        F.K.spmv(p.data(), q.data());
        const double alpha = delta / dot(p, q);
        for (int64_t i = 0; i < n; ++i) {
            x[i] = x[i] + alpha * p[i];
            r[i] = r[i] - alpha * q[i];
        }
        precond(r, z);
        const double dold = delta;
        delta = dot(r, z);
        const double beta = delta / dold;
        for (int64_t i = 0; i < n; ++i) p[i] = z[i] + beta * p[i];
        ++it;
    }
    std::copy(x.begin(), x.end(), xout);
    if (relres) *relres = bn > 0 ? std::sqrt(dot(r, r)) / bn : 0.0;
    return it;
}

int orc_num_threads(void) { return omp_get_max_threads(); }

}  // extern "C"

// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// CPU restatement of the reference's MGPIS (MGPIS.h) on its own data layout (condensed scalar
// CSR per level, realProl[l] CSR), used only by tests/ and bench.py's cpu_baseline leg as the
// checker.  Pinned against the reference's golden vectors (tests/test_oracle.py): one SGS
// V-cycle application (vcycle_z), CG_SOLV(1) / CG_SOLV(0) solutions and iteration counts.
//   orc_mult_vcyc   MGPIS::MULT_VCYC  MGPIS.h:55-128  (symmetric Gauss-Seidel V(1,1))
//   orc_cg_solv     MGPIS::CG_SOLV    MGPIS.h:163-225 (x0 = 0, rtol on the recursive residual)
//   orc_mult_solv   MGPIS::MULT_SOLV  MGPIS.h:130-160 (V-cycles from x, 5-residual stagnation stop)
//   orc_bicgstab    MGPIS::BiCGSTAB_SOLV MGPIS.h:350-432
//   orc_gmres       MGPIS::GMRES_SOLV MGPIS.h:228-348 (left-preconditioned GMRES(10), classical
//                   Gram-Schmidt Arnoldi, Gram-Schmidt QR of the Hessenberg, true-residual stop)
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

// shared by the three drivers below
static void orc_precond(const Mgpis& M, int prec, const std::vector<double>& r, std::vector<double>& z) {
    const int L = (int)M.lev.size() - 1;
    const Level& F = M.lev[L];
    if (prec == 0)
        for (size_t i = 0; i < r.size(); ++i) z[i] = (1.0 / F.D[i]) * r[i];
    else {
        std::fill(z.begin(), z.end(), 0.0);
        M.vcycle(L, r.data(), z);
    }
}

// VECT_MEDI_OSCI (PREP.h:147-153): median := (max + min) / 2, oscillation := max - min
static void medi_osci(const std::vector<double>& v, double& medi, double& osci) {
    const double mx = *std::max_element(v.begin(), v.end()), mn = *std::min_element(v.begin(), v.end());
    medi = (mx + mn) / 2.0;
    osci = mx - mn;
}

// MGPIS::MULT_SOLV (MGPIS.h:130-160): x0 = 0, repeated V-cycles on (b, x) until the last five
// residual norms oscillate by less than 0.1 of their median.  Returns iterNumb at exit.
int64_t orc_mult_solv(void* h, const double* b, double* xout, int64_t maxit, double* relres) {
    const Mgpis& M = *static_cast<Mgpis*>(h);
    const int L = (int)M.lev.size() - 1;
    const Level& F = M.lev[L];
    const int64_t n = F.K.n;
    std::vector<double> x(n, 0.0), kx(n), r(n), moni(5, 0.0);
    int64_t it = 0;
    double rn = 0.0;
    while (it < maxit) {
        M.vcycle(L, b, x);
        F.K.spmv(x.data(), kx.data());
        for (int64_t i = 0; i < n; ++i) r[i] = b[i] - kx[i];
        rn = std::sqrt(dot(r, r));
        moni[it % 5] = rn;
        if (it >= 4) {
            double medi, osci;
            medi_osci(moni, medi, osci);
            if (osci < 0.1 * medi) break;
        }
        ++it;
    }
    std::copy(x.begin(), x.end(), xout);
    double bn = 0.0;
    for (int64_t i = 0; i < n; ++i) bn += b[i] * b[i];
    if (relres) *relres = bn > 0 ? rn / std::sqrt(bn) : 0.0;
    return it;
}

// MGPIS::BiCGSTAB_SOLV (MGPIS.h:350-432): right-preconditioned BiCGSTAB, x0 = 0, shadow residual
// = r0, stop on the recursive residual.  Returns iterNumb at exit.
int64_t orc_bicgstab(void* h, int prec, const double* b, double* xout, double rtol, int64_t maxit, double* relres,
                     int* breakdown) {
    const Mgpis& M = *static_cast<Mgpis*>(h);
    const Level& F = M.lev.back();
    const int64_t n = F.K.n;
    std::vector<double> x(n, 0.0), r(b, b + n), rh(b, b + n), p(n, 0.0), v(n, 0.0), ph(n), s(n), sh(n), t(n);
    const double tol = rtol * std::sqrt(dot(r, r));
    double rho[2] = {0.0, 0.0}, alph = 0.0, omeg = 0.0;
    int64_t it = 0;
    if (breakdown) *breakdown = 0;
    while (it < maxit && std::sqrt(dot(r, r)) > tol) {
        double& rc = rho[(it + 1) % 2];
        rc = dot(rh, r);
        if (std::fabs(rc) == 0.0) {  // the reference's "ERROR 1" exit (MGPIS.h:386-389)
            if (breakdown) *breakdown = 1;
            break;
        }
        if (it == 0)
            p = r;
        else {
            const double beta = (rc / rho[it % 2]) * (alph / omeg);
            for (int64_t i = 0; i < n; ++i) p[i] = r[i] + beta * (p[i] - omeg * v[i]);
        }
        orc_precond(M, prec, p, ph);
        F.K.spmv(ph.data(), v.data());
        alph = rc / dot(rh, v);
        for (int64_t i = 0; i < n; ++i) s[i] = r[i] - alph * v[i];
        if (std::sqrt(dot(s, s)) <= 0.0) {
            for (int64_t i = 0; i < n; ++i) x[i] += alph * ph[i];
            break;
        }
        orc_precond(M, prec, s, sh);
        F.K.spmv(sh.data(), t.data());
        omeg = dot(t, s) / dot(t, t);
        for (int64_t i = 0; i < n; ++i) {
            x[i] += alph * ph[i] + omeg * sh[i];
            r[i] = s[i] - omeg * t[i];
        }
        ++it;
    }
    std::copy(x.begin(), x.end(), xout);
    const double bn = std::sqrt(dot(rh, rh));
    if (relres) *relres = bn > 0 ? std::sqrt(dot(r, r)) / bn : 0.0;
    return it;
}

// MGPIS::GMRES_SOLV (MGPIS.h:228-348): GMRES(restart) on M^-1 K, x0 = 0.  Per restart cycle the
// basis starts at M^-1 (b - K x0) / ||.||; each step appends one Arnoldi vector (one classical
// Gram-Schmidt pass), extends the Gram-Schmidt QR of the Hessenberg by one column, solves
// R y = ||M^-1 r0|| Q(0,:)^T and forms x = x0 + V y; the stop test is on the true residual
// ||b - K x|| over a window of `restart` values: <= tol, or <= 100 tol with an oscillation below
// 0.1 of the median.  Returns iterNumb at exit.
int64_t orc_gmres(void* h, int prec, const double* b, double* xout, double rtol, int64_t maxit, int64_t restart,
                  double* relres) {
    const Mgpis& M = *static_cast<Mgpis*>(h);
    const Level& F = M.lev.back();
    const int64_t n = F.K.n;
    const int64_t m = restart;
    std::vector<double> x(n, 0.0), x0(n), r(n), pr(n), kv(n), pv(n), kx(n), moni(m, 0.0);
    std::vector<std::vector<double>> V;
    std::vector<double> H, Q, R;  // column-major, leading dimension m + 1
    const int64_t ld = m + 1;
    double bn = 0.0;
    for (int64_t i = 0; i < n; ++i) bn += b[i] * b[i];
    bn = std::sqrt(bn);
    const double tol = rtol * bn;
    double nr0 = 0.0, rn = 0.0;
    int64_t it = 0;
    while (it < maxit) {
        const int64_t j = it % m;
        if (j == 0) {
            x0 = x;
            F.K.spmv(x0.data(), kx.data());
            for (int64_t i = 0; i < n; ++i) r[i] = b[i] - kx[i];
            orc_precond(M, prec, r, pr);
            nr0 = std::sqrt(dot(pr, pr));
            V.assign(1, pr);
            for (double& e : V[0]) e /= nr0;
            H.assign(ld * m, 0.0);
            Q.assign(ld * m, 0.0);
            R.assign(ld * m, 0.0);
        }
        F.K.spmv(V[j].data(), kv.data());
        orc_precond(M, prec, kv, pv);
        std::vector<double> bi(j + 1);
        for (int64_t k = 0; k <= j; ++k) bi[k] = dot(V[k], pv);
        std::vector<double> q(pv);
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = 0; k <= j; ++k) s += V[k][i] * bi[k];
            q[i] -= s;
        }
        const double nq = std::sqrt(dot(q, q));
        for (int64_t k = 0; k <= j; ++k) H[j * ld + k] = bi[k];
        H[j * ld + j + 1] = nq;
        for (double& e : q) e /= nq;
        V.push_back(q);
        if (j == 0) {
            const double hn = std::sqrt(H[0] * H[0] + H[1] * H[1]);
            Q[0] = H[0] / hn;
            Q[1] = H[1] / hn;
            R[0] = hn;
        } else {
            // R(0:j, j) = Q(:, 0:j)^T H(:, j) over j + 2 rows (new row of Q is zero)
            for (int64_t c = 0; c < j; ++c) {
                double s = 0.0;
                for (int64_t k = 0; k <= j + 1; ++k) s += Q[c * ld + k] * H[j * ld + k];
                R[j * ld + c] = s;
            }
            double qq = 0.0;
            for (int64_t k = 0; k <= j + 1; ++k) {
                double s = 0.0;
                for (int64_t c = 0; c < j; ++c) s += Q[c * ld + k] * R[j * ld + c];
                Q[j * ld + k] = H[j * ld + k] - s;
                qq += Q[j * ld + k] * Q[j * ld + k];
            }
            const double rjj = std::sqrt(qq);
            R[j * ld + j] = rjj;
            for (int64_t k = 0; k <= j + 1; ++k) Q[j * ld + k] /= rjj;
        }
        std::vector<double> y(j + 1, 0.0);
        for (int64_t t = j; t >= 0; --t) {
            double s = 0.0;
            for (int64_t c = t + 1; c <= j; ++c) s += R[c * ld + t] * y[c];
            y[t] = (nr0 * Q[t * ld + 0] - s) / R[t * ld + t];
        }
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = 0; k <= j; ++k) s += V[k][i] * y[k];
            x[i] = x0[i] + s;
        }
        F.K.spmv(x.data(), kx.data());
        for (int64_t i = 0; i < n; ++i) r[i] = b[i] - kx[i];
        rn = std::sqrt(dot(r, r));
        moni[it % m] = rn;
        if (it >= m - 1) {
            double medi, osci;
            medi_osci(moni, medi, osci);
            if (rn <= tol || (rn <= 1e2 * tol && osci < 0.1 * medi)) break;
        }
        ++it;
    }
    std::copy(x.begin(), x.end(), xout);
    if (relres) *relres = bn > 0 ? rn / bn : 0.0;
    return it;
}

int orc_num_threads(void) { return omp_get_max_threads(); }

// y (+)= A x for a scalar CSR, OpenMP over rows like Eigen's row-major product
// (SparseDenseProduct.h:47-57): the interface-step products of bench.py's CPU baseline
// (MCONTACT.h:2520-2521, 2632-2704)
void orc_csr_matvec(int64_t nrow, const int64_t* ptr, const int32_t* col, const double* val, const double* x,
                    double* y, int accumulate) {
#pragma omp parallel for schedule(static, 1024)
    for (int64_t r = 0; r < nrow; ++r) {
        double s = 0.0;
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) s += val[k] * x[col[k]];
        y[r] = accumulate ? y[r] + s : s;
    }
}

}  // extern "C"

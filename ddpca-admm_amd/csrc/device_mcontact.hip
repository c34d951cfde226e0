// MCONTACT device path: the ADMM loop of CONTACT_ANALYSIS (MCONTACT.h:2493-2723) for the
// subdomains and interface sides owned by one rank (one process per GPU).
//
// Per iteration (same data flow as the reference):
//   body balance   b_tv = consForc + consOper (systTran_pena aux - systTran lambda)   (2514-2524)
//                  u_tv = OUTP_SUB1(MGPIS PCG(b_tv))                                 (2531-2533)
//                  -- all owned subdomains solve concurrently, one HIP stream each
//   interface      gamma = 1/2 (L0 l0 - L1 l1 + R0 u0 - R1 u1 - pema g)              (2632-2636)
//                  -- each side contributes its half; sides on different ranks swap their
//                     halves with one RCCL send/recv pair over xGMI (no global collective)
//                  normal / Coulomb projection                                        (2637-2668)
//                  aux = (M^rho)^-1 (T^T u + M l + I gamma)                           (2671-2684)
//   Lagrange       l += M^-1 (T^T u - M^rho aux)                                      (2689-2704)
//   MONITOR        squared norms reduced on device, one small RCCL all-reduce,
//                  reference stopping logic on the host                               (2725-2845)
// The surface mass solves (LDLT in the reference, < 120000 rows) run as a batched Jacobi-PCG,
// one workgroup per system, to a 1e-14 relative residual.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>

#include "../../include/ddpca_amd.h"
#include "device_mgpis.hpp"
#include "problem.hpp"

using namespace ddpca;

namespace {

#define DDPCA_NCCL(call)                                                                                  \
    do {                                                                                                  \
        ncclResult_t r_ = (call);                                                                         \
        if (r_ != ncclSuccess) throw ApiError(DDPCA_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

struct DevCsr {
    int64_t nrow = 0, ncol = 0;
    DevBuf<int64_t> ptr;
    DevBuf<int32_t> col;
    DevBuf<double> val;
    void upload(const Csr& m) {
        nrow = m.nrow;
        ncol = m.ncol;
        ptr.upload(m.ptr);
        col.upload(m.col);
        val.upload(m.val);
    }
};

Csr transpose(const Csr& A) {
    Csr T;
    T.nrow = A.ncol;
    T.ncol = A.nrow;
    T.ptr.assign(T.nrow + 1, 0);
    for (int32_t c : A.col) T.ptr[c + 1]++;
    for (int64_t r = 0; r < T.nrow; ++r) T.ptr[r + 1] += T.ptr[r];
    T.col.resize(A.col.size());
    T.val.resize(A.val.size());
    std::vector<int64_t> fill(T.ptr.begin(), T.ptr.end() - 1);
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t p = fill[A.col[k]]++;
            T.col[p] = (int32_t)r;
            T.val[p] = A.val[k];
        }
    return T;
}

// ------------------------------------------------------------------------------- kernels
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double csr_row(const int64_t* ptr, const int32_t* col, const double* val, const double* x,
                                          int64_t r) {
    double s = 0.0;
    for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) s += val[k] * x[col[k]];
    return s;
}

// b[rows[i]] += sum_k val[k] state[col[k]]  (coupling of the body-balance RHS)
__global__ void k_cpl(const int32_t* rows, const int64_t* ptr, const int32_t* col, const double* val,
                      const double* state, double* b, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    b[rows[i]] += csr_row(ptr, col, val, state, i);
}

// u = mask ? x : prescribed  (OUTP_SUB1 without rotations)
__global__ void k_outp(const double* x, const uint8_t* mask, const double* presc, double* u, int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const uint8_t m = mask[i];
    for (int a = 0; a < 3; ++a) u[3 * i + a] = ((m >> a) & 1) ? x[3 * i + a] : presc[3 * i + a];
}

// gamma_seg += sgn/2 (L lambda + R u) + cst
__global__ void k_gamma(const int64_t* lp, const int32_t* lc, const double* lv, const double* lam, const int64_t* rp,
                        const int32_t* rc, const double* rv, const double* u, const double* cst, double sgn,
                        double* gam, int64_t mip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= mip) return;
    const double c = 0.5 * sgn * (csr_row(lp, lc, lv, lam, i) + csr_row(rp, rc, rv, u, i));
    gam[i] += cst ? c + cst[i] : c;
}

__global__ void k_add(double* y, const double* x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] += x[i];
}

// normal / Coulomb projection at integration points (MCONTACT.h:2637-2668)
__global__ void k_project(double* g, int32_t* stat, int64_t nip, int comp, double fric) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nip) return;
    if (comp == 1) {
        g[q] = fmax(0.0, g[q]);
        stat[q] = 0;
        return;
    }
    double* v = g + 3 * q;
    if (fric < 0.0) {
        stat[q] = 0;
        return;
    }
    v[0] = fmax(0.0, v[0]);
    if (fric == 0.0) {
        stat[q] = 0;
        return;
    }
    if (v[0] > 0.0) {
        const double slid = fric * v[0];
        const double nt = sqrt(v[1] * v[1] + v[2] * v[2]);
        if (nt >= slid) {
            v[1] = slid / nt * v[1];
            v[2] = slid / nt * v[2];
            stat[q] = 1;
        } else {
            stat[q] = 2;
        }
    } else {
        v[1] = 0.0;
        v[2] = 0.0;
        stat[q] = 0;
    }
}

// rhs = A u + B l + C g   (B, C optional; sign sb on B)
__global__ void k_rhs3(const int64_t* ap, const int32_t* ac, const double* av, const double* u, const int64_t* bp,
                       const int32_t* bc, const double* bv, const double* l, double sb, const int64_t* cp,
                       const int32_t* cc, const double* cv, const double* g, double* rhs, int64_t m) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double s = csr_row(ap, ac, av, u, i);
    if (bp) s += sb * csr_row(bp, bc, bv, l, i);
    if (cp) s += csr_row(cp, cc, cv, g, i);
    rhs[i] = s;
}

struct MassSys {
    const int64_t* ptr;
    const int32_t* col;
    const double* val;
    const double* dinv;
    const double* b;
    double* x;     // solution (overwritten) or increment target when accumulate
    double* r;
    double* p;
    double* q;
    int64_t n;
    int accumulate;  // 1: x += solution
};

__device__ double block_sum1024(double v, double* red) {
    v = wsum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < nw; ++k) s += red[k];
    return s;
}

// Batched Jacobi-preconditioned CG, one workgroup per SPD surface-mass system.
__global__ __launch_bounds__(1024) void k_mass_cg(const MassSys* sys, double rtol, int maxit) {
    __shared__ double red[16];
    const MassSys S = sys[blockIdx.x];
    const int64_t n = S.n;
    double* xs = S.accumulate ? S.q + n : S.x;  // accumulate: solve into scratch, then add
    double rz = 0.0, bb = 0.0;
    {
        double a = 0.0, c = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const double bi = S.b[i];
            xs[i] = 0.0;
            S.r[i] = bi;
            const double zi = S.dinv[i] * bi;
            S.p[i] = zi;
            a += bi * zi;
            c += bi * bi;
        }
        rz = block_sum1024(a, red);
        bb = block_sum1024(c, red);
    }
    const double tol2 = rtol * rtol * bb;
    for (int it = 0; it < maxit && bb > 0.0; ++it) {
        __syncthreads();
        double pq = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const double qi = csr_row(S.ptr, S.col, S.val, S.p, i);
            S.q[i] = qi;
            pq += S.p[i] * qi;
        }
        pq = block_sum1024(pq, red);
        const double al = rz / pq;
        double rr = 0.0, rzn = 0.0;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            xs[i] += al * S.p[i];
            const double ri = S.r[i] - al * S.q[i];
            S.r[i] = ri;
            rr += ri * ri;
            rzn += ri * S.dinv[i] * ri;
        }
        rr = block_sum1024(rr, red);
        rzn = block_sum1024(rzn, red);
        if (rr <= tol2) break;
        const double be = rzn / rz;
        rz = rzn;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) S.p[i] = S.dinv[i] * S.r[i] + be * S.p[i];
    }
    __syncthreads();
    if (S.accumulate)
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) S.x[i] += xs[i];
}

// partial[2b], partial[2b+1] = sum (a-o)^2, sum a^2 over block b of one vector pair
__global__ void k_pair_norms(const double* a, const double* o, int64_t n, double* partial) {
    __shared__ double r1[4], r2[4];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double d = 0.0, s = 0.0;
    if (i < n) {
        const double ai = a[i], di = ai - o[i];
        d = di * di;
        s = ai * ai;
    }
    d = wsum(d);
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) {
        r1[threadIdx.x >> 6] = d;
        r2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = (r1[0] + r1[1]) + (r1[2] + r1[3]);
        partial[2 * blockIdx.x + 1] = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    }
}

__global__ void k_reduce_pairs(const double* partial, int64_t nb, double* out2) {
    __shared__ double r1[4], r2[4];
    double d = 0.0, s = 0.0;
    for (int64_t k = threadIdx.x; k < nb; k += blockDim.x) {
        d += partial[2 * k];
        s += partial[2 * k + 1];
    }
    d = wsum(d);
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) {
        r1[threadIdx.x >> 6] = d;
        r2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        out2[0] = (r1[0] + r1[1]) + (r1[2] + r1[3]);
        out2[1] = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    }
}

inline int nb256(int64_t n) { return (int)std::max<int64_t>(1, (n + 255) / 256); }

}  // namespace

// ================================================================================ handle
struct ddpca_mcontact {
    struct Sub {
        int64_t tv = 0;
        std::unique_ptr<MgpisDevice> mg;
        DevBuf<double> cf;      // consForc scattered to the nodal layout
        DevBuf<double> presc;   // prescribed dof values (nodal)
        DevBuf<double> u, uo;   // resuDisp (nodal) and previous iterate
        DevBuf<int32_t> crow;   // coupling rows (nodal dofs, free only)
        DevBuf<int64_t> cptr;
        DevBuf<int32_t> ccol;
        DevBuf<double> cval;
        int64_t ncrow = 0, nn = 0;
        int64_t last_iters = 0;
        int64_t pred_iters = 0;
    };
    struct Side {
        int64_t ts = 0, s = 0, tv = 0, m = 0, mip = 0;
        int64_t soff = 0;  // offset of [aux ; lambda] in the rank state vector
        DevCsr lagr, pemr, tTp, mass, massp, iinpo;
        DevBuf<double> dmass, dmassp, rhs, scratch;  // scratch: r, p, q, x2 (4m)
    };
    struct Itf {
        int64_t ts = 0, mip = 0, goff = 0;
        int comp = 1;
        double fric = -1.0;
        int owner[2] = {0, 0};
        bool mine = false, cross = false;
        DevBuf<double> cgap;  // -1/2 pema g (added by the side-0 owner)
        DevBuf<int32_t> stat;
        DevBuf<double> recv;
    };
    int device = 0, rank = 0, nranks = 1;
    int64_t nsub = 0, nint = 0;
    std::vector<int32_t> owner;
    std::vector<Sub> subs;
    std::vector<Side> sides;
    std::vector<Itf> itfs;
    DevBuf<double> state, state_old, gamma, partial, moni;
    DevBuf<MassSys> sys_aux, sys_lam;
    std::vector<double> moni_host;
    hipStream_t main = nullptr;
    ncclComm_t comm = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // reference MONITOR state (MCONTACT.h:2494-2498, 2725-2845)
    int64_t tc = 0;
    int64_t mult_maxi = 1000;  // PREP.h:75 (global in the reference)
    std::vector<std::vector<double>> moniReco;
    std::vector<std::vector<double>> rows;
    double timing[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<int64_t> last_pcg;
    mgpis_options_t opt{};
};

namespace {

void build(ddpca_mcontact& H, Problem& P) {
    MCONTACT& mc = P.mc;
    H.nsub = (int64_t)mc.multGrid.size();
    H.nint = (int64_t)mc.searCont.size();
    // ---- owned interface sides: state layout [aux ; lambda] per side
    int64_t soff = 0;
    std::map<std::pair<int64_t, int64_t>, size_t> side_of;
    for (int64_t ts = 0; ts < H.nint; ++ts) {
        const Interface& itf = mc.searCont[ts];
        for (int s = 0; s < 2; ++s) {
            if (H.owner[itf.body[s]] != H.rank) continue;
            ddpca_mcontact::Side sd;
            sd.ts = ts;
            sd.s = s;
            sd.tv = itf.body[s];
            sd.m = itf.mside(s);
            sd.mip = itf.mip();
            sd.soff = soff;
            soff += 2 * sd.m;
            sd.lagr.upload(itf.inpoLagr[s]);
            sd.pemr.upload(itf.pemaInpo_r[s]);
            sd.tTp.upload(transpose(itf.systTran_pena[s]));
            sd.mass.upload(itf.inteMass[s]);
            sd.massp.upload(itf.inteMass_pena[s]);
            sd.iinpo.upload(itf.inteInpo[s]);
            auto diag_inv = [](const Csr& A) {
                std::vector<double> d(A.nrow, 0.0);
                for (int64_t r = 0; r < A.nrow; ++r)
                    for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k)
                        if (A.col[k] == r) d[r] = 1.0 / A.val[k];
                return d;
            };
            sd.dmass.upload(diag_inv(itf.inteMass[s]));
            sd.dmassp.upload(diag_inv(itf.inteMass_pena[s]));
            sd.rhs.alloc(std::max<int64_t>(sd.m, 1));
            sd.scratch.alloc(std::max<int64_t>(5 * sd.m, 1));
            side_of[{ts, s}] = H.sides.size();
            H.sides.push_back(std::move(sd));
        }
    }
    H.state.alloc(std::max<int64_t>(soff, 1));
    H.state_old.alloc(std::max<int64_t>(soff, 1));
    H.state.zero(H.main);
    H.state_old.zero(H.main);
    // ---- interfaces: gamma layout (cross-rank interfaces first, then rank-local)
    int64_t goff = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int64_t ts = 0; ts < H.nint; ++ts) {
            const Interface& itf = mc.searCont[ts];
            const int o0 = H.owner[itf.body[0]], o1 = H.owner[itf.body[1]];
            const bool cross = o0 != o1;
            if ((pass == 0) != cross) continue;
            ddpca_mcontact::Itf I;
            I.ts = ts;
            I.mip = itf.mip();
            I.comp = itf.comp();
            I.fric = itf.fric;
            I.owner[0] = o0;
            I.owner[1] = o1;
            I.cross = cross;
            I.mine = (o0 == H.rank || o1 == H.rank);
            I.goff = goff;
            goff += I.mip;
            if (I.mine) {
                std::vector<double> cg(I.mip);
                for (int64_t i = 0; i < I.mip; ++i) cg[i] = -0.5 * (itf.pemaDiag[i] * itf.inpoNgap[i]);
                I.cgap.upload(cg);
                I.stat.alloc(std::max<int64_t>(I.mip / I.comp, 1));
                if (cross) I.recv.alloc(I.mip);
            }
            H.itfs.push_back(std::move(I));
        }
    std::sort(H.itfs.begin(), H.itfs.end(), [](const auto& a, const auto& b) { return a.ts < b.ts; });
    H.gamma.alloc(std::max<int64_t>(goff, 1));
    // ---- owned subdomains
    for (int64_t tv = 0; tv < H.nsub; ++tv) {
        if (H.owner[tv] != H.rank) continue;
        if (P.owned.size() != (size_t)H.nsub || !P.owned[tv])
            throw ApiError(DDPCA_ESTATE, "subdomain " + std::to_string(tv) + " is owned by this rank but was not established");
        const MULTIGRID& g = mc.multGrid[tv];
        ddpca_mcontact::Sub S;
        S.tv = tv;
        S.nn = g.numNodes();
        std::vector<int64_t> nn(g.leveCount.begin(), g.leveCount.end());
        std::vector<const Bsr3*> Bp;
        std::vector<const Stencil*> Sp;
        for (const auto& b : g.levelStif) Bp.push_back(&b);
        for (const auto& s : g.scalProl) Sp.push_back(&s);
        S.mg = std::make_unique<MgpisDevice>(H.device, nn, Bp, g.consFlag, Sp, H.opt);
        std::vector<double> cf(3 * S.nn, 0.0), pr(3 * S.nn, 0.0);
        for (int64_t d = 0; d < 3 * S.nn; ++d)
            if (g.consFlag[d]) cf[d] = g.consForc[g.freeIndex[d]];
        for (const auto& kv : g.consDofv) pr[kv.first] = kv.second;
        S.cf.upload(cf);
        S.presc.upload(pr);
        S.u.alloc(3 * S.nn);
        S.uo.alloc(3 * S.nn);
        S.u.zero(H.main);
        S.uo.zero(H.main);
        // coupling rows: sum over incident sides of [systTran_pena | -systTran] on free dofs
        std::map<int64_t, std::vector<std::pair<int32_t, double>>> rowmap;
        for (int64_t ts = 0; ts < H.nint; ++ts) {
            const Interface& itf = mc.searCont[ts];
            for (int s = 0; s < 2; ++s) {
                if (itf.body[s] != tv) continue;
                const auto& sd = H.sides[side_of.at({ts, s})];
                const Csr& Tp = itf.systTran_pena[s];
                const Csr& T = itf.systTran[s];
                for (int64_t r = 0; r < Tp.nrow; ++r) {
                    if (!g.consFlag[r]) continue;
                    for (int64_t k = Tp.ptr[r]; k < Tp.ptr[r + 1]; ++k)
                        rowmap[r].push_back({(int32_t)(sd.soff + Tp.col[k]), Tp.val[k]});
                    for (int64_t k = T.ptr[r]; k < T.ptr[r + 1]; ++k)
                        rowmap[r].push_back({(int32_t)(sd.soff + sd.m + T.col[k]), -T.val[k]});
                }
            }
        }
        std::vector<int32_t> crow;
        std::vector<int64_t> cptr{0};
        std::vector<int32_t> ccol;
        std::vector<double> cval;
        for (const auto& kv : rowmap) {
            crow.push_back((int32_t)kv.first);
            for (const auto& e : kv.second) {
                ccol.push_back(e.first);
                cval.push_back(e.second);
            }
            cptr.push_back((int64_t)ccol.size());
        }
        S.ncrow = (int64_t)crow.size();
        S.crow.upload(crow);
        S.cptr.upload(cptr);
        S.ccol.upload(ccol);
        S.cval.upload(cval);
        H.subs.push_back(std::move(S));
    }
    // ---- batched mass systems
    auto make_sys = [&](bool aux) {
        std::vector<MassSys> v;
        for (auto& sd : H.sides) {
            MassSys m{};
            const DevCsr& A = aux ? sd.massp : sd.mass;
            m.ptr = A.ptr.p;
            m.col = A.col.p;
            m.val = A.val.p;
            m.dinv = aux ? sd.dmassp.p : sd.dmass.p;
            m.b = sd.rhs.p;
            m.x = H.state.p + sd.soff + (aux ? 0 : sd.m);
            m.r = sd.scratch.p;
            m.p = sd.scratch.p + sd.m;
            m.q = sd.scratch.p + 2 * sd.m;  // accumulate mode uses q + n as the solution scratch
            m.n = sd.m;
            m.accumulate = aux ? 0 : 1;
            v.push_back(m);
        }
        return v;
    };
    H.sys_aux.upload(make_sys(true));
    H.sys_lam.upload(make_sys(false));
    int64_t maxn = 1;
    for (auto& S : H.subs) maxn = std::max(maxn, 3 * S.nn);
    for (auto& sd : H.sides) maxn = std::max(maxn, 2 * sd.m);
    H.partial.alloc(2 * nb256(maxn));
    const int64_t nmon = 2 * H.nsub + 8 * H.nint;
    H.moni.alloc(nmon);
    H.moni_host.assign(nmon, 0.0);
    H.moniReco.assign(H.nsub + 4 * H.nint, std::vector<double>(10, 0.0));
    DDPCA_HIP(hipStreamSynchronize(H.main));
}

void pair_norm(ddpca_mcontact& H, const double* a, const double* o, int64_t n, int64_t slot) {
    const int nb = nb256(n);
    hipLaunchKernelGGL(k_pair_norms, dim3(nb), dim3(256), 0, H.main, a, o, n, H.partial.p);
    hipLaunchKernelGGL(k_reduce_pairs, dim3(1), dim3(256), 0, H.main, H.partial.p, (int64_t)nb, H.moni.p + slot);
}

// Reference MONITOR (MCONTACT.h:2725-2845) on the reduced norms; true = converged.
bool monitor(ddpca_mcontact& H) {
    const int64_t cyc = 10;
    const int64_t tc = H.tc;
    bool flag0 = tc >= cyc, flag1 = true;
    const double c0 = 0.1, c1 = 1.0e-12;
    double convValu = 0.0, convCrit = 0.0;
    std::vector<double> row;
    auto medi_osci = [](const std::vector<double>& v, double& medi, double& osci) {
        const double mx = *std::max_element(v.begin(), v.end()), mn = *std::min_element(v.begin(), v.end());
        medi = (mx + mn) / 2.0;
        osci = mx - mn;
    };
    for (int64_t tv = 0; tv < H.nsub; ++tv) {
        const double d = H.moni_host[2 * tv], a = H.moni_host[2 * tv + 1];
        H.moniReco[tv][tc % cyc] = d;
        convValu += d;
        convCrit += a;
        row.push_back(d);
        row.push_back(a);
        if (tc >= cyc) {
            double me, os;
            medi_osci(H.moniReco[tv], me, os);
            if (os > c0 * me) flag0 = false;
        }
        if (d > c1 * a) flag1 = false;
    }
    for (int64_t ts = 0; ts < H.nint; ++ts)
        for (int s = 0; s < 2; ++s) {
            const double* m = &H.moni_host[2 * H.nsub + 8 * ts + 4 * s];
            const int64_t idx = H.nsub + 4 * ts + 2 * s;
            H.moniReco[idx][tc % cyc] = m[0];
            convValu += m[0];
            convCrit += m[1];
            row.insert(row.end(), {m[0], m[1], m[2], m[3]});
            if (tc >= cyc) {
                double me, os;
                medi_osci(H.moniReco[idx], me, os);
                if (os > c0 * me) flag0 = false;
            }
            if (m[0] > c1 * m[1]) flag1 = false;
            H.moniReco[idx + 1][tc % cyc] = m[2];  // lambda criteria disabled in the reference
        }
    row.push_back(convValu);
    row.push_back(convCrit);
    H.rows.push_back(row);
    if (flag0) H.mult_maxi = tc;
    return flag1;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// One ADMM iteration; returns true when MONITOR reports convergence.
bool iterate_once(ddpca_mcontact& H, bool check) {
    const auto t0 = std::chrono::steady_clock::now();
    // snapshot for MONITOR (resuDisp_0 / inteAuxi_0 / inteLagr_0, MCONTACT.h:2507-2509)
    if (H.state.n) DDPCA_HIP(hipMemcpyAsync(H.state_old.p, H.state.p, H.state.n * sizeof(double), hipMemcpyDeviceToDevice, H.main));
    DDPCA_HIP(hipEventRecord(H.ev[0], H.main));
    // ---- body balance: all owned subdomains concurrently
    for (auto& S : H.subs) {
        MgpisDevice& D = *S.mg;
        DDPCA_HIP(hipStreamWaitEvent(D.stream, H.ev[0], 0));
        std::swap(S.u.p, S.uo.p);
        DDPCA_HIP(hipMemcpyAsync(D.bs.p, S.cf.p, 3 * S.nn * sizeof(double), hipMemcpyDeviceToDevice, D.stream));
        if (S.ncrow)
            hipLaunchKernelGGL(k_cpl, dim3(nb256(S.ncrow)), dim3(256), 0, D.stream, S.crow.p, S.cptr.p, S.ccol.p, S.cval.p,
                               H.state.p, D.bs.p, S.ncrow);
        D.pcg_begin(1, 1.0e-14, D.nfree);
        // pre-enqueue the predicted number of graph replays
        const int64_t k = std::max(1, D.opt.iters_per_graph);
        const int64_t pre = S.pred_iters > 0 ? std::max<int64_t>(1, S.pred_iters / k) : 1;
        for (int64_t r = 0; r < pre; ++r) D.pcg_step(1);
    }
    std::vector<bool> done(H.subs.size(), false);
    size_t left = H.subs.size();
    while (left) {
        for (size_t i = 0; i < H.subs.size(); ++i) {
            if (done[i]) continue;
            MgpisDevice& D = *H.subs[i].mg;
            if (D.pcg_poll()) {
                done[i] = true;
                --left;
                if (D.sc_host->fail) throw ApiError(DDPCA_ENUMERIC, "subdomain PCG breakdown");
                H.subs[i].last_iters = D.sc_host->iter;
                H.subs[i].pred_iters = D.sc_host->iter;
            } else {
                D.pcg_step(1);
            }
        }
    }
    for (auto& S : H.subs) {
        MgpisDevice& D = *S.mg;
        hipLaunchKernelGGL(k_outp, dim3(nb256(S.nn)), dim3(256), 0, D.stream, D.xs.p, D.lev.back().mask.p, S.presc.p,
                           S.u.p, S.nn);
        DDPCA_HIP(hipEventRecord(H.ev[1], D.stream));
        DDPCA_HIP(hipStreamWaitEvent(H.main, H.ev[1], 0));
    }
    DDPCA_HIP(hipEventRecord(H.ev[1], H.main));
    const double t_solve = ms_since(t0);
    // ---- interface balance: gamma contributions of owned sides
    if (H.gamma.n) DDPCA_HIP(hipMemsetAsync(H.gamma.p, 0, H.gamma.n * sizeof(double), H.main));
    auto sub_u = [&](int64_t tv) -> const double* {
        for (auto& S : H.subs)
            if (S.tv == tv) return S.u.p;
        return nullptr;
    };
    for (auto& sd : H.sides) {
        const auto& I = *std::find_if(H.itfs.begin(), H.itfs.end(), [&](const auto& x) { return x.ts == sd.ts; });
        hipLaunchKernelGGL(k_gamma, dim3(nb256(sd.mip)), dim3(256), 0, H.main, sd.lagr.ptr.p, sd.lagr.col.p,
                           sd.lagr.val.p, H.state.p + sd.soff + sd.m, sd.pemr.ptr.p, sd.pemr.col.p, sd.pemr.val.p,
                           sub_u(sd.tv), sd.s == 0 ? I.cgap.p : nullptr, sd.s == 0 ? 1.0 : -1.0, H.gamma.p + I.goff,
                           sd.mip);
    }
    const auto tc0 = std::chrono::steady_clock::now();
    bool any_cross = false;
    for (auto& I : H.itfs) any_cross |= (I.cross && I.mine);
    if (any_cross) {
        if (!H.comm) throw ApiError(DDPCA_ESTATE, "cross-rank interfaces need mcontact_gpu_comm_init");
        DDPCA_NCCL(ncclGroupStart());
        for (auto& I : H.itfs) {
            if (!(I.cross && I.mine)) continue;
            const int peer = I.owner[0] == H.rank ? I.owner[1] : I.owner[0];
            DDPCA_NCCL(ncclSend(H.gamma.p + I.goff, I.mip, ncclDouble, peer, H.comm, H.main));
            DDPCA_NCCL(ncclRecv(I.recv.p, I.mip, ncclDouble, peer, H.comm, H.main));
        }
        DDPCA_NCCL(ncclGroupEnd());
        for (auto& I : H.itfs)
            if (I.cross && I.mine)
                hipLaunchKernelGGL(k_add, dim3(nb256(I.mip)), dim3(256), 0, H.main, H.gamma.p + I.goff, I.recv.p, I.mip);
    }
    DDPCA_HIP(hipEventRecord(H.ev[2], H.main));
    for (auto& I : H.itfs)
        if (I.mine)
            hipLaunchKernelGGL(k_project, dim3(nb256(I.mip / I.comp)), dim3(256), 0, H.main, H.gamma.p + I.goff, I.stat.p,
                               I.mip / I.comp, I.comp, I.fric);
    // ---- aux = (M^rho)^-1 (T^T u + M lambda + I gamma)
    for (auto& sd : H.sides) {
        const auto& I = *std::find_if(H.itfs.begin(), H.itfs.end(), [&](const auto& x) { return x.ts == sd.ts; });
        hipLaunchKernelGGL(k_rhs3, dim3(nb256(sd.m)), dim3(256), 0, H.main, sd.tTp.ptr.p, sd.tTp.col.p, sd.tTp.val.p,
                           sub_u(sd.tv), sd.mass.ptr.p, sd.mass.col.p, sd.mass.val.p, H.state.p + sd.soff + sd.m, 1.0,
                           sd.iinpo.ptr.p, sd.iinpo.col.p, sd.iinpo.val.p, H.gamma.p + I.goff, sd.rhs.p, sd.m);
    }
    if (!H.sides.empty()) hipLaunchKernelGGL(k_mass_cg, dim3(H.sides.size()), dim3(1024), 0, H.main, H.sys_aux.p, 1.0e-14, 2000);
    // ---- lambda += M^-1 (T^T u - M^rho aux)
    for (auto& sd : H.sides)
        hipLaunchKernelGGL(k_rhs3, dim3(nb256(sd.m)), dim3(256), 0, H.main, sd.tTp.ptr.p, sd.tTp.col.p, sd.tTp.val.p,
                           sub_u(sd.tv), sd.massp.ptr.p, sd.massp.col.p, sd.massp.val.p, H.state.p + sd.soff, -1.0,
                           nullptr, nullptr, nullptr, nullptr, sd.rhs.p, sd.m);
    if (!H.sides.empty()) hipLaunchKernelGGL(k_mass_cg, dim3(H.sides.size()), dim3(1024), 0, H.main, H.sys_lam.p, 1.0e-14, 2000);
    // ---- MONITOR norms (owned entries; others zero) and their reduction across ranks
    DDPCA_HIP(hipMemsetAsync(H.moni.p, 0, H.moni.n * sizeof(double), H.main));
    for (auto& S : H.subs) pair_norm(H, S.u.p, S.uo.p, 3 * S.nn, 2 * S.tv);
    for (auto& sd : H.sides) {
        const int64_t base = 2 * H.nsub + 8 * sd.ts + 4 * sd.s;
        pair_norm(H, H.state.p + sd.soff, H.state_old.p + sd.soff, sd.m, base);
        pair_norm(H, H.state.p + sd.soff + sd.m, H.state_old.p + sd.soff + sd.m, sd.m, base + 2);
    }
    if (H.nranks > 1) DDPCA_NCCL(ncclAllReduce(H.moni.p, H.moni.p, H.moni.n, ncclDouble, ncclSum, H.comm, H.main));
    DDPCA_HIP(hipEventRecord(H.ev[3], H.main));
    DDPCA_HIP(hipMemcpyAsync(H.moni_host.data(), H.moni.p, H.moni.n * sizeof(double), hipMemcpyDeviceToHost, H.main));
    DDPCA_HIP(hipStreamSynchronize(H.main));
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, H.ev[1], H.ev[3]);
    (void)hipEventElapsedTime(&b, H.ev[1], H.ev[2]);
    H.timing[0] += ms_since(t0);
    H.timing[1] += t_solve;
    H.timing[2] += a;
    H.timing[3] += any_cross ? b : 0.0;
    (void)tc0;
    for (auto& S : H.subs) {
        H.timing[6] += (double)S.last_iters;
        H.timing[8] += (double)S.last_iters * (double)S.mg->nfree;
        if (S.mg->timed_kernel_samples) {
            H.timing[7] += S.mg->fine_kernel_bytes() * (double)S.mg->timed_kernel_samples;
            H.timing[4] += S.mg->timed_kernel_ms;
            H.timing[5] += (double)S.mg->timed_kernel_samples;
            S.mg->timed_kernel_ms = 0.0;
            S.mg->timed_kernel_samples = 0;
        }
    }
    const bool conv = monitor(H);
    H.tc += 1;
    return check && conv;
}

}  // namespace

extern "C" {

int mcontact_gpu_create(ddpca_problem_t p, int device, int rank, int nranks, const int32_t* owner,
                        const mgpis_options_t* opt, mcontact_t* out) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (!P.established) throw ApiError(DDPCA_ESTATE, "problem not established");
        if (nranks < 1 || rank < 0 || rank >= nranks || !owner || !out) throw ApiError(DDPCA_EINVAL, "rank/owner");
        select_device(device);
        auto H = std::make_unique<ddpca_mcontact>();
        H->device = device;
        H->rank = rank;
        H->nranks = nranks;
        H->owner.assign(owner, owner + P.mc.multGrid.size());
        for (int32_t o : H->owner)
            if (o < 0 || o >= nranks) throw ApiError(DDPCA_EINVAL, "owner out of range");
        if (opt) H->opt = *opt;
        else mgpis_default_options(&H->opt);
        DDPCA_HIP(hipStreamCreateWithFlags(&H->main, hipStreamNonBlocking));
        for (auto& e : H->ev) DDPCA_HIP(hipEventCreate(&e));
        build(*H, P);
        *out = H.release();
    });
}

int mcontact_gpu_unique_id(void* out128) {
    return guarded([&] {
        ncclUniqueId id;
        DDPCA_NCCL(ncclGetUniqueId(&id));
        std::memcpy(out128, &id, sizeof(id));
    });
}

int mcontact_gpu_comm_init(mcontact_t h, const void* uid) {
    return guarded([&] {
        select_device(h->device);
        if (h->nranks == 1) return;
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        DDPCA_NCCL(ncclCommInitRank(&h->comm, h->nranks, id, h->rank));
    });
}

int64_t mcontact_gpu_iterate(mcontact_t h, int64_t maxit, int check) {
    int64_t n = 0;
    const int rc = guarded([&] {
        select_device(h->device);
        for (double& t : h->timing) t = 0.0;
        for (auto& S : h->subs) S.mg->time_kernel = true;
        for (; n < maxit;) {
            const bool conv = iterate_once(*h, check != 0);
            ++n;
            if (conv) break;
        }
    });
    return rc < 0 ? rc : n;
}

int64_t mcontact_gpu_monitor(mcontact_t h, double* out, int64_t cap_rows) {
    const int64_t rows = (int64_t)h->rows.size();
    if (!out) return rows;
    const int64_t ncol = 2 * h->nsub + 8 * h->nint + 2;
    for (int64_t r = 0; r < std::min(rows, cap_rows); ++r) std::memcpy(out + r * ncol, h->rows[r].data(), ncol * sizeof(double));
    return std::min(rows, cap_rows);
}

int64_t mcontact_gpu_get(mcontact_t h, const char* what, int64_t index, void* out, int64_t cap) {
    int64_t n = 0;
    const int rc = guarded([&] {
        select_device(h->device);
        const std::string w(what);
        DDPCA_HIP(hipStreamSynchronize(h->main));
        if (w == "resuDisp") {
            for (auto& S : h->subs)
                if (S.tv == index) {
                    n = 3 * S.nn;
                    if (out) DDPCA_HIP(hipMemcpy(out, S.u.p, std::min(n, cap) * sizeof(double), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "subdomain not owned by this rank");
        }
        if (w == "inteAuxi" || w == "inteLagr") {
            for (auto& sd : h->sides)
                if (2 * sd.ts + sd.s == index) {
                    n = sd.m;
                    const double* src = h->state.p + sd.soff + (w == "inteAuxi" ? 0 : sd.m);
                    if (out) DDPCA_HIP(hipMemcpy(out, src, std::min(n, cap) * sizeof(double), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "interface side not owned by this rank");
        }
        if (w == "inpoGamm") {
            for (auto& I : h->itfs)
                if (I.ts == index && I.mine) {
                    n = I.mip;
                    if (out) DDPCA_HIP(hipMemcpy(out, h->gamma.p + I.goff, std::min(n, cap) * sizeof(double), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "interface not handled by this rank");
        }
        if (w == "pcg_iters") {
            n = (int64_t)h->subs.size();
            if (out)
                for (int64_t i = 0; i < std::min(n, cap); ++i) static_cast<int64_t*>(out)[i] = h->subs[i].last_iters;
            return;
        }
        if (w == "owned") {
            n = (int64_t)h->subs.size();
            if (out)
                for (int64_t i = 0; i < std::min(n, cap); ++i) static_cast<int64_t*>(out)[i] = h->subs[i].tv;
            return;
        }
        throw ApiError(DDPCA_EINVAL, "unknown quantity " + w);
    });
    return rc < 0 ? rc : n;
}

int mcontact_gpu_timing(mcontact_t h, double* out10) {
    std::memcpy(out10, h->timing, sizeof(h->timing));
    if (h->timing[5] > 0) out10[7] = h->timing[7] / h->timing[5];  // bytes per timed launch
    double dofs = 0.0;
    for (auto& S : h->subs) dofs += (double)S.mg->nfree;
    out10[9] = dofs;
    return DDPCA_OK;
}

int mcontact_gpu_destroy(mcontact_t h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        if (h->main) (void)hipStreamSynchronize(h->main);
        if (h->comm) (void)ncclCommDestroy(h->comm);
        for (auto& e : h->ev)
            if (e) (void)hipEventDestroy(e);
        h->subs.clear();
        if (h->main) (void)hipStreamDestroy(h->main);
        delete h;
    });
}

}  // extern "C"

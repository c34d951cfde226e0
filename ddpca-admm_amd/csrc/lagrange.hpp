// MCONTACT::LAGRANGE (MCONTACT.h:2847-3701): the monolithic dual-mortar Lagrange-multiplier
// contact solver with a semi-smooth Newton active set -- the reference's alternative to the ADMM
// loop.  Host assembly restated here (lagrange.cpp); the linear solve of every Newton step (the
// condensed, generally nonsymmetric system) runs as MGPIS-preconditioned BiCGSTAB on the device
// (capi_lagrange.hip) through the `Solve` callback.
#pragma once
#include <array>
#include <functional>
#include <map>
#include <vector>

#include "sparse.hpp"

namespace ddpca {

// One subdomain as LAGRANGE reads it after TRANSFER / STIF_MATR / CONSTRAINT (MCONTACT.h:2851-2860)
struct LagrangeSub {
    int nlev = 0;
    std::vector<int64_t> nnodes, nfree;          // per level (level-ordered numbering)
    std::vector<std::vector<int32_t>> free_dof;  // per level: condensed index -> nodal dof (increasing)
    std::vector<Csr> K;                          // mgpi.consStif[l]
    std::vector<Csr> P;                          // mgpi.realProl[l], l < nlev - 1
    std::vector<double> consForc;
    int64_t nall = 0;         // nodes of the node-id numbering (nodeCoor.size())
    Csr G;                    // 3 nall x nfree[L]: earlTran prolOper[L] consOper[L]^T (MCONTACT.h:3086-3088)
    std::vector<uint8_t> hanging;  // per node id: on level maxiLeve + 1 (nodeLepo, MCONTACT.h:2880)
};

struct LagrangeIp {  // INTEGRAL_POINT (CSEARCH.h:19-32) + its dual shape values
    int64_t node[2][4];
    double shap[2][4];
    double basis[3][3];  // basiVect[0..2] (normal first)
    double gap = 0.0, w = 0.0;
    double dual[4] = {0, 0, 0, 0};
};

struct LagrangeItf {
    int64_t body[2] = {0, 0};
    double fric = 0.0;  // < 0 glued (no active-set update), 0 frictionless, > 0 Coulomb
    std::vector<LagrangeIp> ips;
};

// the condensed system of one Newton step and the MGPIS hierarchy the reference builds for it
// (MCONTACT.h:3419-3561): K[l], realProl[l] over the non-condensed dofs of every subdomain, in the
// reference's order (subdomain-major, increasing condensed index); dofs[l][r] = (tv, condensed
// index on level l) of hierarchy row r
struct LagrangeSystem {
    std::vector<Csr> K, P;
    std::vector<double> F;
    std::vector<std::vector<std::pair<int32_t, int32_t>>> dofs;
};

// solve K[L] x = F to the reference's BiCGSTAB stop rule; returns the iteration count
using LagrangeSolve = std::function<int64_t(const LagrangeSystem&, std::vector<double>& x)>;

struct LagrangeResult {
    int64_t newton = 0;  // tc at convergence (the reference's "Converge after tc-th iteration")
    bool converged = false;
    std::vector<int64_t> solver_iters;        // per Newton step
    std::vector<int64_t> changes;             // per Newton step: seneNumb
    std::vector<std::vector<double>> u;       // per subdomain: condensed displacement (slidDisp)
    // per interface, non-mortar nodes in the reference's (body, node) key order
    std::vector<std::vector<int64_t>> node, status;
    std::vector<std::vector<double>> lambda;  // 3 per node: (n, t1, t2) multiplier, resuLagr
    std::vector<std::vector<double>> wedi;    // 3 per node: nmnoWedi (relative displacement, gap)
};

LagrangeResult run_lagrange(std::vector<LagrangeSub>& subs, std::vector<LagrangeItf>& itfs, int64_t max_newton,
                            const LagrangeSolve& solve);

}  // namespace ddpca

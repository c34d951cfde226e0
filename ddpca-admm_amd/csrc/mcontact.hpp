// MCONTACT: host restatement of the reference's interface operator assembly
// (MCONTACT::ESTABLISH, MCONTACT.h:181-896) and the per-iteration data contract of
// CONTACT_ANALYSIS (MCONTACT.h:2493-2723).  The ADMM loop itself runs on the GPU
// (device_mcontact.hip); this file only builds operands.
#pragma once
#include <array>
#include <cstdint>
#include <vector>

#include "multigrid.hpp"

namespace ddpca {

// CSEARCH::INTEGRAL_POINT (CSEARCH.h:19-32): the setup-time data contract of one interface.
struct IntegralPoint {
    int64_t node[2][4];
    double shap[2][4];
    double basis[3][3];  // 0 normal (master side), 1/2 tangents
    double gap;          // initNgap
    double w;            // quadWeig
};

struct Interface {
    int64_t body[2] = {0, 0};      // contBody[ts]
    double fric = -1.0;            // fricCoef: <0 glued, 0 frictionless, >0 Coulomb
    double penN = 0.0, penF = 0.0;  // penaFact_n / penaFact_f
    std::vector<IntegralPoint> ip;
    // ---- operators (MCONTACT.h:213-810); side s in {0, 1}
    std::vector<int64_t> nodeCont[2];  // contact index -> body node id (insertion order)
    Csr systMass[2], systTran[2], systTran_pena[2];
    Csr inteMass[2], inteMass_pena[2];
    Csr inpoLagr[2], inpoDisp[2], inteInpo[2], pemaInpo_r[2];
    std::vector<double> inpoNgap;  // m_ip
    std::vector<double> pemaDiag;  // pemaInpo diagonal, m_ip
    int comp() const { return fric == 0.0 ? 1 : 3; }
    int64_t mip() const { return comp() * (int64_t)ip.size(); }
    int64_t mside(int s) const { return comp() * (int64_t)nodeCont[s].size(); }
    // the per-ip operators were assembled here from `ip` (BUILD): every row of inpoLagr /
    // pemaInpo_r / inteInpo is an outer product of one ip's shape values and basis, so the device
    // may apply them in that factored form (operators handed over by a caller are not assumed so)
    bool factored = false;
    void BUILD(const MULTIGRID& g0, const MULTIGRID& g1);
};

// Interface-eliminated coarse space (MCONTACT::MULTISCALE_1, MCONTACT.h:1672-2301).  Built
// rank-locally: rows/columns that belong to owned subdomains and owned interface sides.
struct CoarseSpace {
    bool ready = false;
    std::vector<uint8_t> built;               // per subdomain: its rows were assembled here
    std::vector<int64_t> baseReco;            // nsub + 1 (MCONTACT.h:849-857)
    int64_t n = 0;                            // globCoup_1 dimension
    Csr globCoup_1;                           // n x n, rows of built subdomains
    std::vector<double> globForc_1;           // n, rows of built subdomains
    std::vector<std::array<Csr, 2>> globTran_1;  // [ts][s] n x comp*nnc_s (owned sides)
    std::vector<Csr> globTran_S;              // [tv] n x 3N_tv: interface part of globTran_D_1
                                              // (the stiffness part Rc consStif[L] C_L is applied
                                              // in factored form)
    std::vector<Stencil> accuQ;               // [tv] fine node -> level-d node prolongation chain (3x3
                                              // block entries where a nodal rotation enters)
    // assembled variant (operator-level builder: the caller's own MULTISCALE_1 output): the full
    // globTran_D_1[tv] (n x 3N_tv) and accuProl[tv] (nfree_L x nfree_d) replace the factored
    // stiffness part / globTran_S and accuQ
    bool assembled = false;
    std::vector<Csr> globTran_D_full, accuProl_full;
    // LATIN-type coarse space (MULTISCALE, muscSett bit 0; assembled only): globCoup_1 holds
    // globCoup (displacement blocks + coarse contact unknowns, rows >= baseReco[nsub]), the
    // right-hand side is sum over sides of globTran lambda - globTran_pena aux + globTran_D u
    bool latin = false;
    bool rank_local = false;  // latin rows of the coarse contact unknowns hold this rank's share only
    std::vector<std::array<Csr, 2>> globTran_L, globTran_pena_L, globTran_D_L;  // [ts][s]
    // coarse contact unknowns of interface ts: level-doleMcsc node positions of contBody[ts][0]
    // (MULTISCALE's coarNode, MCONTACT.h:903-957), comp unknowns each -- DOUBLE_M's hierarchy
    // coarsens them (empty: not known, e.g. a caller's operators without them)
    std::vector<std::vector<int64_t>> coarNode;
};

// prolOper[L-1] ... prolOper[d] of one grid as a single scalar stencil (no masks)
Stencil accumulated_stencil(const MULTIGRID& g, int64_t d);

class MCONTACT {
public:
    std::vector<MULTIGRID> multGrid;
    std::vector<Interface> searCont;
    int64_t muscSett = 0;                  // bit 1: interface-eliminated coarse space
    std::vector<int64_t> doleMcsc;         // coarse level per subdomain (MCONTACT.h:23)
    CoarseSpace coarse;
    void MULTISCALE_1(const std::vector<uint8_t>* owned = nullptr);
    void MULTISCALE(const std::vector<uint8_t>* owned = nullptr);  // LATIN-type (muscSett bit 0)
    Csr globTran_D_1(int64_t tv) const;    // assembled (tests)
    Csr accuProl(int64_t tv) const;        // assembled (tests)
    // ESTABLISH: interface operators, systMass added to each body's stiffness, then
    // TRANSFER / STIF_MATR / CONSTRAINT(1) per body (MCONTACT.h:812-825).  owned (optional):
    // per-subdomain mask; only owned bodies and interfaces touching them are built (one rank's
    // share of a multi-GPU run).
    void ESTABLISH(const std::vector<uint8_t>* owned = nullptr);
    double GET_CHAR_LENG() const;  // MCONTACT.h:2478-2491
};

// Conforming-face integration points (restatement of CSEARCH::SEGMENT_INTERSECT for two
// coincident quadrilateral faces: polygon = master face, 4 centroid triangles x 4-point
// triangle rule, CSEARCH.h:614-775).  mast/slav: 4 node ids of matching faces, oriented as
// EFACE_SURFACE returns them.  sub > 1: the master face in sub x sub polygons (the intersection
// with a slave face mesh sub times finer), 16 points each.
void conforming_face_ips(const MULTIGRID& gm, const int64_t mast[4], const MULTIGRID& gs,
                         const int64_t slav[4], std::vector<IntegralPoint>& out, int sub = 1);

}  // namespace ddpca

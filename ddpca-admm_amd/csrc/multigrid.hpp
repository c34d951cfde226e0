// MULTIGRID: host restatement of the reference's operator-producing subset (MULTIGRID.h:10-95):
//   REFINE_ALL           MULTIGRID.h:375-545   pattern 0 on every leaf (the generators' uniform
//                                              rounds, lattice-keyed nodes); node creation order
//                                              reproduced exactly, so the level-ordered numbering
//                                              equals the reference's
//   REFINE + GRLE_CHECK  MULTIGRID.h:375-678   local refinement of any leaf set with patterns 0-6,
//                                              level balancing, planSurf (curved faces), spliFlag;
//                                              coordinate-keyed nodes (TRY_ADD_NODE(COOR))
//   TRANSFER             MULTIGRID.h:756-948   level sets + scalar prolongation stencils; on any
//                                              octree (every refinement pattern, locally refined
//                                              meshes): the hanging level past maxiLeve, coupled
//                                              nodes (coupNode / coupReps), the position numbering
//   PATCH                MULTIGRID.h:722-754   hanging nodes moved to their parents' average
//   STIF_MATR            MULTIGRID.h:950-1039  8-node hex, 3x3x3 Gauss, isotropic
//   GET_VOLUME           MULTIGRID.h:1041-1082
//   CONSTRAINT(1)        MULTIGRID.h:1102-1255 nodal rotations (nodeRota: R^T K R and the rotated
//                                              prolongation blocks), the hanging level's Galerkin
//                                              step, the hierarchy, Dirichlet condensation
//   ADDITIONAL_FORCE     MULTIGRID.h:1257-1261
//   OUTP_SUB1            MULTIGRID.h:1263-1281
// A general tree comes in through the C ABI (ddpca_multigrid_*, capi_multigrid.cpp) with the
// element tree the caller built or refined (ddpca_multigrid_refine); TRANSFER then renumbers the
// nodes to the reference's positions (posiNode keeps the original ids: earlTran).  Out of scope
// here: the curved-surface projection itself (CURVEDS: the caller supplies its
// planSurf), stress recovery, text output.
#pragma once
#include <array>
#include <cstdint>
#include <map>
#include <set>
#include <unordered_map>
#include <vector>

#include "sparse.hpp"

namespace ddpca {

struct TreeElem {
    int64_t parent = -1;
    std::array<int64_t, 8> cornNode{};
    int level = 0;
    int64_t firstChild = -1;  // REFINE_ALL: the 8 children are consecutive (ADD_ELEMENT order)
    int refiPatt = 7;         // PREP.h TREE_ELEM: 0 xi-eta-zeta, 1 xi-eta, 2 eta-zeta, 3 zeta-xi,
                              // 4 xi, 5 eta, 6 zeta (the pattern the element WAS refined with), 7 leaf
    std::vector<int64_t> children;  // general trees (capi_multigrid.cpp); REFINE_ALL fills it too
    bool leaf() const { return firstChild < 0 && children.empty(); }
};

class MULTIGRID {
public:
    // ---------------------------------------------------------------- mesh
    std::vector<std::array<double, 3>> nodeCoor;   // node id == reference node id
    std::vector<std::array<int64_t, 3>> nodeLatt;  // integer lattice position (topology key)
    std::vector<int> nodeLevel;
    std::vector<std::vector<int64_t>> nodeParents;  // parents of a refined node (sorted ids)
    std::vector<TreeElem> elemVect;
    std::unordered_map<uint64_t, int64_t> lattNode;  // lattice key -> node (TRY_ADD_NODE lookup)
    // coordinate -> node (the reference's coorNode, COOR's 1e-10 lexicographic order), general trees
    struct CoorLess {
        bool operator()(const std::array<double, 3>& a, const std::array<double, 3>& b) const {
            for (int i = 0; i < 3; ++i) {
                if (a[i] < b[i] - 1.0e-10) return true;
                if (a[i] > b[i] + 1.0e-10) return false;
            }
            return false;
        }
    };
    std::map<std::array<double, 3>, int64_t, CoorLess> coorNode;
    int64_t maxiLeve = -1;
    int64_t TRY_ADD_NODE(const std::array<int64_t, 3>& latt, const std::array<double, 3>& xyz);
    int64_t ADD_ELEMENT(const TreeElem& e);
    // One uniform refinement round: MULTIGRID::REFINE with refiPatt = 0 on every leaf element.
    void REFINE_ALL();
    // MULTIGRID::REFINE (MULTIGRID.h:375-545) on a general tree: GRLE_CHECK's level balancing
    // (547-678: the leaf neighbours across the refined elements' parent edges / faces join with
    // pattern 0), then every element of `split` (each with its refiPatt set) is cut with its
    // pattern; a new node sits at planSurf's position for its corner set (a curved surface) or at
    // the corners' average, nodes deduplicated by coordinates as TRY_ADD_NODE does (1e-10).
    // `split` returns the children spliFlag selects (element -> child indices) for the next round.
    void REFINE(std::set<int64_t>& split, const std::map<int64_t, std::set<int>>& spliFlag,
                const std::map<std::vector<int64_t>, std::array<double, 3>>& planSurf);
    void GRLE_CHECK(std::set<int64_t>& split);
    int64_t TRY_ADD_COOR(const std::array<double, 3>& xyz);  // coordinate-keyed TRY_ADD_NODE
    int64_t numNodes() const { return (int64_t)nodeCoor.size(); }

    // ---------------------------------------------------------------- transfer
    std::vector<int64_t> leveCount;   // nodes of levels <= l  (levels 0..maxiLeve)
    std::vector<Stencil> scalProl;    // level l+1 nodes x level l nodes
    void TRANSFER();
    // general trees (MULTIGRID.h:49-58, 84): coupled nodes represented by coupReps, nodal rotations
    std::set<int64_t> coupNode;
    int64_t coupReps = -1;
    std::map<int64_t, std::array<double, 9>> nodeRota;  // node -> 3x3 row-major
    // after TRANSFER on a general tree: node ids ARE positions (MULTIGRID.h:884-910); posiNode[p] =
    // the node's original id (earlTran), hangStencil = prolOper[maxiLeve]'s stencil (all nodes x
    // level-maxiLeve nodes, identity on the latter), empty without a hanging level
    bool general = false;
    std::vector<int64_t> posiNode;
    Stencil hangStencil;
    // the reference's algorithm on any tree (forced on uniform trees too with force_general, tests)
    void TRANSFER_GENERAL();
    bool force_general = false;
    // Hanging level (operator-level builder only): the reference puts hanging nodes of local
    // refinement and coupled nodes on a level maxiLeve + 1 outside the MGPIS hierarchy
    // (MULTIGRID.h:836-848, 870-875, 884-910); their values are rows of prolOper[maxiLeve] applied
    // to the level-maxiLeve nodal vector (OUTP_SUB1, MULTIGRID.h:1279).  nodeAll = 0: none.
    int64_t nodeAll = 0;
    Csr hangProl;  // 3 (nodeAll - leveCount.back()) x 3 leveCount.back(), position numbering
    // nodes of the subdomain's nodal vectors (resuDisp, interface operator columns)
    int64_t nodalCount() const { return nodeAll ? nodeAll : leveCount.back(); }

    // ---------------------------------------------------------------- stiffness
    double mateElas = 210.0e9;
    double matePois = 0.3;
    Bsr3 origStif;  // full nodal stiffness (reference origStif[maxiLeve + 1])
    void STIF_MATR();
    double GET_VOLUME() const;
    // origStif += A (A given as scalar CSR on the 3N nodal dofs, pattern inside node adjacency)
    void ADD_NODAL(const Csr& A);

    // ---------------------------------------------------------------- constraints
    std::map<int64_t, double> consDofv;  // prescribed dof values
    std::map<int64_t, double> exteForc;  // external nodal forces
    void LOAD_ACCU(int64_t dof, double v);
    std::vector<Bsr3> levelStif;          // unconstrained Galerkin operators origStif[l]
    // prolOper[l] (MULTIGRID.h:1141-1181): scalProl[l] with the nodal rotations' 3x3 blocks as
    // block entries (== scalProl without nodeRota), and the hanging level's prolOper[maxiLeve]
    std::vector<Stencil> prolOper;
    Stencil prolHang;
    std::vector<uint8_t> consFlag;        // 3N: 1 free, 0 constrained
    std::vector<int32_t> freeIndex;       // 3N: condensed index or -1
    std::vector<int64_t> freeCount;       // free dofs on level l
    std::vector<double> consForc;         // condensed load (MULTIGRID::consForc)
    std::vector<double> dispForc;         // prescribed values of constrained dofs, dof order
    void FLAGS();       // the dof bookkeeping of CONSTRAINT only (consFlag/freeIndex/freeCount)
    void PROL_OPER();   // prolOper / prolHang from the stencils and nodeRota (CONSTRAINT's first step;
                        // the coarse spaces read it on subdomains this rank does not build)
    void CONSTRAINT();  // FLAGS + Galerkin hierarchy + condensed load

    // ---------------------------------------------------------------- per-iteration adapters
    // f_free = consOper * prolOper^T * earlTran^T * f_nodal (identities except consOper here)
    void ADDITIONAL_FORCE(const double* f_nodal, double* f_free) const;
    // u_nodal = earlTran * prolOper * [x_free scattered; prescribed values]
    void OUTP_SUB1(const double* x_free, double* u_nodal) const;

    // reference-layout operators (MGPIS::consStif / realProl, condensed scalar CSR)
    Csr consStif(int64_t level) const;
    Csr realProl(int64_t level) const;  // level+1 <- level
    // rows of prolOper[maxiLeve] past the MGPIS fine level (positions x level-maxiLeve positions),
    // the hanging level's values (OUTP_SUB1, MULTIGRID.h:1279)
    Csr hangRows() const;
};

// Coarse-mesh builders used by the examples (node creation order as in the reference).
// BEAM (BEAM.h:61-186, 251-388): subdomain tg of a domaNumb decomposition of the tapered,
// twisted cantilever (domaNumb = {1,1,1}, tg = 0 is MESH_NODD), incl. COOR_ADJU and
// SUBR_COLO with loadType 0 (clamped root, centreline line load).
void build_beam(MULTIGRID& g, const int64_t divi[3], int64_t globLeve, const int64_t doma[3],
                int64_t tg);
// Axis-aligned box with BLOCK.h's corner convention, refined globLeve times.
// latt_off: this block's origin on a lattice shared with its neighbours (coarse units).
void build_box(MULTIGRID& g, const double lo[3], const double hi[3], const int64_t n[3],
               int64_t globLeve, const int64_t latt_off[3] = nullptr);

}  // namespace ddpca

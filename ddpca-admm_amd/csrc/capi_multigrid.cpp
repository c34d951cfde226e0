// C ABI: the MULTIGRID operator pipeline on a caller's element tree (MULTIGRID::TRANSFER + PATCH +
// STIF_MATR + CONSTRAINT(1), MULTIGRID.h:722-1255), for meshes the host generators do not make --
// locally refined octrees with any refinement pattern (hanging nodes on the level past maxiLeve),
// coupled nodes, nodal rotations (nodeRota).  The tree is what the reference's REFINE leaves in
// MULTIGRID::elemVect / nodeCoor; its outputs are the reference's operators in its own layouts
// (position numbering, condensed CSR), and ddpca_problem_set_subdomain_multigrid hands them to the
// operator-level problem builder exactly as the reference binding does with the reference's own
// MULTIGRID (oracle/ref_bind.hpp from_reference).
#include <algorithm>
#include <cstring>
#include <memory>
#include <map>
#include <set>
#include <string>

#include "../../include/ddpca_amd.h"
#include "common.hpp"
#include "problem.hpp"

using namespace ddpca;

struct ddpca_multigrid {
    MULTIGRID g;
    int64_t nnode = 0;                 // node ids of the input (before TRANSFER's renumbering)
    bool built = false;
    std::vector<double> coords_by_id;  // after PATCH, by original node id
    std::vector<int64_t> i64;
    std::vector<uint8_t> u8;
    std::vector<double> f64;
    Csr csr;
    std::vector<int64_t> shape;
    std::vector<int64_t> next_split;   // the children spliFlag selected in the last refine
};

namespace {

template <typename T>
int dtype_code();
template <>
int dtype_code<double>() { return 0; }
template <>
int dtype_code<int64_t>() { return 1; }
template <>
int dtype_code<int32_t>() { return 2; }
template <>
int dtype_code<uint8_t>() { return 3; }

template <typename T>
void put(const std::vector<T>& v, const void** data, int64_t* count, int* dtype) {
    *data = v.data();
    *count = (int64_t)v.size();
    *dtype = dtype_code<T>();
}

ddpca_multigrid& open(ddpca_multigrid_t h, bool want_built) {
    if (!h) throw ApiError(DDPCA_EINVAL, "null handle");
    if (h->built != want_built)
        throw ApiError(DDPCA_ESTATE, want_built ? "ddpca_multigrid_build has not run" : "the operators are already built");
    return *h;
}

}  // namespace

// CURVEDS (CURVEDS.h:8-121): a curved surface as a grid of points indiPoin[i][j] with the reverse
// map point -> (i, j) under the mesh's coordinate comparison.  REFINE_SEARCH: a corner set lies on
// the surface when every corner is a grid point; its new node is the point at the corners'
// averaged (integer) indices.
struct ddpca_curveds {
    int64_t ni = 0, nj = 0;
    std::vector<std::array<double, 3>> pt;  // ni x nj
    std::vector<uint8_t> present;
    std::map<std::array<double, 3>, std::array<int64_t, 2>, MULTIGRID::CoorLess> index;
    // the last plan (ddpca_curveds_plan)
    std::vector<int64_t> plan_ptr, plan_node;
    std::vector<double> plan_xyz;
    void reindex() {  // CURVEDS::INSERT's poinIndi.emplace: the first point of equal coordinates wins
        index.clear();
        for (int64_t i = 0; i < ni; ++i)
            for (int64_t j = 0; j < nj; ++j)
                if (present[i * nj + j]) index.emplace(pt[i * nj + j], std::array<int64_t, 2>{i, j});
    }
    bool search(const std::vector<std::array<double, 3>>& c, std::array<double, 3>& out) const {
        int64_t si = 0, sj = 0;
        for (const auto& p : c) {
            const auto it = index.find(p);
            if (it == index.end()) return false;
            si += it->second[0];
            sj += it->second[1];
        }
        si /= (int64_t)c.size();
        sj /= (int64_t)c.size();
        out = pt[si * nj + sj];
        return true;
    }
};

extern "C" {

int ddpca_curveds_create(int64_t ni, int64_t nj, const double* xyz, const uint8_t* present, ddpca_curveds_t* out) {
    return guarded([&] {
        if (ni < 1 || nj < 1 || !xyz || !out) throw ApiError(DDPCA_EINVAL, "null argument or empty surface grid");
        auto c = std::make_unique<ddpca_curveds>();
        c->ni = ni;
        c->nj = nj;
        c->pt.resize(ni * nj);
        c->present.assign(ni * nj, 1);
        for (int64_t k = 0; k < ni * nj; ++k) {
            for (int a = 0; a < 3; ++a) c->pt[k][a] = xyz[3 * k + a];
            if (present) c->present[k] = present[k] ? 1 : 0;
        }
        c->reindex();
        *out = c.release();
    });
}

int ddpca_curveds_rigid(ddpca_curveds_t c, const double* R, const double* t) {
    return guarded([&] {
        if (!c || !R || !t) throw ApiError(DDPCA_EINVAL, "null argument");
        for (int64_t k = 0; k < c->ni * c->nj; ++k) {
            if (!c->present[k]) continue;
            const std::array<double, 3> p = c->pt[k];
            for (int a = 0; a < 3; ++a) c->pt[k][a] = (R[3 * a] * p[0] + R[3 * a + 1] * p[1] + R[3 * a + 2] * p[2]) + t[a];
        }
        c->reindex();
    });
}

int ddpca_curveds_plan(ddpca_curveds_t c, ddpca_multigrid_t h, int64_t n, const int64_t* elem, const int64_t** plan_ptr,
                       const int64_t** plan_node, const double** plan_xyz, int64_t* nplan) {
    return guarded([&] {
        if (!c || !h || (n > 0 && !elem) || !plan_ptr || !plan_node || !plan_xyz || !nplan)
            throw ApiError(DDPCA_EINVAL, "null argument");
        if (h->built) throw ApiError(DDPCA_ESTATE, "the operators are already built");
        const MULTIGRID& g = h->g;
        // CURVEDS::REFINE (CURVEDS.h:58-101): every line and face of every split element
        static const int line[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6}, {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
        static const int face[6][4] = {{0, 3, 7, 4}, {1, 2, 6, 5}, {0, 4, 5, 1}, {3, 7, 6, 2}, {0, 1, 2, 3}, {4, 5, 6, 7}};
        std::map<std::vector<int64_t>, std::array<double, 3>> plan;
        auto try_key = [&](std::vector<int64_t> key) {
            std::vector<std::array<double, 3>> xyz;
            for (int64_t v : key) xyz.push_back(g.nodeCoor[v]);
            std::array<double, 3> p;
            if (!c->search(xyz, p)) return;
            std::sort(key.begin(), key.end());
            plan.emplace(key, p);  // planSurf.insert: an existing key keeps its point
        };
        for (int64_t k = 0; k < n; ++k) {
            if (elem[k] < 0 || elem[k] >= (int64_t)g.elemVect.size()) throw ApiError(DDPCA_EINVAL, "element out of range");
            const auto& cn = g.elemVect[elem[k]].cornNode;
            for (const auto& l : line) try_key({cn[l[0]], cn[l[1]]});
            for (const auto& f : face) try_key({cn[f[0]], cn[f[1]], cn[f[2]], cn[f[3]]});
        }
        c->plan_ptr.assign(1, 0);
        c->plan_node.clear();
        c->plan_xyz.clear();
        for (const auto& kv : plan) {
            c->plan_node.insert(c->plan_node.end(), kv.first.begin(), kv.first.end());
            c->plan_ptr.push_back((int64_t)c->plan_node.size());
            c->plan_xyz.insert(c->plan_xyz.end(), kv.second.begin(), kv.second.end());
        }
        *plan_ptr = c->plan_ptr.data();
        *plan_node = c->plan_node.data();
        *plan_xyz = c->plan_xyz.data();
        *nplan = (int64_t)plan.size();
    });
}

int ddpca_curveds_destroy(ddpca_curveds_t c) {
    delete c;
    return DDPCA_OK;
}


int ddpca_multigrid_create(int64_t nnode, const double* coords, int64_t nelem, const int64_t* corner,
                           const int64_t* parent, const int64_t* level, const int64_t* refiPatt,
                           const int64_t* child_ptr, const int64_t* child, ddpca_multigrid_t* out) {
    return guarded([&] {
        if (nnode < 8 || nelem < 1 || !coords || !corner || !parent || !level || !refiPatt || !child_ptr || !out)
            throw ApiError(DDPCA_EINVAL, "null argument or empty tree");
        if (nnode >= (int64_t)1 << 31) throw ApiError(DDPCA_EINVAL, "node ids must fit int32");
        auto h = std::make_unique<ddpca_multigrid>();
        MULTIGRID& g = h->g;
        h->nnode = nnode;
        g.nodeCoor.resize(nnode);
        for (int64_t i = 0; i < nnode; ++i)
            for (int a = 0; a < 3; ++a) g.nodeCoor[i][a] = coords[3 * i + a];
        g.nodeLevel.assign(nnode, 0);
        g.nodeParents.assign(nnode, {});
        g.maxiLeve = 0;
        g.elemVect.resize(nelem);
        if (child_ptr[0] != 0) throw ApiError(DDPCA_EINVAL, "child_ptr[0] must be 0");
        for (int64_t e = 0; e < nelem; ++e) {
            TreeElem& t = g.elemVect[e];
            for (int k = 0; k < 8; ++k) {
                t.cornNode[k] = corner[8 * e + k];
                if (t.cornNode[k] < 0 || t.cornNode[k] >= nnode) throw ApiError(DDPCA_EINVAL, "corner node out of range");
            }
            t.parent = parent[e];
            t.level = (int)level[e];
            t.refiPatt = (int)refiPatt[e];
            if (t.parent < -1 || t.parent >= nelem || t.level < 0) throw ApiError(DDPCA_EINVAL, "parent / level out of range");
            const int64_t c0 = child_ptr[e], c1 = child_ptr[e + 1];
            if (c1 < c0 || (c1 > c0 && !child)) throw ApiError(DDPCA_EINVAL, "child_ptr not monotone");
            for (int64_t c = c0; c < c1; ++c) {
                if (child[c] <= e || child[c] >= nelem) throw ApiError(DDPCA_EINVAL, "child index out of range");
                t.children.push_back(child[c]);
            }
            if (!t.children.empty() && (t.refiPatt < 0 || t.refiPatt > 6))
                throw ApiError(DDPCA_EINVAL, "refined element needs a refinement pattern 0..6");
            g.maxiLeve = std::max<int64_t>(g.maxiLeve, t.level);  // ADD_ELEMENT, MULTIGRID.h:371
        }
        *out = h.release();
    });
}

int ddpca_multigrid_set(ddpca_multigrid_t h, const char* what, int64_t n, const int64_t* idx, const double* val) {
    return guarded([&] {
        ddpca_multigrid& M = open(h, false);
        MULTIGRID& g = M.g;
        if (!what || n < 0) throw ApiError(DDPCA_EINVAL, "null argument");
        const std::string w(what);
        auto need = [&](bool i, bool v) {
            if (n > 0 && ((i && !idx) || (v && !val))) throw ApiError(DDPCA_EINVAL, w + ": null array");
        };
        auto node = [&](int64_t v) {
            if (v < 0 || v >= M.nnode) throw ApiError(DDPCA_EINVAL, w + ": node out of range");
            return v;
        };
        auto dof = [&](int64_t d) {  // not node(d / 3): division truncates -1 and -2 to node 0
            if (d < 0 || d >= 3 * M.nnode) throw ApiError(DDPCA_EINVAL, w + ": dof out of range");
            return d;
        };
        if (w == "consDofv") {  // MULTIGRID::consDofv.emplace (first value of a dof wins)
            need(true, true);
            for (int64_t k = 0; k < n; ++k) {
                g.consDofv.emplace(dof(idx[k]), val[k]);
            }
        } else if (w == "exteForc") {  // LOAD_ACCU in the given order (MULTIGRID.h:1084-1100)
            need(true, true);
            for (int64_t k = 0; k < n; ++k) {
                g.LOAD_ACCU(dof(idx[k]), val[k]);
            }
        } else if (w == "nodeRota") {
            need(true, true);
            for (int64_t k = 0; k < n; ++k) {
                std::array<double, 9> R;
                for (int q = 0; q < 9; ++q) R[q] = val[9 * k + q];
                g.nodeRota.emplace(node(idx[k]), R);
            }
        } else if (w == "coupNode") {
            need(true, false);
            for (int64_t k = 0; k < n; ++k) g.coupNode.insert(node(idx[k]));
        } else if (w == "coupReps") {
            need(true, false);
            if (n != 1) throw ApiError(DDPCA_EINVAL, "coupReps: one node (or -1)");
            g.coupReps = idx[0] < 0 ? -1 : node(idx[0]);
        } else if (w == "material") {
            need(false, true);
            if (n != 2 || !(val[0] > 0.0) || !(val[1] > -1.0 && val[1] < 0.5)) throw ApiError(DDPCA_EINVAL, "material: E > 0, -1 < nu < 0.5");
            g.mateElas = val[0];
            g.matePois = val[1];
        } else {
            throw ApiError(DDPCA_EINVAL, "unknown input " + w);
        }
    });
}

int ddpca_multigrid_refine(ddpca_multigrid_t h, int64_t n, const int64_t* elem, const int64_t* patt, int64_t nplan,
                           const int64_t* plan_ptr, const int64_t* plan_node, const double* plan_xyz, int64_t nflag,
                           const int64_t* flag_elem, const int64_t* flag_child) {
    return guarded([&] {
        ddpca_multigrid& M = open(h, false);
        MULTIGRID& g = M.g;
        if (n < 0 || (n > 0 && (!elem || !patt)) || nplan < 0 || (nplan > 0 && (!plan_ptr || !plan_node || !plan_xyz)) ||
            nflag < 0 || (nflag > 0 && (!flag_elem || !flag_child)))
            throw ApiError(DDPCA_EINVAL, "null argument");
        // every argument is checked before the tree changes; REFINE's own checks (GRLE_CHECK's
        // level balance, spliFlag children against the pattern) run on a copy that replaces the
        // tree only when the whole refinement succeeded
        const int64_t ne = (int64_t)g.elemVect.size();
        std::set<int64_t> split;
        for (int64_t k = 0; k < n; ++k) {
            if (elem[k] < 0 || elem[k] >= ne || !g.elemVect[elem[k]].leaf()) throw ApiError(DDPCA_EINVAL, "refine: not a leaf element");
            if (patt[k] < 0 || patt[k] > 6) throw ApiError(DDPCA_EINVAL, "refine: pattern must be 0..6");
            split.insert(elem[k]);
        }
        std::map<std::vector<int64_t>, std::array<double, 3>> plan;
        if (nplan > 0 && plan_ptr[0] != 0) throw ApiError(DDPCA_EINVAL, "plan_ptr[0] must be 0");
        for (int64_t q = 0; q < nplan; ++q)
            if (plan_ptr[q + 1] < plan_ptr[q]) throw ApiError(DDPCA_EINVAL, "refine: plan_ptr must be non-decreasing");
        for (int64_t k = 0; k < (nplan > 0 ? plan_ptr[nplan] : 0); ++k)
            if (plan_node[k] < 0 || plan_node[k] >= M.nnode) throw ApiError(DDPCA_EINVAL, "refine: planSurf node out of range");
        for (int64_t q = 0; q < nplan; ++q) {
            std::vector<int64_t> key(plan_node + plan_ptr[q], plan_node + plan_ptr[q + 1]);
            if (key.size() < 2) throw ApiError(DDPCA_EINVAL, "refine: planSurf key of fewer than 2 nodes");
            std::sort(key.begin(), key.end());
            plan.emplace(key, std::array<double, 3>{plan_xyz[3 * q], plan_xyz[3 * q + 1], plan_xyz[3 * q + 2]});
        }
        std::map<int64_t, std::set<int>> flag;
        for (int64_t k = 0; k < nflag; ++k) {
            if (flag_elem[k] < 0 || flag_elem[k] >= ne) throw ApiError(DDPCA_EINVAL, "refine: spliFlag element out of range");
            if (flag_child[k] < 0 || flag_child[k] > 7) throw ApiError(DDPCA_EINVAL, "refine: spliFlag child must be 0..7");
            flag[flag_elem[k]].insert((int)flag_child[k]);
        }
        MULTIGRID t = g;
        for (int64_t k = 0; k < n; ++k) t.elemVect[elem[k]].refiPatt = (int)patt[k];
        try {
            t.REFINE(split, flag, plan);
        } catch (const std::invalid_argument& e) {
            throw ApiError(DDPCA_EINVAL, e.what());
        }
        g = std::move(t);
        M.next_split.assign(split.begin(), split.end());
        M.nnode = g.numNodes();
        g.nodeLevel.assign(M.nnode, 0);
        g.nodeParents.assign(M.nnode, {});
    });
}

int ddpca_multigrid_tree(ddpca_multigrid_t h, const char* what, const void** data, int64_t* count, int* dtype) {
    return guarded([&] {
        ddpca_multigrid& M = open(h, false);
        const MULTIGRID& g = M.g;
        if (!what || !data || !count || !dtype) throw ApiError(DDPCA_EINVAL, "null argument");
        const std::string w(what);
        M.i64.clear();
        if (w == "nodeCoor") {
            M.f64.resize(3 * M.nnode);
            for (int64_t i = 0; i < M.nnode; ++i)
                for (int a = 0; a < 3; ++a) M.f64[3 * i + a] = g.nodeCoor[i][a];
            put(M.f64, data, count, dtype);
            return;
        }
        if (w == "corner") {
            for (const auto& e : g.elemVect) M.i64.insert(M.i64.end(), e.cornNode.begin(), e.cornNode.end());
        } else if (w == "parent") {
            for (const auto& e : g.elemVect) M.i64.push_back(e.parent);
        } else if (w == "level") {
            for (const auto& e : g.elemVect) M.i64.push_back(e.level);
        } else if (w == "refiPatt") {
            for (const auto& e : g.elemVect) M.i64.push_back(e.refiPatt);
        } else if (w == "child_ptr") {
            M.i64.push_back(0);
            for (const auto& e : g.elemVect) M.i64.push_back(M.i64.back() + (int64_t)e.children.size());
        } else if (w == "child") {
            for (const auto& e : g.elemVect) M.i64.insert(M.i64.end(), e.children.begin(), e.children.end());
        } else if (w == "nextSplit") {
            M.i64 = M.next_split;
        } else {
            throw ApiError(DDPCA_EINVAL, "unknown tree quantity " + w);
        }
        put(M.i64, data, count, dtype);
    });
}

int ddpca_multigrid_build(ddpca_multigrid_t h, const ddpca_csr_t* extra) {
    return guarded([&] {
        ddpca_multigrid& M = open(h, false);
        MULTIGRID& g = M.g;
        if (!g.coupNode.empty() && g.coupReps < 0) throw ApiError(DDPCA_EINVAL, "coupled nodes need coupReps");
        try {
            g.force_general = true;
            g.TRANSFER();  // TRANSFER + PATCH; node ids become positions (g.posiNode = earlTran)
            g.STIF_MATR();
            if (extra) {
                // origStif[maxiLeve + 1] += extra in the node-id numbering (MCONTACT.h:816-822:
                // the contact interfaces' systMass), moved to positions
                if (extra->nrow != 3 * M.nnode || extra->ncol != 3 * M.nnode || (extra->nrow && !extra->ptr))
                    throw ApiError(DDPCA_EINVAL, "extra stiffness: 3N x 3N in node ids");
                std::vector<int64_t> pos(M.nnode);
                for (int64_t p = 0; p < M.nnode; ++p) pos[g.posiNode[p]] = p;
                Csr A;
                A.nrow = A.ncol = 3 * M.nnode;
                std::vector<std::vector<std::pair<int32_t, double>>> rows(A.nrow);
                for (int64_t r = 0; r < extra->nrow; ++r)
                    for (int64_t k = extra->ptr[r]; k < extra->ptr[r + 1]; ++k) {
                        const int32_t c = extra->col[k];
                        if (c < 0 || c >= A.ncol) throw ApiError(DDPCA_EINVAL, "extra stiffness: column out of range");
                        rows[3 * pos[r / 3] + r % 3].push_back({(int32_t)(3 * pos[c / 3] + c % 3), extra->val[k]});
                    }
                A.ptr.assign(A.nrow + 1, 0);
                for (int64_t r = 0; r < A.nrow; ++r) {
                    for (const auto& e : rows[r]) {
                        A.col.push_back(e.first);
                        A.val.push_back(e.second);
                    }
                    A.ptr[r + 1] = (int64_t)A.col.size();
                }
                g.ADD_NODAL(A);
            }
            g.CONSTRAINT();
        } catch (const ApiError&) {
            throw;
        } catch (const std::invalid_argument& e) {
            throw ApiError(DDPCA_EINVAL, e.what());
        } catch (const std::runtime_error& e) {
            throw ApiError(DDPCA_EINVAL, e.what());
        }
        M.coords_by_id.assign(3 * M.nnode, 0.0);
        for (int64_t p = 0; p < M.nnode; ++p)
            for (int a = 0; a < 3; ++a) M.coords_by_id[3 * g.posiNode[p] + a] = g.nodeCoor[p][a];
        M.built = true;
    });
}

int ddpca_multigrid_view(ddpca_multigrid_t h, const char* what, int64_t level, const void** data, int64_t* count,
                         int* dtype) {
    return guarded([&] {
        ddpca_multigrid& M = open(h, true);
        const MULTIGRID& g = M.g;
        if (!what || !data || !count || !dtype) throw ApiError(DDPCA_EINVAL, "null argument");
        const std::string w(what);
        const int64_t L = g.maxiLeve;
        auto lev = [&](int64_t lo, int64_t hi) {
            if (level < lo || level > hi) throw ApiError(DDPCA_EINVAL, w + ": level out of range");
        };
        auto csr_part = [&](const std::string& part) {
            if (part == "ptr") put(M.csr.ptr, data, count, dtype);
            else if (part == "col") put(M.csr.col, data, count, dtype);
            else if (part == "val") put(M.csr.val, data, count, dtype);
            else if (part == "shape") {
                M.shape = {M.csr.nrow, M.csr.ncol};
                put(M.shape, data, count, dtype);
            } else throw ApiError(DDPCA_EINVAL, "CSR part must be ptr, col, val or shape");
        };
        if (w == "posiNode") put(g.posiNode, data, count, dtype);
        else if (w == "nodeCoor") put(M.coords_by_id, data, count, dtype);
        else if (w == "leveCount") {
            M.i64.assign(g.leveCount.begin(), g.leveCount.end());
            M.i64.push_back(g.numNodes());  // the hanging level's end: every position
            put(M.i64, data, count, dtype);
        } else if (w == "freeCount") put(g.freeCount, data, count, dtype);
        else if (w == "consFlag") put(g.consFlag, data, count, dtype);
        else if (w == "consForc") put(g.consForc, data, count, dtype);
        else if (w == "dispForc") put(g.dispForc, data, count, dtype);
        else if (w.rfind("K:", 0) == 0) {  // MGPIS::consStif[level]
            lev(0, L);
            M.csr = g.consStif(level);
            csr_part(w.substr(2));
        } else if (w.rfind("P:", 0) == 0) {  // MGPIS::realProl[level] (level + 1 <- level)
            lev(0, L - 1);
            M.csr = g.realProl(level);
            csr_part(w.substr(2));
        } else if (w.rfind("H:", 0) == 0) {  // prolOper[maxiLeve]'s rows past the fine level
            M.csr = g.hangRows();
            csr_part(w.substr(2));
        } else {
            throw ApiError(DDPCA_EINVAL, "unknown quantity " + w);
        }
    });
}

int ddpca_problem_set_subdomain_multigrid(ddpca_problem_t p, int64_t tv, ddpca_multigrid_t h) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (P.established) throw ApiError(DDPCA_ESTATE, "problem already established");
        if (tv < 0 || tv >= (int64_t)P.mc.multGrid.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
        ddpca_multigrid& M = open(h, true);
        const MULTIGRID& s = M.g;
        // what set_subdomain(_prol) + set_hanging build from the reference's MULTIGRID: the fine
        // level's nodes, the level operators (unconstrained: the device masks constrained dofs),
        // prolOper's stencils with their rotation blocks, the hanging rows
        MULTIGRID g;
        const int64_t L = s.maxiLeve, NL = s.leveCount[L];
        g.maxiLeve = L;
        g.leveCount = s.leveCount;
        g.freeCount = s.freeCount;
        g.levelStif = s.levelStif;
        g.scalProl = s.prolOper;
        g.consFlag.assign(s.consFlag.begin(), s.consFlag.begin() + 3 * NL);
        g.freeIndex.assign(s.freeIndex.begin(), s.freeIndex.begin() + 3 * NL);
        g.consForc = s.consForc;
        for (int64_t d = 0; d < 3 * NL; ++d)
            if (!g.consFlag[d]) {
                const auto it = s.consDofv.find(d);
                const double v = it == s.consDofv.end() ? 0.0 : it->second;
                g.consDofv[d] = v;
                g.dispForc.push_back(v);
            }
        g.nodeCoor.assign(s.nodeCoor.begin(), s.nodeCoor.begin() + NL);
        g.nodeLevel.assign(s.nodeLevel.begin(), s.nodeLevel.begin() + NL);
        g.nodeAll = s.nodeAll;
        g.hangProl = s.hangRows();
        P.mc.multGrid[tv] = std::move(g);
        P.owned[tv] = 1;
    });
}

int ddpca_problem_set_subdomain_tree(ddpca_problem_t p, int64_t tv, ddpca_multigrid_t h) {
    return guarded([&] {
        if (!p) throw ApiError(DDPCA_EINVAL, "null problem");
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (P.established) throw ApiError(DDPCA_ESTATE, "problem already established");
        if (tv < 0 || tv >= (int64_t)P.mc.multGrid.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
        ddpca_multigrid& M = open(h, false);
        if (!M.g.coupNode.empty() && M.g.coupReps < 0) throw ApiError(DDPCA_EINVAL, "coupled nodes need coupReps");
        MULTIGRID g = M.g;
        g.force_general = true;  // TRANSFER's general algorithm: node ids become positions
        P.mc.multGrid[tv] = std::move(g);
        P.owned[tv] = 0;         // established by ddpca_problem_establish(_owned)
    });
}

int ddpca_problem_set_contact(ddpca_problem_t p, int64_t ts, int64_t body0, int64_t body1) {
    return guarded([&] {
        if (!p) throw ApiError(DDPCA_EINVAL, "null problem");
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (P.established) throw ApiError(DDPCA_ESTATE, "problem already established");
        const int64_t nsub = (int64_t)P.mc.multGrid.size();
        if (ts < 0 || ts >= (int64_t)P.mc.searCont.size()) throw ApiError(DDPCA_EINVAL, "interface index");
        if (body0 < 0 || body0 >= nsub || body1 < 0 || body1 >= nsub || body0 == body1)
            throw ApiError(DDPCA_EINVAL, "interface bodies");
        P.mc.searCont[ts].body[0] = body0;
        P.mc.searCont[ts].body[1] = body1;
    });
}

int ddpca_multigrid_destroy(ddpca_multigrid_t h) {
    delete h;
    return DDPCA_OK;
}

}  // extern "C"

// Host restatement of the reference's MULTIGRID operator pipeline (see multigrid.hpp).
#include "multigrid.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <omp.h>

namespace ddpca {

namespace {

uint64_t latt_key(const std::array<int64_t, 3>& p) {
    for (int a = 0; a < 3; ++a)
        if (p[a] < 0 || p[a] >= (int64_t(1) << 21)) throw std::runtime_error("lattice coordinate out of range");
    return (uint64_t(p[0]) << 42) | (uint64_t(p[1]) << 21) | uint64_t(p[2]);
}

// Corner positions of a hex on the 3x3x3 subdivision grid (reference refiTemp_2, corners).
const int kCornerPos[8][3] = {{0, 0, 0}, {2, 0, 0}, {2, 2, 0}, {0, 2, 0},
                              {0, 0, 2}, {2, 0, 2}, {2, 2, 2}, {0, 2, 2}};
// Creation order of the 19 new nodes of a pattern-0 refinement (12 edge midpoints, 6 face
// centres, 1 body centre) as positions on the subdivision grid (MULTIGRID.h:382-443).
const int kNewPos[19][3] = {{1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {0, 0, 1}, {2, 0, 1}, {2, 2, 1},
                            {0, 2, 1}, {1, 0, 2}, {2, 1, 2}, {1, 2, 2}, {0, 1, 2}, {0, 1, 1}, {2, 1, 1},
                            {1, 0, 1}, {1, 2, 1}, {1, 1, 0}, {1, 1, 2}, {1, 1, 1}};
// Local corner offsets of a child element on the subdivision grid (MULTIGRID.h:445-453).
const int kHexOff[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0},
                           {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};

// 3-point Gauss rule (PREP.h:235-281): index g = i*9 + j*3 + k over (xi, eta, zeta).
struct HexQuad {
    double w[27];
    double dN[27][3][8];
    HexQuad() {
        const double pt[3] = {-std::sqrt(3.0 / 5.0), 0.0, std::sqrt(3.0 / 5.0)};
        const double wt[3] = {5.0 / 9.0, 8.0 / 9.0, 5.0 / 9.0};
        const double nc[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                                 {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                for (int k = 0; k < 3; ++k) {
                    const int g = i * 9 + j * 3 + k;
                    const double x = pt[i], y = pt[j], z = pt[k];
                    w[g] = wt[i] * wt[j] * wt[k];
                    for (int n = 0; n < 8; ++n) {
                        dN[g][0][n] = nc[n][0] * (1.0 + nc[n][1] * y) * (1.0 + nc[n][2] * z) / 8.0;
                        dN[g][1][n] = (1.0 + nc[n][0] * x) * nc[n][1] * (1.0 + nc[n][2] * z) / 8.0;
                        dN[g][2][n] = (1.0 + nc[n][0] * x) * (1.0 + nc[n][1] * y) * nc[n][2] / 8.0;
                    }
                }
    }
};
const HexQuad& hexquad() {
    static HexQuad q;
    return q;
}

double jacobian(const double dN[3][8], const double X[8][3], double J[3][3]) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int n = 0; n < 8; ++n) s += dN[r][n] * X[n][c];
            J[r][c] = s;
        }
    return J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
           J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
}

// 24x24 element stiffness, K_E = sum_g w_g det(J) B^T D B  (MULTIGRID.h:988-1014)
void element_stiffness(const double X[8][3], const double D[6][6], double KE[24][24]) {
    const HexQuad& q = hexquad();
    for (int a = 0; a < 24; ++a)
        for (int b = 0; b < 24; ++b) KE[a][b] = 0.0;
    for (int g = 0; g < 27; ++g) {
        double J[3][3];
        const double det = jacobian(q.dN[g], X, J);
        double Ji[3][3];
        Ji[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / det;
        Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
        Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
        Ji[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / det;
        Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
        Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
        Ji[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / det;
        Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
        Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
        double B[6][24] = {};
        for (int n = 0; n < 8; ++n) {
            double d[3];
            for (int c = 0; c < 3; ++c) d[c] = Ji[c][0] * q.dN[g][0][n] + Ji[c][1] * q.dN[g][1][n] + Ji[c][2] * q.dN[g][2][n];
            B[0][3 * n + 0] = d[0];
            B[1][3 * n + 1] = d[1];
            B[2][3 * n + 2] = d[2];
            B[3][3 * n + 0] = d[1];
            B[3][3 * n + 1] = d[0];
            B[4][3 * n + 1] = d[2];
            B[4][3 * n + 2] = d[1];
            B[5][3 * n + 0] = d[2];
            B[5][3 * n + 2] = d[0];
        }
        double DB[6][24];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 24; ++c) {
                double s = 0;
                for (int k = 0; k < 6; ++k) s += D[r][k] * B[k][c];
                DB[r][c] = s;
            }
        const double f = q.w[g] * det;
        for (int a = 0; a < 24; ++a)
            for (int b = 0; b < 24; ++b) {
                double s = 0;
                for (int k = 0; k < 6; ++k) s += B[k][a] * DB[k][b];
                KE[a][b] += f * s;
            }
    }
}

}  // namespace

// ---------------------------------------------------------------------------------- mesh
int64_t MULTIGRID::TRY_ADD_NODE(const std::array<int64_t, 3>& latt, const std::array<double, 3>& xyz) {
    const uint64_t key = latt_key(latt);
    auto it = lattNode.find(key);
    if (it != lattNode.end()) return it->second;
    const int64_t id = (int64_t)nodeCoor.size();
    lattNode.emplace(key, id);
    nodeCoor.push_back(xyz);
    nodeLatt.push_back(latt);
    nodeLevel.push_back(0);
    nodeParents.emplace_back();
    return id;
}

int64_t MULTIGRID::ADD_ELEMENT(const TreeElem& e) {
    elemVect.push_back(e);
    maxiLeve = std::max<int64_t>(maxiLeve, e.level);
    return (int64_t)elemVect.size() - 1;
}

void MULTIGRID::REFINE_ALL() {
    const int64_t ne = (int64_t)elemVect.size();
    for (int64_t e = 0; e < ne; ++e) {
        if (!elemVect[e].leaf()) continue;
        const std::array<int64_t, 8> corn = elemVect[e].cornNode;
        const int lev = elemVect[e].level;
        int64_t grid[3][3][3];
        for (int k = 0; k < 8; ++k) grid[kCornerPos[k][0]][kCornerPos[k][1]][kCornerPos[k][2]] = corn[k];
        for (int t = 0; t < 19; ++t) {
            const int* q = kNewPos[t];
            std::vector<int64_t> par;
            for (int k = 0; k < 8; ++k) {
                bool on = true;
                for (int a = 0; a < 3; ++a) on &= (q[a] == 1 || q[a] == kCornerPos[k][a]);
                if (on) par.push_back(corn[k]);
            }
            std::sort(par.begin(), par.end());
            std::array<int64_t, 3> latt{0, 0, 0};
            std::array<double, 3> xyz{0.0, 0.0, 0.0};
            for (int64_t p : par)
                for (int a = 0; a < 3; ++a) {
                    latt[a] += nodeLatt[p][a];
                    xyz[a] = xyz[a] + nodeCoor[p][a];
                }
            for (int a = 0; a < 3; ++a) {
                if (latt[a] % (int64_t)par.size()) throw std::runtime_error("lattice too coarse for refinement");
                latt[a] /= (int64_t)par.size();
                xyz[a] = xyz[a] / (double)par.size();
            }
            const int64_t before = numNodes();
            const int64_t id = TRY_ADD_NODE(latt, xyz);
            if (id == before) {
                nodeLevel[id] = lev + 1;
                nodeParents[id] = par;
            }
            grid[q[0]][q[1]][q[2]] = id;
        }
        elemVect[e].firstChild = (int64_t)elemVect.size();
        elemVect[e].refiPatt = 0;
        for (int c = 0; c < 8; ++c) elemVect[e].children.push_back((int64_t)elemVect.size() + c);
        for (int c = 0; c < 8; ++c) {
            TreeElem ch;
            ch.parent = e;
            ch.level = lev + 1;
            for (int m = 0; m < 8; ++m)
                ch.cornNode[m] = grid[(c & 1) + kHexOff[m][0]][((c >> 1) & 1) + kHexOff[m][1]][((c >> 2) & 1) + kHexOff[m][2]];
            ADD_ELEMENT(ch);
        }
    }
}

// ---------------------------------------------------------------------------------- local refinement
namespace {

// The 12 edges and 6 faces every element registers (PREP.h hexaLine / hexaFace; ADD_ELEMENT,
// MULTIGRID.h:335-373)
const int kHexLine[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {4, 5}, {5, 6}, {6, 7}, {7, 4}};
const int kHexFace[6][4] = {{0, 3, 2, 1}, {4, 5, 6, 7}, {0, 4, 7, 3}, {1, 2, 6, 5}, {0, 1, 5, 4}, {3, 7, 6, 2}};

// Refinement patterns (PREP.h TREE_ELEM::refiPatt; MULTIGRID.h:382-478): the positions on the
// element's 3x3x3 subdivision grid (corners at 0 / 2) of the nodes a pattern creates, in creation
// order -- a node's parents are the corners matching it on every coordinate that is not 1 -- and
// the children: corner grid position + (0/1 per kHexOff) x the child's extent, children in order.
const std::vector<std::vector<std::array<int, 3>>> kPattNew = {
    {{1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {0, 0, 1}, {2, 0, 1}, {2, 2, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 2},
     {1, 2, 2}, {0, 1, 2}, {0, 1, 1}, {2, 1, 1}, {1, 0, 1}, {1, 2, 1}, {1, 1, 0}, {1, 1, 2}, {1, 1, 1}},
    {{1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {1, 0, 2}, {2, 1, 2}, {1, 2, 2}, {0, 1, 2}, {1, 1, 0}, {1, 1, 2}},
    {{0, 1, 0}, {0, 2, 1}, {0, 1, 2}, {0, 0, 1}, {2, 1, 0}, {2, 2, 1}, {2, 1, 2}, {2, 0, 1}, {0, 1, 1}, {2, 1, 1}},
    {{0, 0, 1}, {1, 0, 2}, {2, 0, 1}, {1, 0, 0}, {0, 2, 1}, {1, 2, 2}, {2, 2, 1}, {1, 2, 0}, {1, 0, 1}, {1, 2, 1}},
    {{1, 0, 0}, {1, 2, 0}, {1, 0, 2}, {1, 2, 2}},
    {{0, 1, 0}, {2, 1, 0}, {0, 1, 2}, {2, 1, 2}},
    {{0, 0, 1}, {2, 0, 1}, {0, 2, 1}, {2, 2, 1}}};
const std::vector<std::vector<std::array<int, 3>>> kPattChild = {
    {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}, {0, 0, 1}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}},
    {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}},
    {{0, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 1, 1}},
    {{0, 0, 0}, {0, 0, 1}, {1, 0, 0}, {1, 0, 1}},
    {{0, 0, 0}, {1, 0, 0}},
    {{0, 0, 0}, {0, 1, 0}},
    {{0, 0, 0}, {0, 0, 1}}};
const std::array<int, 3> kPattExtent[7] = {{1, 1, 1}, {1, 1, 2}, {2, 1, 1}, {1, 2, 1}, {1, 2, 2}, {2, 1, 2}, {2, 2, 1}};
// GRLE_CHECK (MULTIGRID.h:551-614): per parent pattern and child, the parent's edges / faces (corner
// indices) the child lies on -- a leaf neighbour using one of them must be refined too
const std::vector<std::vector<std::vector<std::array<int, 2>>>> kPareLine = {
    {{{0, 1}, {0, 3}, {0, 4}}, {{1, 0}, {1, 2}, {1, 5}}, {{3, 0}, {3, 2}, {3, 7}}, {{2, 1}, {2, 3}, {2, 6}},
     {{4, 0}, {4, 5}, {4, 7}}, {{5, 1}, {5, 4}, {5, 6}}, {{7, 3}, {7, 6}, {7, 4}}, {{6, 2}, {6, 5}, {6, 7}}},
    {{{0, 1}, {0, 3}, {4, 5}, {4, 7}}, {{1, 0}, {1, 2}, {5, 4}, {5, 6}}, {{3, 0}, {3, 2}, {7, 4}, {7, 6}},
     {{2, 1}, {2, 3}, {6, 5}, {6, 7}}},
    {{{0, 3}, {0, 4}, {1, 2}, {1, 5}}, {{3, 0}, {3, 7}, {2, 1}, {2, 6}}, {{4, 0}, {4, 7}, {5, 1}, {5, 6}},
     {{7, 3}, {7, 4}, {6, 2}, {6, 5}}},
    {{{0, 1}, {0, 4}, {3, 2}, {3, 7}}, {{4, 0}, {4, 5}, {7, 3}, {7, 6}}, {{1, 0}, {1, 5}, {2, 3}, {2, 6}},
     {{5, 1}, {5, 4}, {6, 2}, {6, 7}}},
    {{{0, 1}, {4, 5}, {2, 3}, {7, 6}}, {{0, 1}, {4, 5}, {2, 3}, {7, 6}}},
    {{{0, 3}, {1, 2}, {4, 7}, {5, 6}}, {{0, 3}, {1, 2}, {4, 7}, {5, 6}}},
    {{{0, 4}, {1, 5}, {3, 7}, {2, 6}}, {{0, 4}, {1, 5}, {3, 7}, {2, 6}}}};
const std::vector<std::vector<std::vector<std::array<int, 4>>>> kPareFace = {
    {{{0, 1, 2, 3}, {0, 3, 7, 4}, {0, 4, 5, 1}}, {{1, 2, 3, 0}, {1, 2, 6, 5}, {1, 0, 4, 5}},
     {{3, 0, 1, 2}, {3, 7, 4, 0}, {3, 7, 6, 2}}, {{2, 3, 0, 1}, {2, 6, 5, 1}, {2, 3, 7, 6}},
     {{4, 5, 6, 7}, {4, 0, 3, 7}, {4, 5, 1, 0}}, {{5, 6, 7, 4}, {5, 1, 2, 6}, {5, 1, 0, 4}},
     {{7, 4, 5, 6}, {7, 4, 0, 3}, {7, 6, 2, 3}}, {{6, 7, 4, 5}, {6, 5, 1, 2}, {6, 2, 3, 7}}},
    {{{0, 1, 2, 3}, {0, 3, 7, 4}, {0, 4, 5, 1}, {4, 5, 6, 7}}, {{1, 2, 3, 0}, {1, 2, 6, 5}, {1, 0, 4, 5}, {5, 6, 7, 4}},
     {{3, 0, 1, 2}, {3, 7, 4, 0}, {3, 7, 6, 2}, {7, 4, 5, 6}}, {{2, 3, 0, 1}, {2, 6, 5, 1}, {2, 3, 7, 6}, {6, 7, 4, 5}}},
    {{{0, 3, 7, 4}, {1, 2, 6, 5}, {0, 4, 5, 1}, {0, 1, 2, 3}}, {{3, 7, 4, 0}, {2, 6, 5, 1}, {3, 7, 6, 2}, {3, 0, 1, 2}},
     {{4, 0, 3, 7}, {5, 1, 2, 6}, {4, 5, 6, 7}, {4, 5, 1, 0}}, {{7, 4, 0, 3}, {6, 5, 1, 2}, {7, 6, 2, 3}, {7, 4, 5, 6}}},
    {{{0, 4, 5, 1}, {3, 7, 6, 2}, {0, 3, 7, 4}, {0, 1, 2, 3}}, {{4, 5, 1, 0}, {7, 6, 2, 3}, {4, 5, 6, 7}, {4, 0, 3, 7}},
     {{1, 0, 4, 5}, {2, 3, 7, 6}, {1, 2, 3, 0}, {1, 2, 6, 5}}, {{5, 1, 0, 4}, {6, 2, 3, 7}, {5, 6, 7, 4}, {5, 1, 2, 6}}},
    {{{0, 1, 2, 3}, {0, 4, 5, 1}, {4, 5, 6, 7}, {3, 7, 6, 2}}, {{0, 1, 2, 3}, {0, 4, 5, 1}, {4, 5, 6, 7}, {3, 7, 6, 2}}},
    {{{0, 3, 7, 4}, {4, 5, 6, 7}, {1, 2, 6, 5}, {0, 1, 2, 3}}, {{0, 3, 7, 4}, {4, 5, 6, 7}, {1, 2, 6, 5}, {0, 1, 2, 3}}},
    {{{0, 4, 5, 1}, {3, 7, 6, 2}, {0, 3, 7, 4}, {1, 2, 6, 5}}, {{0, 4, 5, 1}, {3, 7, 6, 2}, {0, 3, 7, 4}, {1, 2, 6, 5}}}};

}  // namespace

int64_t MULTIGRID::TRY_ADD_COOR(const std::array<double, 3>& xyz) {
    if (coorNode.empty())
        for (int64_t i = 0; i < numNodes(); ++i) coorNode.emplace(nodeCoor[i], i);
    auto it = coorNode.find(xyz);
    if (it != coorNode.end()) return it->second;
    const int64_t id = numNodes();
    coorNode.emplace(xyz, id);
    nodeCoor.push_back(xyz);
    nodeLatt.clear();  // a general tree has no lattice
    nodeLevel.push_back(0);
    nodeParents.emplace_back();
    return id;
}

void MULTIGRID::GRLE_CHECK(std::set<int64_t>& split) {
    // lineUsed / faceUsed (ADD_ELEMENT, MULTIGRID.h:338-369): every element using an edge / face
    std::map<std::vector<int64_t>, std::vector<int64_t>> used;
    for (int64_t e = 0; e < (int64_t)elemVect.size(); ++e) {
        const auto& c = elemVect[e].cornNode;
        for (const auto& ln : kHexLine) {
            std::vector<int64_t> k{c[ln[0]], c[ln[1]]};
            std::sort(k.begin(), k.end());
            used[k].push_back(e);
        }
        for (const auto& f : kHexFace) {
            std::vector<int64_t> k{c[f[0]], c[f[1]], c[f[2]], c[f[3]]};
            std::sort(k.begin(), k.end());
            used[k].push_back(e);
        }
    }
    std::set<int64_t> front = split;
    for (;;) {
        std::set<int64_t> added;
        auto visit = [&](std::vector<int64_t> key) {
            std::sort(key.begin(), key.end());
            const auto it = used.find(key);
            if (it == used.end()) return;
            for (int64_t n : it->second)
                if (elemVect[n].leaf() && !split.count(n)) {
                    added.insert(n);
                    elemVect[n].refiPatt = 0;
                }
        };
        for (int64_t e : front) {
            const TreeElem& t = elemVect[e];
            if (t.parent < 0) continue;
            const TreeElem& P = elemVect[t.parent];
            const int p = P.refiPatt;
            const auto pos = std::find(P.children.begin(), P.children.end(), e);
            if (p < 0 || p > 6 || pos == P.children.end()) throw std::invalid_argument("GRLE_CHECK: child not in its parent");
            const size_t isub = (size_t)(pos - P.children.begin());
            if (isub >= kPareLine[p].size()) throw std::invalid_argument("GRLE_CHECK: child index beyond the pattern");
            for (const auto& ln : kPareLine[p][isub]) visit({P.cornNode[ln[0]], P.cornNode[ln[1]]});
            for (const auto& f : kPareFace[p][isub]) visit({P.cornNode[f[0]], P.cornNode[f[1]], P.cornNode[f[2]], P.cornNode[f[3]]});
        }
        if (added.empty()) break;
        front = added;
        split.insert(added.begin(), added.end());
    }
}

void MULTIGRID::REFINE(std::set<int64_t>& split, const std::map<int64_t, std::set<int>>& spliFlag,
                       const std::map<std::vector<int64_t>, std::array<double, 3>>& planSurf) {
    for (int64_t e : split)
        if (e < 0 || e >= (int64_t)elemVect.size() || !elemVect[e].leaf()) throw std::invalid_argument("REFINE: not a leaf element");
    GRLE_CHECK(split);
    std::set<int64_t> next;
    for (int64_t e : split) {
        const std::array<int64_t, 8> corn = elemVect[e].cornNode;
        const int s = elemVect[e].refiPatt;
        if (s < 0 || s > 6) throw std::invalid_argument("REFINE: element without a refinement pattern 0..6");
        int64_t grid[3][3][3];
        for (int k = 0; k < 8; ++k) grid[kCornerPos[k][0]][kCornerPos[k][1]][kCornerPos[k][2]] = corn[k];
        for (const auto& q : kPattNew[s]) {
            std::vector<int64_t> par;
            for (int k = 0; k < 8; ++k) {
                bool on = true;
                for (int a = 0; a < 3; ++a) on &= (q[a] == 1 || q[a] == kCornerPos[k][a]);
                if (on) par.push_back(corn[k]);
            }
            std::sort(par.begin(), par.end());
            const auto ps = planSurf.find(par);
            std::array<double, 3> xyz{0.0, 0.0, 0.0};
            if (ps != planSurf.end()) {
                xyz = ps->second;
            } else {
                for (int64_t p : par)
                    for (int a = 0; a < 3; ++a) xyz[a] = xyz[a] + nodeCoor[p][a];
                for (int a = 0; a < 3; ++a) xyz[a] = xyz[a] / (double)par.size();
            }
            grid[q[0]][q[1]][q[2]] = TRY_ADD_COOR(xyz);
        }
        const auto& ext = kPattExtent[s];
        for (const auto& b : kPattChild[s]) {
            TreeElem ch;
            ch.parent = e;
            ch.level = elemVect[e].level + 1;
            for (int m = 0; m < 8; ++m)
                ch.cornNode[m] = grid[b[0] + kHexOff[m][0] * ext[0]][b[1] + kHexOff[m][1] * ext[1]][b[2] + kHexOff[m][2] * ext[2]];
            const int64_t id = ADD_ELEMENT(ch);  // may reallocate elemVect
            elemVect[e].children.push_back(id);
        }
        const auto fl = spliFlag.find(e);
        if (fl != spliFlag.end())
            for (int c : fl->second) {
                if (c < 0 || c >= (int)elemVect[e].children.size()) throw std::invalid_argument("REFINE: spliFlag child out of range");
                next.insert(elemVect[e].children[c]);
            }
    }
    split.swap(next);
}

// ---------------------------------------------------------------------------------- transfer
void MULTIGRID::TRANSFER() {
    const int64_t N = numNodes();
    // uniform refinement of a generator (REFINE_ALL, no coupling): node ids are already the
    // reference's positions and every new node's parents are recorded -- the fast path below is
    // the general algorithm's result on such a tree (tests/test_host_operators.py checks that)
    bool fast = !force_general && coupNode.empty() && coupReps < 0 && (int64_t)nodeLevel.size() == N;
    for (int64_t i = 1; i < N && fast; ++i) fast = nodeLevel[i] >= nodeLevel[i - 1];
    for (const auto& e : elemVect) fast = fast && (e.leaf() ? e.level == maxiLeve : e.firstChild >= 0);
    if (!fast) {
        TRANSFER_GENERAL();
        return;
    }
    general = false;
    leveCount.assign(maxiLeve + 1, 0);
    for (int64_t i = 0; i < N; ++i) leveCount[nodeLevel[i]]++;
    for (int64_t l = 1; l <= maxiLeve; ++l) leveCount[l] += leveCount[l - 1];
    scalProl.assign(maxiLeve, Stencil());
    for (int64_t l = 0; l < maxiLeve; ++l) {
        Stencil& S = scalProl[l];
        S.nc = leveCount[l];
        S.nf = leveCount[l + 1];
        S.ptr.assign(S.nf + 1, 0);
        for (int64_t i = 0; i < S.nf; ++i) {
            if (i < S.nc) {
                S.col.push_back((int32_t)i);
                S.w.push_back(1.0);
            } else {
                const auto& par = nodeParents[i];
                for (int64_t p : par) {
                    S.col.push_back((int32_t)p);
                    S.w.push_back(1.0 / (double)par.size());
                }
            }
            S.ptr[i + 1] = (int64_t)S.col.size();
        }
    }
}

namespace {

// Per refinement pattern, the edges / faces of a refined element whose
// midpoint / centre node the refinement created: {corner a, corner b, child, child corner} and
// {4 corners, child, child corner} (TRANSFER's elemLine / elemFace, MULTIGRID.h:759-792).
struct LineNew { int a, b, child, corner; };
struct FaceNew { int c[4], child, corner; };
const std::vector<std::vector<LineNew>> kPattLine = {
    {{0, 1, 0, 1}, {1, 2, 1, 2}, {2, 3, 3, 3}, {3, 0, 2, 0}, {0, 4, 0, 4}, {1, 5, 1, 5}, {2, 6, 3, 6}, {3, 7, 2, 7},
     {4, 5, 4, 5}, {5, 6, 5, 6}, {6, 7, 7, 7}, {7, 4, 6, 4}},
    {{0, 1, 0, 1}, {1, 2, 1, 2}, {2, 3, 3, 3}, {3, 0, 2, 0}, {4, 5, 0, 5}, {5, 6, 1, 6}, {6, 7, 3, 7}, {7, 4, 2, 4}},
    {{0, 3, 0, 3}, {3, 7, 1, 7}, {7, 4, 3, 4}, {4, 0, 2, 0}, {1, 2, 0, 2}, {2, 6, 1, 6}, {6, 5, 3, 5}, {5, 1, 2, 1}},
    {{0, 4, 0, 4}, {4, 5, 1, 5}, {5, 1, 3, 1}, {1, 0, 2, 0}, {3, 7, 0, 7}, {7, 6, 1, 6}, {6, 2, 3, 2}, {2, 3, 2, 3}},
    {{0, 1, 0, 1}, {2, 3, 0, 2}, {4, 5, 0, 5}, {6, 7, 0, 6}},
    {{0, 3, 0, 3}, {1, 2, 0, 2}, {4, 7, 0, 7}, {5, 6, 0, 6}},
    {{0, 4, 0, 4}, {1, 5, 0, 5}, {3, 7, 0, 7}, {2, 6, 0, 6}}};
const std::vector<std::vector<FaceNew>> kPattFace = {
    {{{0, 1, 2, 3}, 0, 2}, {{4, 5, 6, 7}, 4, 6}, {{0, 3, 7, 4}, 0, 7}, {{1, 2, 6, 5}, 3, 5}, {{0, 4, 5, 1}, 0, 5},
     {{3, 7, 6, 2}, 3, 7}},
    {{{0, 1, 2, 3}, 0, 2}, {{4, 5, 6, 7}, 0, 6}},
    {{{0, 3, 7, 4}, 0, 7}, {{1, 2, 6, 5}, 0, 6}},
    {{{0, 4, 5, 1}, 0, 5}, {{3, 7, 6, 2}, 0, 6}},
    {}, {}, {}};

struct KeyHash {
    size_t operator()(const std::array<int64_t, 4>& k) const {
        uint64_t h = 1469598103934665603ull;
        for (int64_t v : k) h = (h ^ (uint64_t)v) * 1099511628211ull;
        return (size_t)h;
    }
};

}  // namespace

// TRANSFER on any octree (MULTIGRID.h:756-948) + PATCH (722-754), then the node ids are moved to
// the reference's positions.
//   * every edge / face midpoint a refinement created (the pattern's elemLine / elemFace rows) is
//     a node of level (element level + 1) with the edge's 2 / face's 4 corners as parents -- or,
//     when an element using that edge / face is still a leaf (a hanging node), a node of the
//     hanging level maxiLeve + 1 with the parents in prolOper[maxiLeve]; a pattern-0 element's
//     body centre has its 8 corners; the first insertion of a parent set wins (std::map insert)
//   * PATCH moves every hanging node to the average of its parents (the refined surface's
//     position would break the patch test)
//   * positions: level by level, node ids ascending inside a level (std::set order); coupReps on
//     level 0, the other coupled nodes on the hanging level
//   * scalProl[l] (level l+1 <- l): identity on the level-l positions, parents' weights 1/count
//     (duplicates summed: a coupled parent becomes coupReps); prolOper[maxiLeve]'s stencil also
//     maps every coupled node to coupReps
void MULTIGRID::TRANSFER_GENERAL() {
    const int64_t N = numNodes(), L = maxiLeve;
    const int64_t ne = (int64_t)elemVect.size();
    for (auto& e : elemVect)
        if (e.firstChild >= 0 && e.children.empty())
            for (int c = 0; c < 8; ++c) e.children.push_back(e.firstChild + c);
    // does a leaf element use this edge / face (lineUsed / faceUsed, MULTIGRID.h:338-369)?
    std::unordered_map<std::array<int64_t, 4>, bool, KeyHash> leafUse;
    leafUse.reserve((size_t)ne * 10);
    auto reg = [&](std::array<int64_t, 4> k, bool leaf) {
        auto it = leafUse.emplace(k, leaf);
        if (!it.second) it.first->second = it.first->second || leaf;
    };
    for (const auto& e : elemVect) {
        for (const auto& ln : kHexLine) {
            std::array<int64_t, 4> k{std::min(e.cornNode[ln[0]], e.cornNode[ln[1]]), std::max(e.cornNode[ln[0]], e.cornNode[ln[1]]), -1, -1};
            reg(k, e.leaf());
        }
        for (const auto& f : kHexFace) {
            std::array<int64_t, 4> k{e.cornNode[f[0]], e.cornNode[f[1]], e.cornNode[f[2]], e.cornNode[f[3]]};
            std::sort(k.begin(), k.end());
            reg(k, e.leaf());
        }
    }
    std::vector<std::map<std::vector<int64_t>, int64_t>> ininTran(L + 1);
    std::vector<std::set<int64_t>> leveNode_s(L + 2);
    auto child_corner = [&](const TreeElem& e, int child, int corner) {
        if (child >= (int)e.children.size()) throw std::invalid_argument("TRANSFER: refined element without that child");
        const int64_t c = e.children[child];
        if (c < 0 || c >= ne) throw std::invalid_argument("TRANSFER: child index out of range");
        return elemVect[c].cornNode[corner];
    };
    for (const auto& e : elemVect) {
        if (e.level == 0)
            for (int k = 0; k < 8; ++k) leveNode_s[0].insert(e.cornNode[k]);
        if (e.leaf()) continue;
        const int s = e.refiPatt;
        if (s < 0 || s > 6) throw std::invalid_argument("TRANSFER: refined element with refinement pattern outside 0..6");
        if (e.level + 1 > L + 1 || e.level < 0) throw std::invalid_argument("TRANSFER: element level beyond maxiLeve");
        if (s == 0) {
            std::vector<int64_t> corn(e.cornNode.begin(), e.cornNode.end());
            std::sort(corn.begin(), corn.end());
            const int64_t nd = child_corner(e, 0, 6);
            ininTran[e.level].emplace(corn, nd);
            leveNode_s[e.level + 1].insert(nd);
        }
        for (const LineNew& ln : kPattLine[s]) {
            std::vector<int64_t> key{e.cornNode[ln.a], e.cornNode[ln.b]};
            std::sort(key.begin(), key.end());
            const auto it = leafUse.find({key[0], key[1], -1, -1});
            const bool hang = it != leafUse.end() && it->second;
            const int64_t nd = child_corner(e, ln.child, ln.corner);
            const int64_t lv = hang ? L : e.level;
            ininTran[lv].emplace(key, nd);
            leveNode_s[lv + 1].insert(nd);
        }
        for (const FaceNew& fc : kPattFace[s]) {
            std::vector<int64_t> key{e.cornNode[fc.c[0]], e.cornNode[fc.c[1]], e.cornNode[fc.c[2]], e.cornNode[fc.c[3]]};
            std::sort(key.begin(), key.end());
            const auto it = leafUse.find({key[0], key[1], key[2], key[3]});
            const bool hang = it != leafUse.end() && it->second;
            const int64_t nd = child_corner(e, fc.child, fc.corner);
            const int64_t lv = hang ? L : e.level;
            ininTran[lv].emplace(key, nd);
            leveNode_s[lv + 1].insert(nd);
        }
    }
    // PATCH (MULTIGRID.h:722-754): in the map's key order, coordinates summed from zero in the
    // parents' order, then divided by their count
    for (const auto& kv : ininTran[L]) {
        std::array<double, 3> c{0.0, 0.0, 0.0};
        for (int64_t p : kv.first)
            for (int a = 0; a < 3; ++a) c[a] = c[a] + nodeCoor[p][a];
        for (int a = 0; a < 3; ++a) c[a] = c[a] / (double)kv.first.size();
        nodeCoor[kv.second] = c;
    }
    // positions (MULTIGRID.h:884-910)
    std::vector<std::vector<int64_t>> leveNode(L + 2);
    for (int64_t t = 0; t <= L + 1; ++t)
        for (int64_t nd : leveNode_s[t]) {
            if (nd == coupReps) leveNode[0].push_back(nd);
            else if (coupNode.count(nd)) leveNode[L + 1].push_back(nd);
            else leveNode[t].push_back(nd);
        }
    std::vector<int64_t> pos(N, -1);
    posiNode.clear();
    std::vector<int> plev;
    for (int64_t t = 0; t <= L + 1; ++t)
        for (int64_t nd : leveNode[t]) {
            if (nd < 0 || nd >= N) throw std::invalid_argument("TRANSFER: node id out of range");
            if (pos[nd] >= 0) throw std::invalid_argument("TRANSFER: node " + std::to_string(nd) + " on two levels");
            pos[nd] = (int64_t)posiNode.size();
            posiNode.push_back(nd);
            plev.push_back((int)t);
        }
    if ((int64_t)posiNode.size() != N) throw std::invalid_argument("TRANSFER: nodes used by no element");
    const int64_t repPos = coupReps >= 0 ? pos.at(coupReps) : -1;
    // stencils in positions: identity on the level-t positions, the parents with 1/count
    scalProl.assign(L, Stencil());
    int64_t accu = 0;
    for (int64_t t = 0; t <= L; ++t) {
        const int64_t nc = accu + (int64_t)leveNode[t].size(), nf = nc + (int64_t)leveNode[t + 1].size();
        std::vector<std::vector<std::pair<int64_t, double>>> rows(nf);
        for (int64_t r = 0; r < nc; ++r) rows[r].push_back({r, 1.0});
        for (const auto& kv : ininTran[t]) {
            if (coupNode.count(kv.second)) continue;
            const int64_t r = pos[kv.second];
            const double w = 1.0 / (double)kv.first.size();
            for (int64_t p : kv.first) rows.at(r).push_back({coupNode.count(p) ? repPos : pos[p], w});
        }
        if (t == L)
            for (int64_t c : coupNode) rows.at(pos[c]).push_back({repPos, 1.0});
        Stencil S;
        S.nf = nf;
        S.nc = nc;
        S.ptr.assign(nf + 1, 0);
        for (int64_t r = 0; r < nf; ++r) {
            // setFromTriplets: duplicates summed in insertion order, columns ascending
            auto& v = rows[r];
            std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
            for (size_t k = 0; k < v.size();) {
                size_t q = k;
                double w = 0.0;
                for (; q < v.size() && v[q].first == v[k].first; ++q) w += v[q].second;
                if (v[k].first < 0 || v[k].first >= nc) throw std::invalid_argument("TRANSFER: parent outside the coarser levels");
                S.col.push_back((int32_t)v[k].first);
                S.w.push_back(w);
                k = q;
            }
            S.ptr[r + 1] = (int64_t)S.col.size();
        }
        if (t < L) scalProl[t] = std::move(S);
        else hangStencil = std::move(S);
        accu = nc;
    }
    leveCount.assign(L + 1, 0);
    for (int64_t t = 0, acc = 0; t <= L; ++t) leveCount[t] = (acc += (int64_t)leveNode[t].size());
    nodeAll = N > leveCount[L] ? N : 0;
    if (!nodeAll) hangStencil = Stencil();
    // move every node-indexed member to positions (earlTran, MULTIGRID.h:1126-1139)
    auto perm_dofmap = [&](std::map<int64_t, double>& m) {
        std::map<int64_t, double> o;
        for (const auto& kv : m) o.emplace(3 * pos[kv.first / 3] + kv.first % 3, kv.second);
        m.swap(o);
    };
    perm_dofmap(consDofv);
    perm_dofmap(exteForc);
    std::map<int64_t, std::array<double, 9>> rot;
    for (const auto& kv : nodeRota) rot.emplace(pos.at(kv.first), kv.second);
    nodeRota.swap(rot);
    std::set<int64_t> cp;
    for (int64_t c : coupNode) cp.insert(pos[c]);
    coupNode.swap(cp);
    if (coupReps >= 0) coupReps = repPos;
    std::vector<std::array<double, 3>> xyz(N);
    for (int64_t p = 0; p < N; ++p) xyz[p] = nodeCoor[posiNode[p]];
    nodeCoor.swap(xyz);
    if ((int64_t)nodeLatt.size() == N) {
        std::vector<std::array<int64_t, 3>> lt(N);
        for (int64_t p = 0; p < N; ++p) lt[p] = nodeLatt[posiNode[p]];
        nodeLatt.swap(lt);
    }
    nodeLevel = plev;
    nodeParents.assign(N, {});
    lattNode.clear();
    for (auto& e : elemVect)
        for (auto& c : e.cornNode) c = pos[c];
    general = true;
}

// ---------------------------------------------------------------------------------- stiffness
void MULTIGRID::STIF_MATR() {
    const int64_t N = numNodes();
    const double lam = mateElas * matePois / (1.0 + matePois) / (1.0 - 2.0 * matePois);
    const double mu = mateElas / 2.0 / (1.0 + matePois);
    double D[6][6] = {};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) D[a][b] = lam + (a == b ? 2.0 * mu : 0.0);
    D[3][3] = D[4][4] = D[5][5] = mu;
    std::vector<int64_t> leaves;
    for (int64_t e = 0; e < (int64_t)elemVect.size(); ++e)
        if (elemVect[e].leaf()) leaves.push_back(e);
    // colour leaf elements so that one colour shares no node (uniform octree: lattice parity)
    int64_t h = -1;
    bool uniform = !nodeLatt.empty() && !general;
    for (int64_t e : leaves) {
        if (!uniform) break;
        const auto& c0 = nodeLatt[elemVect[e].cornNode[0]];
        int64_t ext = 0;
        for (int k = 1; k < 8; ++k)
            for (int a = 0; a < 3; ++a) ext = std::max<int64_t>(ext, std::llabs(nodeLatt[elemVect[e].cornNode[k]][a] - c0[a]));
        if (h < 0) h = ext;
        if (ext != h) uniform = false;
    }
    std::vector<std::vector<int64_t>> colour(uniform ? 8 : 1);
    for (int64_t e : leaves) {
        if (!uniform) { colour[0].push_back(e); continue; }
        int64_t lo[3] = {INT64_MAX, INT64_MAX, INT64_MAX};
        for (int k = 0; k < 8; ++k)
            for (int a = 0; a < 3; ++a) lo[a] = std::min(lo[a], nodeLatt[elemVect[e].cornNode[k]][a]);
        colour[((lo[0] / h) & 1) | (((lo[1] / h) & 1) << 1) | (((lo[2] / h) & 1) << 2)].push_back(e);
    }
    // node adjacency (nodes sharing a leaf element): flat buffer of 64 candidates per node,
    // filled colour by colour (no two elements of a colour share a node), then sort + unique
    {
        std::vector<int32_t> cnt(N, 0), flat(N * 64);
        for (const auto& list : colour) {
#pragma omp parallel for schedule(static) if (uniform)
            for (int64_t t = 0; t < (int64_t)list.size(); ++t) {
                const TreeElem& el = elemVect[list[t]];
                for (int a = 0; a < 8; ++a) {
                    const int64_t r = el.cornNode[a];
                    if (cnt[r] + 8 > 64) throw std::runtime_error("STIF_MATR: node in more than 8 elements");
                    for (int b = 0; b < 8; ++b) flat[r * 64 + cnt[r] + b] = (int32_t)el.cornNode[b];
                    cnt[r] += 8;
                }
            }
        }
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) {
            int32_t* b = &flat[i * 64];
            std::sort(b, b + cnt[i]);
            cnt[i] = (int32_t)(std::unique(b, b + cnt[i]) - b);
        }
        origStif = Bsr3();
        origStif.nb = origStif.mb = N;
        origStif.ptr.assign(N + 1, 0);
        for (int64_t i = 0; i < N; ++i) origStif.ptr[i + 1] = origStif.ptr[i] + cnt[i];
        origStif.col.resize(origStif.ptr[N]);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) std::copy(&flat[i * 64], &flat[i * 64] + cnt[i], origStif.col.begin() + origStif.ptr[i]);
        origStif.val.assign(9 * origStif.ptr[N], 0.0);
    }
    for (const auto& list : colour) {
#pragma omp parallel if (uniform)
        {
            double KE[24][24];
            double Xlast[8][3];
            bool have = false;
#pragma omp for schedule(static)
            for (int64_t t = 0; t < (int64_t)list.size(); ++t) {
                const TreeElem& el = elemVect[list[t]];
                double X[8][3], R[8][3];
                double ext = 0.0;
                for (int k = 0; k < 8; ++k)
                    for (int a = 0; a < 3; ++a) {
                        X[k][a] = nodeCoor[el.cornNode[k]][a];
                        R[k][a] = X[k][a] - X[0][a];
                        ext = std::max(ext, std::abs(R[k][a]));
                    }
                // congruent element (same corner offsets up to last-bit noise of the refined
                // coordinates): reuse the previous element stiffness
                bool same = have;
                for (int k = 0; k < 8 && same; ++k)
                    for (int a = 0; a < 3; ++a) same &= std::abs(R[k][a] - Xlast[k][a]) <= 1e-13 * ext;
                if (!same) {
                    element_stiffness(X, D, KE);
                    for (int k = 0; k < 8; ++k)
                        for (int a = 0; a < 3; ++a) Xlast[k][a] = R[k][a];
                    have = true;
                }
                for (int a = 0; a < 8; ++a) {
                    const int64_t r = el.cornNode[a];
                    const int32_t* cb = &origStif.col[origStif.ptr[r]];
                    const int64_t len = origStif.ptr[r + 1] - origStif.ptr[r];
                    for (int b = 0; b < 8; ++b) {
                        const int64_t pos = origStif.ptr[r] + (std::lower_bound(cb, cb + len, (int32_t)el.cornNode[b]) - cb);
                        double* blk = origStif.block(pos);
                        for (int i = 0; i < 3; ++i)
                            for (int j = 0; j < 3; ++j) blk[3 * i + j] += KE[3 * a + i][3 * b + j];
                    }
                }
            }
        }
    }
}

double MULTIGRID::GET_VOLUME() const {
    const HexQuad& q = hexquad();
    const int64_t ne = (int64_t)elemVect.size();
    const int64_t part = 50000;
    const int64_t np = (ne + part - 1) / part;
    std::vector<double> pv(np, 0.0);
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < np; ++p)
        for (int64_t e = p * part; e < std::min(ne, (p + 1) * part); ++e) {
            if (!elemVect[e].leaf()) continue;
            double X[8][3], J[3][3];
            for (int k = 0; k < 8; ++k)
                for (int a = 0; a < 3; ++a) X[k][a] = nodeCoor[elemVect[e].cornNode[k]][a];
            for (int g = 0; g < 27; ++g) pv[p] += q.w[g] * jacobian(q.dN[g], X, J);
        }
    double v = 0.0;
    for (double x : pv) v += x;
    return v;
}

void MULTIGRID::ADD_NODAL(const Csr& A) {
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t i = r / 3, j = A.col[k] / 3;
            const int32_t* cb = &origStif.col[origStif.ptr[i]];
            const int64_t len = origStif.ptr[i + 1] - origStif.ptr[i];
            const int32_t* hit = std::lower_bound(cb, cb + len, (int32_t)j);
            if (hit == cb + len || *hit != j) throw std::runtime_error("ADD_NODAL: entry outside stiffness pattern");
            origStif.block(origStif.ptr[i] + (hit - cb))[3 * (r % 3) + (A.col[k] % 3)] += A.val[k];
        }
}

// ---------------------------------------------------------------------------------- constraints
void MULTIGRID::LOAD_ACCU(int64_t dof, double v) {
    if (consDofv.count(dof)) return;  // MULTIGRID.h:1084-1100: loads on constrained dofs dropped
    auto it = exteForc.find(dof);
    if (it == exteForc.end()) exteForc.emplace(dof, v);
    else it->second = it->second + v;
}

void MULTIGRID::FLAGS() {
    const int64_t N = numNodes();
    const int64_t L = maxiLeve;
    // consFlag over every position (the hanging level's too); the condensed numbering and the
    // prescribed values cover the MGPIS fine level only (consOper[maxiLeve], dispForc:
    // MULTIGRID.h:1186-1204)
    const int64_t NL = leveCount.empty() ? N : leveCount[L];
    consFlag.assign(3 * N, 1);
    std::vector<double> dfull(3 * N, 0.0);
    for (const auto& kv : consDofv) {
        consFlag[kv.first] = 0;
        dfull[kv.first] = kv.second;
    }
    freeIndex.assign(3 * N, -1);
    freeCount.assign(L + 1, 0);
    int64_t nf = 0;
    dispForc.clear();
    for (int64_t d = 0; d < 3 * NL; ++d) {
        if (consFlag[d]) freeIndex[d] = (int32_t)nf++;
        else dispForc.push_back(dfull[d]);
    }
    for (int64_t l = 0; l <= L; ++l) {
        int64_t c = 0;
        for (int64_t d = 0; d < 3 * leveCount[l]; ++d) c += consFlag[d];
        freeCount[l] = c;
    }
}

namespace {
// prolOper's blocks from a position stencil (MULTIGRID.h:1147-1178): an entry between a fine node
// and a parent of which exactly one is rotated becomes w R_off^T (fine node rotated) or w R_par
// (parent rotated); both rotated: w I ("only one pattern of nodeRota"); the coupled nodes' map to
// coupReps stays w I.  Identity rows of the coarse nodes are never rotated.
Stencil rotate_stencil(const Stencil& S, const std::map<int64_t, std::array<double, 9>>& rot,
                       const std::set<int64_t>& coup, int64_t reps) {
    Stencil P = S;
    P.bent.clear();
    P.bval.clear();
    if (rot.empty()) return P;
    for (int64_t r = S.nc; r < S.nf; ++r)
        for (int64_t k = S.ptr[r]; k < S.ptr[r + 1]; ++k) {
            const int64_t c = S.col[k];
            const auto ro = rot.find(r), rp = rot.find(c);
            if (ro == rot.end() && rp == rot.end()) continue;
            if (c == reps && coup.count(r)) continue;
            if (ro != rot.end() && rp != rot.end()) continue;
            const double w = S.w[k];
            double B[9];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b)
                    B[3 * a + b] = ro != rot.end() ? w * ro->second[3 * b + a] : w * rp->second[3 * a + b];
            P.w[k] = 0.0;
            P.bent.push_back(k);
            P.bval.insert(P.bval.end(), B, B + 9);
        }
    return P;
}

// y (nc nodes) = P^T x (nf nodes), P = S (x) I3 + block entries
void stencil_apply_t(const Stencil& S, const double* x, double* y) {
    std::vector<int64_t> blk_of(S.col.size(), -1);
    for (size_t q = 0; q < S.bent.size(); ++q) blk_of[S.bent[q]] = (int64_t)q;
    for (int64_t r = 0; r < S.nf; ++r)
        for (int64_t k = S.ptr[r]; k < S.ptr[r + 1]; ++k) {
            const int64_t c = S.col[k];
            if (blk_of[k] >= 0) {
                const double* B = &S.bval[9 * blk_of[k]];
                for (int b = 0; b < 3; ++b) y[3 * c + b] += B[b] * x[3 * r] + B[3 + b] * x[3 * r + 1] + B[6 + b] * x[3 * r + 2];
            } else {
                for (int a = 0; a < 3; ++a) y[3 * c + a] += S.w[k] * x[3 * r + a];
            }
        }
}
}  // namespace

void MULTIGRID::PROL_OPER() {
    if (!prolOper.empty() || scalProl.size() != (size_t)maxiLeve) return;
    for (int64_t l = 0; l < maxiLeve; ++l) prolOper.push_back(rotate_stencil(scalProl[l], nodeRota, coupNode, coupReps));
    prolHang = nodeAll ? rotate_stencil(hangStencil, nodeRota, coupNode, coupReps) : Stencil();
}

void MULTIGRID::CONSTRAINT() {
    const int64_t N = numNodes();
    const int64_t L = maxiLeve;
    const int64_t NL = leveCount[L];
    // R^T K R on the rotated nodes (MULTIGRID.h:1105-1124)
    Bsr3 K = origStif;
    if (!nodeRota.empty()) {
        auto R = [&](int64_t i) -> const double* {
            auto it = nodeRota.find(i);
            return it == nodeRota.end() ? nullptr : it->second.data();
        };
        static const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < K.nb; ++i) {
            const double* Ri = R(i);
            for (int64_t k = K.ptr[i]; k < K.ptr[i + 1]; ++k) {
                const double* Rj = R(K.col[k]);
                if (!Ri && !Rj) continue;
                const double* A = Ri ? Ri : I3;
                const double* Bm = Rj ? Rj : I3;
                double* blk = K.block(k);
                double T[9], O[9];
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) T[3 * a + b] = blk[3 * a] * Bm[b] + blk[3 * a + 1] * Bm[3 + b] + blk[3 * a + 2] * Bm[6 + b];
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) O[3 * a + b] = A[a] * T[b] + A[3 + a] * T[3 + b] + A[6 + a] * T[6 + b];
                std::copy(O, O + 9, blk);
            }
        }
    }
    prolOper.clear();
    PROL_OPER();
    // the hanging level's Galerkin step, then the hierarchy (MULTIGRID.h:1182-1184)
    levelStif.assign(L + 1, Bsr3());
    levelStif[L] = nodeAll ? galerkin_rap(K, prolHang) : std::move(K);
    for (int64_t l = L - 1; l >= 0; --l) levelStif[l] = galerkin_rap(levelStif[l + 1], prolOper[l]);
    FLAGS();
    // consForc = consOper (prolOper[maxiLeve]^T f - K_L d), loads not rotated, d the prescribed
    // values of the fine level's constrained dofs (MULTIGRID.h:1186-1243)
    std::vector<double> f(3 * N, 0.0);
    for (const auto& kv : exteForc) f[kv.first] += kv.second;
    std::vector<double> fL(3 * NL, 0.0);
    if (nodeAll) stencil_apply_t(prolHang, f.data(), fL.data());
    else fL = f;
    std::vector<double> dL(3 * NL, 0.0);
    for (const auto& kv : consDofv)
        if (kv.first < 3 * NL) dL[kv.first] = kv.second;
    std::vector<double> Kd(3 * NL, 0.0);
    if (!consDofv.empty()) levelStif[L].apply(dL.data(), Kd.data());
    consForc.assign(freeCount[L], 0.0);
    for (int64_t d = 0; d < 3 * NL; ++d)
        if (freeIndex[d] >= 0) consForc[freeIndex[d]] = fL[d] - Kd[d];
}

void MULTIGRID::ADDITIONAL_FORCE(const double* f_nodal, double* f_free) const {
    // consOper prolOper[maxiLeve]^T f (position numbering: earlTran is the identity here)
    const int64_t n = 3 * numNodes(), nL = 3 * leveCount[maxiLeve];
    std::vector<double> fL(f_nodal, f_nodal + nL);
    if (nodeAll) {
        std::fill(fL.begin(), fL.end(), 0.0);
        stencil_apply_t(prolHang, f_nodal, fL.data());
    }
    (void)n;
    for (int64_t d = 0; d < nL; ++d)
        if (freeIndex[d] >= 0) f_free[freeIndex[d]] = fL[d];
}

void MULTIGRID::OUTP_SUB1(const double* x_free, double* u_nodal) const {
    // the fine level: free values and the prescribed ones; the hanging level: prolOper[maxiLeve]'s rows
    const int64_t nL = 3 * leveCount[maxiLeve];
    for (int64_t d = 0; d < nL; ++d) u_nodal[d] = freeIndex[d] >= 0 ? x_free[freeIndex[d]] : 0.0;
    for (const auto& kv : consDofv)
        if (kv.first < nL) u_nodal[kv.first] = kv.second;
    if (nodeAll) {
        const Csr Hr = hangRows();
        for (int64_t r = 0; r < Hr.nrow; ++r) {
            double s = 0.0;
            for (int64_t k = Hr.ptr[r]; k < Hr.ptr[r + 1]; ++k) s += Hr.val[k] * u_nodal[Hr.col[k]];
            u_nodal[nL + r] = s;
        }
    }
}

Csr MULTIGRID::hangRows() const {
    Csr H;
    const int64_t NL = leveCount[maxiLeve], N = nodeAll ? nodeAll : NL;
    H.nrow = 3 * (N - NL);
    H.ncol = 3 * NL;
    H.ptr.assign(H.nrow + 1, 0);
    if (!nodeAll) return H;
    const Stencil& S = prolHang.nf ? prolHang : hangStencil;
    std::vector<int64_t> blk_of(S.col.size(), -1);
    for (size_t q = 0; q < S.bent.size(); ++q) blk_of[S.bent[q]] = (int64_t)q;
    for (int64_t i = NL; i < N; ++i)
        for (int a = 0; a < 3; ++a) {
            std::vector<std::pair<int32_t, double>> row;
            for (int64_t k = S.ptr[i]; k < S.ptr[i + 1]; ++k) {
                const int64_t c = S.col[k];
                if (blk_of[k] >= 0)
                    for (int b = 0; b < 3; ++b) row.push_back({(int32_t)(3 * c + b), S.bval[9 * blk_of[k] + 3 * a + b]});
                else
                    row.push_back({(int32_t)(3 * c + a), S.w[k]});
            }
            std::sort(row.begin(), row.end());
            for (const auto& e : row) {
                H.col.push_back(e.first);
                H.val.push_back(e.second);
            }
            H.ptr[3 * (i - NL) + a + 1] = (int64_t)H.col.size();
        }
    return H;
}

Csr MULTIGRID::consStif(int64_t level) const {
    return condense(levelStif[level], freeIndex, freeCount[level]);
}

Csr MULTIGRID::realProl(int64_t level) const {
    // consOper[l+1] prolOper[l] consOper[l]^T (MULTIGRID.h:1246-1249); rotated blocks expanded
    const Stencil& S = (int64_t)prolOper.size() > level ? prolOper[level] : scalProl[level];
    std::vector<int64_t> blk_of(S.col.size(), -1);
    for (size_t q = 0; q < S.bent.size(); ++q) blk_of[S.bent[q]] = (int64_t)q;
    Csr P;
    P.nrow = freeCount[level + 1];
    P.ncol = freeCount[level];
    P.ptr.assign(P.nrow + 1, 0);
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t i = 0; i < S.nf; ++i)
        for (int a = 0; a < 3; ++a) {
            const int32_t r = freeIndex[3 * i + a];
            if (r < 0) continue;
            row.clear();
            for (int64_t k = S.ptr[i]; k < S.ptr[i + 1]; ++k) {
                const int64_t j = S.col[k];
                if (blk_of[k] >= 0) {
                    for (int b = 0; b < 3; ++b) {
                        const int32_t c = freeIndex[3 * j + b];
                        if (c >= 0) row.push_back({c, S.bval[9 * blk_of[k] + 3 * a + b]});
                    }
                } else {
                    const int32_t c = freeIndex[3 * j + a];
                    if (c >= 0) row.push_back({c, S.w[k]});
                }
            }
            std::sort(row.begin(), row.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            for (const auto& e : row) {
                P.col.push_back(e.first);
                P.val.push_back(e.second);
            }
            P.ptr[r + 1] = (int64_t)P.col.size();
        }
    return P;
}

// ---------------------------------------------------------------------------------- builders
void build_beam(MULTIGRID& g, const int64_t divi[3], int64_t globLeve, const int64_t doma[3], int64_t tg) {
    const double PI = std::acos(-1.0);
    const double leng[3] = {1.0, 0.12, 0.06};
    const double lengFact = 1.0 / 3.0;
    const double angl = 45.0 * PI / 180.0;
    const double loadInte = -8000.0;
    const int64_t real[3] = {divi[0] / doma[0], divi[1] / doma[1], divi[2] / doma[2]};
    const int64_t t0 = tg / (doma[1] * doma[2]);
    const int64_t t1 = (tg % (doma[1] * doma[2])) / doma[2];
    const int64_t t2 = (tg % (doma[1] * doma[2])) % doma[2];
    const int64_t scale = int64_t(1) << globLeve;
    std::vector<int64_t> id((real[0] + 1) * (real[1] + 1) * (real[2] + 1));
    auto I = [&](int64_t i, int64_t j, int64_t k) { return (i * (real[1] + 1) + j) * (real[2] + 1) + k; };
    for (int64_t i = 0; i <= real[0]; ++i) {
        const int64_t ir = t0 * real[0] + i;
        const double x = leng[0] / divi[0] * ir;
        const double heig = leng[1] * (1.0 - (double)ir / divi[0] * lengFact);
        const double widt = leng[2] * (1.0 - (double)ir / divi[0] * lengFact);
        for (int64_t j = 0; j <= real[1]; ++j) {
            const int64_t jr = t1 * real[1] + j;
            const double y = -heig / 2.0 + heig / divi[1] * (double)jr;
            for (int64_t k = 0; k <= real[2]; ++k) {
                const int64_t kr = t2 * real[2] + k;
                const double z = -widt / 2.0 + widt / divi[2] * (double)kr;
                id[I(i, j, k)] = g.TRY_ADD_NODE({ir * scale, jr * scale, kr * scale}, {x, y, z});
            }
        }
    }
    for (int64_t i = 0; i < real[0]; ++i)
        for (int64_t j = 0; j < real[1]; ++j)
            for (int64_t k = 0; k < real[2]; ++k) {
                TreeElem e;
                e.cornNode = {id[I(i, j, k)],         id[I(i, j + 1, k)],         id[I(i, j + 1, k + 1)],
                              id[I(i, j, k + 1)],     id[I(i + 1, j, k)],         id[I(i + 1, j + 1, k)],
                              id[I(i + 1, j + 1, k + 1)], id[I(i + 1, j, k + 1)]};
                g.ADD_ELEMENT(e);
            }
    for (int64_t r = 0; r < globLeve; ++r) g.REFINE_ALL();
    if (g.maxiLeve < 0) g.maxiLeve = 0;
    // COOR_ADJU (BEAM.h:79-99): twist about the x axis, angle proportional to x
    for (auto& c : g.nodeCoor) {
        const double a = 1.0 * (angl * c[0] / leng[0]);
        const double y = std::cos(a) * c[1] - std::sin(a) * c[2];
        const double z = std::sin(a) * c[1] + std::cos(a) * c[2];
        c[1] = y;
        c[2] = z;
    }
    // SUBR_COLO, loadType 0 (BEAM.h:101-141)
    for (int64_t n = 0; n < g.numNodes(); ++n)
        if (g.nodeCoor[n][0] <= 1.0e-10)
            for (int a = 0; a < 3; ++a) g.consDofv.emplace(3 * n + a, 0.0);
    static const int kLine[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {0, 4}, {1, 5},
                                     {2, 6}, {3, 7}, {4, 5}, {5, 6}, {6, 7}, {7, 4}};
    for (const auto& el : g.elemVect) {
        if (el.firstChild >= 0) continue;
        for (const auto& ln : kLine) {
            const int64_t n0 = el.cornNode[ln[0]], n1 = el.cornNode[ln[1]];
            bool on = true;
            for (int64_t n : {n0, n1})
                if (std::abs(g.nodeCoor[n][1]) > 1.0e-10 || std::abs(g.nodeCoor[n][2]) > 1.0e-10) on = false;
            if (!on) continue;
            const double f = loadInte * std::abs(g.nodeCoor[n0][0] - g.nodeCoor[n1][0]) / 2.0 / 4.0;
            for (int64_t n : {n0, n1})
                if (g.nodeCoor[n][0] > 1.0e-10) g.LOAD_ACCU(3 * n + 2, f);
        }
    }
}

void build_box(MULTIGRID& g, const double lo[3], const double hi[3], const int64_t n[3], int64_t globLeve,
               const int64_t latt_off[3]) {
    const int64_t scale = int64_t(1) << globLeve;
    const int64_t o[3] = {latt_off ? latt_off[0] : 0, latt_off ? latt_off[1] : 0, latt_off ? latt_off[2] : 0};
    std::vector<int64_t> id((n[0] + 1) * (n[1] + 1) * (n[2] + 1));
    auto I = [&](int64_t i, int64_t j, int64_t k) { return (i * (n[1] + 1) + j) * (n[2] + 1) + k; };
    for (int64_t i = 0; i <= n[0]; ++i)
        for (int64_t j = 0; j <= n[1]; ++j)
            for (int64_t k = 0; k <= n[2]; ++k)
                id[I(i, j, k)] = g.TRY_ADD_NODE({(o[0] + i) * scale, (o[1] + j) * scale, (o[2] + k) * scale},
                                                {lo[0] + (hi[0] - lo[0]) / n[0] * i, lo[1] + (hi[1] - lo[1]) / n[1] * j,
                                                 lo[2] + (hi[2] - lo[2]) / n[2] * k});
    for (int64_t i = 0; i < n[0]; ++i)
        for (int64_t j = 0; j < n[1]; ++j)
            for (int64_t k = 0; k < n[2]; ++k) {
                TreeElem e;
                e.cornNode = {id[I(i, j, k)],     id[I(i + 1, j, k)],     id[I(i + 1, j + 1, k)],     id[I(i, j + 1, k)],
                              id[I(i, j, k + 1)], id[I(i + 1, j, k + 1)], id[I(i + 1, j + 1, k + 1)], id[I(i, j + 1, k + 1)]};
                g.ADD_ELEMENT(e);
            }
    for (int64_t r = 0; r < globLeve; ++r) g.REFINE_ALL();
    if (g.maxiLeve < 0) g.maxiLeve = 0;
}

}  // namespace ddpca

// C ABI: host problem construction (setup-only restatement of MULTIGRID / MCONTACT::ESTABLISH).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <exception>
#include <map>
#include <set>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>

#include "../../include/ddpca_amd.h"
#include "common.hpp"
#include "mcontact.hpp"
#include "problem.hpp"

using namespace ddpca;

namespace {

const int kHexFace[6][4] = {{0, 3, 2, 1}, {4, 5, 6, 7}, {0, 4, 7, 3}, {1, 2, 6, 5}, {0, 1, 5, 4}, {3, 7, 6, 2}};

// Leaf-element faces of g whose four corners satisfy latt[axis] == value, in EFACE_SURFACE
// order (elements by id, faces in hexaFace order, CSEARCH.h:50-80).
std::vector<std::array<int64_t, 4>> plane_faces(const MULTIGRID& g, int axis, int64_t value) {
    std::vector<std::array<int64_t, 4>> out;
    for (const auto& el : g.elemVect) {
        if (el.firstChild >= 0) continue;
        for (const auto& f : kHexFace) {
            bool on = true;
            std::array<int64_t, 4> nodes;
            for (int k = 0; k < 4; ++k) {
                nodes[k] = el.cornNode[f[k]];
                on &= g.nodeLatt[nodes[k]][axis] == value;
            }
            if (on) out.push_back(nodes);
        }
    }
    return out;
}

// A conforming interface pairs every face of one side with a face of the other: the same count on
// both sides of the plane, and (checked per face below) a mate for every slave face -- otherwise
// the interface would silently lose integration points.
void check_face_match(size_t nm, size_t ns, int axis) {
    if (nm == 0 || nm != ns)
        throw std::invalid_argument("conforming interface on axis " + std::to_string(axis) + ": " + std::to_string(nm) +
                                    " master faces vs " + std::to_string(ns) + " slave faces");
}

// Conforming interface on a shared lattice plane: master faces of body m, slave faces of body
// s; integration points in CONTACT_SEARCH order (slave segments, CSEARCH.h:777-817).
void conforming_interface(const MULTIGRID& gm, const MULTIGRID& gs, int axis, int64_t value,
                          std::vector<IntegralPoint>& ips, int sub = 1) {
    auto key = [](const MULTIGRID& g, const std::array<int64_t, 4>& f) {
        std::array<std::array<int64_t, 3>, 4> k;
        for (int i = 0; i < 4; ++i) k[i] = g.nodeLatt[f[i]];
        std::sort(k.begin(), k.end());
        return k;
    };
    std::map<std::array<std::array<int64_t, 3>, 4>, std::array<int64_t, 4>> mast;
    const auto mf = plane_faces(gm, axis, value), sf = plane_faces(gs, axis, value);
    for (const auto& f : mf) mast.emplace(key(gm, f), f);
    check_face_match(mf.size(), sf.size(), axis);
    for (const auto& f : sf) {
        auto it = mast.find(key(gs, f));
        if (it == mast.end()) throw std::invalid_argument("conforming interface: a slave face without its master face");
        conforming_face_ips(gm, it->second.data(), gs, f.data(), ips, sub);
    }
}

// The same on a general tree (local refinement: the new nodes carry no lattice coordinates):
// leaf faces on the coordinate plane x[axis] == value, matched by their corners' coordinates.
std::vector<std::array<int64_t, 4>> plane_faces_xyz(const MULTIGRID& g, int axis, double value) {
    std::vector<std::array<int64_t, 4>> out;
    for (const auto& el : g.elemVect) {
        if (!el.leaf()) continue;
        for (const auto& f : kHexFace) {
            bool on = true;
            std::array<int64_t, 4> nodes;
            for (int k = 0; k < 4; ++k) {
                nodes[k] = el.cornNode[f[k]];
                on &= std::abs(g.nodeCoor[nodes[k]][axis] - value) <= 1e-12;
            }
            if (on) out.push_back(nodes);
        }
    }
    return out;
}

void conforming_interface_xyz(const MULTIGRID& gm, const MULTIGRID& gs, int axis, double value,
                              std::vector<IntegralPoint>& ips, int sub) {
    auto key = [](const MULTIGRID& g, const std::array<int64_t, 4>& f) {
        std::array<std::array<int64_t, 3>, 4> k;
        for (int i = 0; i < 4; ++i)
            for (int a = 0; a < 3; ++a) k[i][a] = std::llround(g.nodeCoor[f[i]][a] * 1.0e9);
        std::sort(k.begin(), k.end());
        return k;
    };
    std::map<std::array<std::array<int64_t, 3>, 4>, std::array<int64_t, 4>> mast;
    const auto mf = plane_faces_xyz(gm, axis, value), sf = plane_faces_xyz(gs, axis, value);
    for (const auto& f : mf) mast.emplace(key(gm, f), f);
    check_face_match(mf.size(), sf.size(), axis);
    for (const auto& f : sf) {
        auto it = mast.find(key(gs, f));
        if (it == mast.end()) throw std::invalid_argument("conforming interface: a slave face without its master face");
        conforming_face_ips(gm, it->second.data(), gs, f.data(), ips, sub);
    }
}

void face_traction(MULTIGRID& g, int axis, int64_t value, const double t[3]) {
    for (const auto& el : g.elemVect) {
        if (el.firstChild >= 0) continue;
        for (const auto& f : kHexFace) {
            bool on = true;
            for (int k = 0; k < 4; ++k) on &= g.nodeLatt[el.cornNode[f[k]]][axis] == value;
            if (!on) continue;
            double c[4][3];
            for (int k = 0; k < 4; ++k)
                for (int a = 0; a < 3; ++a) c[k][a] = g.nodeCoor[el.cornNode[f[k]]][a];
            double u[3], v[3];
            for (int a = 0; a < 3; ++a) { u[a] = c[2][a] - c[0][a]; v[a] = c[3][a] - c[1][a]; }
            const double cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2], cz = u[0] * v[1] - u[1] * v[0];
            const double area = 0.5 * std::sqrt(cx * cx + cy * cy + cz * cz);
            for (int k = 0; k < 4; ++k)
                for (int d = 0; d < 3; ++d) g.LOAD_ACCU(3 * el.cornNode[f[k]] + d, t[d] * area / 4.0);
        }
    }
}

void set_penalty(Problem& P) {
    const double charLeng = P.mc.GET_CHAR_LENG();
    for (auto& itf : P.mc.searCont) itf.penN = itf.penF = 210.0e9 * 25.0 / charLeng;
}

void make_beam(Problem& P, const double* q) {
    const int64_t divi[3] = {(int64_t)q[0], (int64_t)q[1], (int64_t)q[2]};
    const int64_t gl = (int64_t)q[3];
    const int64_t doma[3] = {(int64_t)q[4], (int64_t)q[5], (int64_t)q[6]};
    const int64_t nsub = doma[0] * doma[1] * doma[2];
    for (int a = 0; a < 3; ++a)
        if (divi[a] <= 0 || doma[a] <= 0 || divi[a] % doma[a]) throw std::invalid_argument("beam: diviNumb must be divisible by domaNumb");
    P.mc.multGrid.resize(nsub);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t tg = 0; tg < nsub; ++tg) build_beam(P.mc.multGrid[tg], divi, gl, doma, tg);
    if (nsub == 1) return;
    // interface numbering of BEAM::SOLVE_DD (BEAM.h:428-470)
    const int64_t xyzN[3] = {(doma[0] - 1) * doma[1] * doma[2], (doma[1] - 1) * doma[0] * doma[2],
                             (doma[2] - 1) * doma[0] * doma[1]};
    P.mc.searCont.resize(xyzN[0] + xyzN[1] + xyzN[2]);
    const int64_t scale = int64_t(1) << gl;
    const int64_t real[3] = {divi[0] / doma[0], divi[1] / doma[1], divi[2] / doma[2]};
    std::vector<std::array<int64_t, 3>> plane(P.mc.searCont.size());  // axis, value
    for (int64_t t0 = 0; t0 < doma[0]; ++t0)
        for (int64_t t1 = 0; t1 < doma[1]; ++t1)
            for (int64_t t2 = 0; t2 < doma[2]; ++t2) {
                const int64_t m = t0 * doma[1] * doma[2] + t1 * doma[2] + t2;
                if (t0 <= doma[0] - 2) {
                    const int64_t ts = m;
                    P.mc.searCont[ts].body[0] = m;
                    P.mc.searCont[ts].body[1] = m + doma[1] * doma[2];
                    plane[ts] = {0, (t0 + 1) * real[0] * scale, 0};
                }
                if (t1 <= doma[1] - 2) {
                    const int64_t ts = xyzN[0] + t1 * doma[0] * doma[2] + t0 * doma[2] + t2;
                    P.mc.searCont[ts].body[0] = m;
                    P.mc.searCont[ts].body[1] = m + doma[2];
                    plane[ts] = {1, (t1 + 1) * real[1] * scale, 0};
                }
                if (t2 <= doma[2] - 2) {
                    const int64_t ts = xyzN[0] + xyzN[1] + t2 * doma[0] * doma[1] + t0 * doma[1] + t1;
                    P.mc.searCont[ts].body[0] = m;
                    P.mc.searCont[ts].body[1] = m + 1;
                    plane[ts] = {2, (t2 + 1) * real[2] * scale, 0};
                }
            }
    std::vector<std::exception_ptr> err(P.mc.searCont.size());
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t ts = 0; ts < (int64_t)P.mc.searCont.size(); ++ts) {
        Interface& itf = P.mc.searCont[ts];
        itf.fric = -1.0;
        try {
            conforming_interface(P.mc.multGrid[itf.body[0]], P.mc.multGrid[itf.body[1]], (int)plane[ts][0], plane[ts][1], itf.ip);
        } catch (...) {
            err[ts] = std::current_exception();
        }
    }
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    set_penalty(P);
}

void make_twoblock(Problem& P, const double* q) {
    const double fric = q[0];
    const int64_t gl = (int64_t)q[1];
    const double L = 0.02, H = 0.01, p = 1.0e7;
    const int64_t n[3] = {2, 2, 1};
    P.mc.multGrid.resize(2);
    const double lo0[3] = {0, 0, 0}, hi0[3] = {L, L, H}, lo1[3] = {0, 0, H}, hi1[3] = {L, L, 2 * H};
    const int64_t off0[3] = {0, 0, 0}, off1[3] = {0, 0, n[2]};
    build_box(P.mc.multGrid[0], lo0, hi0, n, gl, off0);
    build_box(P.mc.multGrid[1], lo1, hi1, n, gl, off1);
    for (int b = 0; b < 2; ++b) {
        MULTIGRID& g = P.mc.multGrid[b];
        for (int64_t i = 0; i < g.numNodes(); ++i) {
            const auto& c = g.nodeCoor[i];
            if (c[0] <= 1e-12 && (b == 0 || fric == 0.0)) g.consDofv.emplace(3 * i + 0, 0.0);
            if (c[1] <= 1e-12) g.consDofv.emplace(3 * i + 1, 0.0);
            if (b == 0 && c[2] <= 1e-12) g.consDofv.emplace(3 * i + 2, 0.0);
        }
    }
    const int64_t scale = int64_t(1) << gl;
    const double t[3] = {fric > 0 ? 0.5 * fric * p : 0.0, 0.0, -p};
    face_traction(P.mc.multGrid[1], 2, 2 * n[2] * scale, t);
    P.mc.searCont.resize(1);
    Interface& itf = P.mc.searCont[0];
    itf.body[0] = 0;
    itf.body[1] = 1;
    itf.fric = fric;
    conforming_interface(P.mc.multGrid[0], P.mc.multGrid[1], 2, n[2] * scale, itf.ip);
    set_penalty(P);
}

// Synthetic DEHW-shaped chain: G groups; group g = worm block W_g
// (subdomain 2g, z in [0,H]) under wheel block H_g (subdomain 2g+1, z in [H,2H]) with a
// frictional contact (interface g, master = worm); worm blocks glued along x
// (interfaces G + g), wheel blocks glued along x (interfaces 2G - 1 + g).  Worm bottom on
// rollers (uz = 0), both chains clamped at x = 0, wheel tops loaded by pressure p and shear
// 0.5 fric p (partial slip).  E = 210e9 (worm) / 110e9 (wheel) as in DEHW.h:2248.
// q[6], q[7] (optional, default 0): integration density of the contact / glued faces -- each face
// integrated over 2^k x 2^k polygons, as against a slave surface mesh 2^k times finer (DEHW's
// adaptively refined contact bands, DEHW.h:1562, 2079, carry ~0.8 integration points per DOF).
void make_dehw(Problem& P, const double* q, int nq) {
    const int64_t G = (int64_t)q[0];
    const int64_t n[3] = {(int64_t)q[1], (int64_t)q[2], (int64_t)q[3]};
    const int64_t gl = (int64_t)q[4];
    const double fric = q[5];
    const int kc = nq > 6 ? (int)q[6] : 0, kg = nq > 7 ? (int)q[7] : 0;
    // DEHW's general-mesh features (q[8], q[9], default off):
    //   band: the contact band refined once more (DEHW.h:1562, 2079: adaptively refined contact
    //         zones): the layer of elements on either side of each worm/wheel contact plane is cut
    //         with pattern 0 (MULTIGRID::REFINE + GRLE_CHECK) -- a general tree, renumbered by
    //         TRANSFER, whose band/bulk faces leave hanging nodes on the level past the MGPIS
    //         hierarchy; the contact faces (and the glued faces in the band) are the refined ones
    //   rot:  nodal frames on the worms' supported faces (DEHW.h:197, 272, 352: the hub's rotated
    //         nodes): each node of a worm's bottom face off the glued planes is rotated about x by
    //         an angle varying with y and supported along its local z (a curved roller bed) --
    //         prolongation blocks off w I, R^T K R, CONSTRAINT with nodeRota (MULTIGRID.h:1102-1255)
    const bool band = nq > 8 && q[8] != 0.0, rot = nq > 9 && q[9] != 0.0;
    //   uneven (q[10], default off): group g is (1 + g mod 3) times n[0] cells long in x -- subdomains
    //         of three sizes, as DEHW's 52 uneven subdomains (DEHW.h:2238-2258) that LPT packs onto ranks
    const bool uneven = nq > 10 && q[10] != 0.0;
    if (G < 1) throw std::invalid_argument("dehw: ngroups >= 1");
    if (kc < 0 || kc > 4 || kg < 0 || kg > 4) throw std::invalid_argument("dehw: integration refinement in [0, 4]");
    const double h = 0.01;  // cubic coarse elements
    const double Ly = n[1] * h, H = n[2] * h, p = 1.0e7;
    std::vector<int64_t> nxg(G), xo(G + 1, 0);  // per group: cells along x, first cell
    for (int64_t g = 0; g < G; ++g) {
        nxg[g] = uneven ? n[0] * (1 + g % 3) : n[0];
        xo[g + 1] = xo[g] + nxg[g];
    }
    P.mc.multGrid.resize(2 * G);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t s = 0; s < 2 * G; ++s) {
        const int64_t g = s / 2, wheel = s % 2;
        const double lo[3] = {xo[g] * h, 0.0, wheel * H}, hi[3] = {xo[g + 1] * h, Ly, (wheel + 1) * H};
        const int64_t off[3] = {xo[g], 0, wheel * n[2]}, ng[3] = {nxg[g], n[1], n[2]};
        MULTIGRID& m = P.mc.multGrid[s];
        if (wheel) m.mateElas = 110.0e9;
        build_box(m, lo, hi, ng, gl, off);
        if (wheel) {  // (on the lattice, before any local refinement)
            const double t[3] = {0.5 * fric * p, 0.0, -p};
            face_traction(m, 2, 2 * n[2] * (int64_t(1) << gl), t);
        }
        if (band) {
            // the element layer touching the contact plane (lattice z = n[2] 2^gl)
            const int64_t zc = n[2] * (int64_t(1) << gl);
            std::set<int64_t> split;
            for (int64_t e = 0; e < (int64_t)m.elemVect.size(); ++e) {
                if (!m.elemVect[e].leaf()) continue;
                int on = 0;
                for (int64_t c : m.elemVect[e].cornNode) on += m.nodeLatt[c][2] == zc;
                if (on == 4) {
                    m.elemVect[e].refiPatt = 0;
                    split.insert(e);
                }
            }
            m.REFINE(split, {}, {});
        }
        for (int64_t i = 0; i < m.numNodes(); ++i) {
            const auto& c = m.nodeCoor[i];
            if (g == 0 && c[0] <= 1e-12)
                for (int a = 0; a < 3; ++a) m.consDofv.emplace(3 * i + a, 0.0);
            if (!wheel && c[2] <= 1e-12) {
                m.consDofv.emplace(3 * i + 2, 0.0);
                // (not on the glued x planes: a rotated node's dofs are in its own frame, as the
                // reference's, which the interface operators would mix with the mate's)
                if (rot && c[0] > lo[0] + 1e-12 && c[0] < hi[0] - 1e-12) {
                    const double th = 0.3 * (c[1] / Ly - 0.5), cs = std::cos(th), sn = std::sin(th);
                    m.nodeRota.emplace(i, std::array<double, 9>{1.0, 0.0, 0.0, 0.0, cs, -sn, 0.0, sn, cs});
                }
            }
        }
    }
    const int64_t scale = int64_t(1) << gl;
    const int64_t nint = G + 2 * (G - 1);
    P.mc.searCont.resize(nint);
    std::vector<std::array<int64_t, 2>> plane(nint);
    for (int64_t g = 0; g < G; ++g) {
        P.mc.searCont[g].body[0] = 2 * g;
        P.mc.searCont[g].body[1] = 2 * g + 1;
        P.mc.searCont[g].fric = fric;
        plane[g] = {2, n[2] * scale};
    }
    for (int64_t g = 0; g + 1 < G; ++g)
        for (int64_t w = 0; w < 2; ++w) {
            const int64_t ts = G + w * (G - 1) + g;
            P.mc.searCont[ts].body[0] = 2 * g + w;
            P.mc.searCont[ts].body[1] = 2 * (g + 1) + w;
            P.mc.searCont[ts].fric = -1.0;
            plane[ts] = {0, xo[g + 1] * scale};
        }
    std::vector<std::exception_ptr> err(nint);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t ts = 0; ts < nint; ++ts) {
      try {
        Interface& itf = P.mc.searCont[ts];
        const int k = ts < G ? kc : kg;
        if (band) {
            // refined contact faces are half as wide: one subdivision level less keeps the
            // integration points per unit area
            const int ke = ts < G ? std::max(k - 1, 0) : k;
            const double v = (double)plane[ts][1] / (double)scale * h;
            conforming_interface_xyz(P.mc.multGrid[itf.body[0]], P.mc.multGrid[itf.body[1]], (int)plane[ts][0], v, itf.ip,
                                     1 << ke);
        } else {
            conforming_interface(P.mc.multGrid[itf.body[0]], P.mc.multGrid[itf.body[1]], (int)plane[ts][0], plane[ts][1],
                                 itf.ip, 1 << k);
        }
      } catch (...) {
        err[ts] = std::current_exception();
      }
    }
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    set_penalty(P);
}

template <typename T> int dtype_of();
template <> int dtype_of<double>() { return 0; }
template <> int dtype_of<int64_t>() { return 1; }
template <> int dtype_of<int32_t>() { return 2; }
template <> int dtype_of<uint8_t>() { return 3; }

template <typename T>
int put(const std::vector<T>& v, const void** data, int64_t* count, int* dtype) {
    *data = v.data();
    *count = (int64_t)v.size();
    *dtype = dtype_of<T>();
    return DDPCA_OK;
}

}  // namespace

extern "C" {

int ddpca_problem_create(const char* kind, const double* params, int nparams, ddpca_problem_t* out) {
    return guarded([&] {
        if (!kind || !out) throw ApiError(DDPCA_EINVAL, "null argument");
        auto P = std::make_unique<Problem>();
        const std::string k(kind);
        if (k == "beam") {
            if (nparams < 7) throw ApiError(DDPCA_EINVAL, "beam needs 7 params");
            make_beam(*P, params);
        } else if (k == "twoblock") {
            if (nparams < 2) throw ApiError(DDPCA_EINVAL, "twoblock needs 2 params");
            make_twoblock(*P, params);
        } else if (k == "dehw") {
            if (nparams < 6) throw ApiError(DDPCA_EINVAL, "dehw needs 6 params");
            make_dehw(*P, params, nparams);
        } else {
            throw ApiError(DDPCA_EINVAL, "unknown problem kind " + k);
        }
        *out = reinterpret_cast<ddpca_problem_t>(P.release());
    });
}

int ddpca_problem_set_ips(ddpca_problem_t h, int64_t ts, int64_t n, const int64_t* node, const double* shap,
                          const double* basis, const double* gap, const double* w, double fric, double penN,
                          double penF) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(h);
        if (ts < 0 || ts >= (int64_t)P.mc.searCont.size()) throw ApiError(DDPCA_EINVAL, "interface index");
        if (P.established) throw ApiError(DDPCA_ESTATE, "set_ips after establish");
        Interface& itf = P.mc.searCont[ts];
        itf.ip.resize(n);
        for (int64_t q = 0; q < n; ++q) {
            IntegralPoint& p = itf.ip[q];
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    p.node[s][k] = node[8 * q + 4 * s + k];
                    p.shap[s][k] = shap[8 * q + 4 * s + k];
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) p.basis[a][b] = basis[9 * q + 3 * a + b];
            p.gap = gap[q];
            p.w = w[q];
        }
        itf.fric = fric;
        itf.penN = penN;
        itf.penF = penF;
    });
}

int ddpca_problem_set_coarse(ddpca_problem_t h, int64_t muscSett, const int64_t* doleMcsc) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(h);
        if (P.established) throw ApiError(DDPCA_ESTATE, "set_coarse after establish");
        if (muscSett < 0 || muscSett > 2) throw ApiError(DDPCA_EINVAL, "muscSett must be 0, 1 (MULTISCALE) or 2 (MULTISCALE_1)");
        P.mc.muscSett = muscSett;
        const int64_t nsub = (int64_t)P.mc.multGrid.size();
        P.mc.doleMcsc.assign(nsub, 0);
        for (int64_t tv = 0; tv < nsub; ++tv) {
            const int64_t d = doleMcsc ? doleMcsc[tv] : 0;
            if (d < 0 || d > P.mc.multGrid[tv].maxiLeve) throw ApiError(DDPCA_EINVAL, "doleMcsc out of range");
            P.mc.doleMcsc[tv] = d;
        }
    });
}

int ddpca_problem_establish(ddpca_problem_t h) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(h);
        if (P.established) return;
        P.mc.ESTABLISH();
        P.owned.assign(P.mc.multGrid.size(), 1);
        P.established = true;
    });
}

int ddpca_problem_establish_owned(ddpca_problem_t h, const int32_t* owner, int rank) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(h);
        if (P.established) throw ApiError(DDPCA_ESTATE, "problem already established");
        if (!owner) throw ApiError(DDPCA_EINVAL, "null owner");
        P.owned.assign(P.mc.multGrid.size(), 0);
        for (size_t tv = 0; tv < P.owned.size(); ++tv) P.owned[tv] = owner[tv] == rank ? 1 : 0;
        P.mc.ESTABLISH(&P.owned);
        P.established = true;
    });
}

int ddpca_problem_destroy(ddpca_problem_t h) {
    delete reinterpret_cast<Problem*>(h);
    return DDPCA_OK;
}

int ddpca_problem_view(ddpca_problem_t h, const char* cname, int64_t index, int64_t level, const void** data,
                       int64_t* count, int* dtype) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(h);
        const std::string name(cname);
        const int64_t nsub = (int64_t)P.mc.multGrid.size(), nint = (int64_t)P.mc.searCont.size();
        if (name == "sizes") {
            auto& v = P.cache_i64["sizes"];
            v = {nsub, nint, P.established ? 1 : 0};
            put(v, data, count, dtype);
            return;
        }
        const std::string key = name + "#" + std::to_string(index) + "#" + std::to_string(level);
        // ---- coarse space (MCONTACT::MULTISCALE_1 output)
        {
            const CoarseSpace& cs = P.mc.coarse;
            auto put_csr = [&](const Csr& m, const std::string& part) {
                if (part == "ptr") put(m.ptr, data, count, dtype);
                else if (part == "col") put(m.col, data, count, dtype);
                else if (part == "val") put(m.val, data, count, dtype);
                else if (part == "shape") { auto& v = P.cache_i64[key]; v = {m.nrow, m.ncol}; put(v, data, count, dtype); }
                else throw ApiError(DDPCA_EINVAL, "csr part");
            };
            auto need = [&] { if (!cs.ready) throw ApiError(DDPCA_ESTATE, "no coarse space (set_coarse before establish)"); };
            if (name == "baseReco") { need(); put(cs.baseReco, data, count, dtype); return; }
            if (name == "globForc_1") { need(); put(cs.globForc_1, data, count, dtype); return; }
            if (name == "doleMcsc") { put(P.mc.doleMcsc, data, count, dtype); return; }
            if (name.rfind("globCoup_1:", 0) == 0) { need(); put_csr(cs.globCoup_1, name.substr(11)); return; }
            // LATIN-type (MULTISCALE) right-hand-side operators, index = 2*ts + side
            for (const char* base : {"globTran:", "globTran_pena:", "globTran_D:"}) {
                const std::string b(base);
                if (name.rfind(b, 0) != 0) continue;
                need();
                if (!cs.latin) throw ApiError(DDPCA_ESTATE, "not a LATIN-type coarse space (muscSett = 1)");
                if (index < 0 || index >= 2 * nint) throw ApiError(DDPCA_EINVAL, "side index");
                const auto& M = b == "globTran:" ? cs.globTran_L : b == "globTran_pena:" ? cs.globTran_pena_L : cs.globTran_D_L;
                put_csr(M[index / 2][index % 2], name.substr(b.size()));
                return;
            }
            if (name.rfind("globTran_1:", 0) == 0) {
                need();
                if (index < 0 || index >= 2 * nint) throw ApiError(DDPCA_EINVAL, "side index");
                put_csr(cs.globTran_1[index / 2][index % 2], name.substr(11));
                return;
            }
            for (const char* base : {"globTran_D_1:", "accuProl:"}) {
                const std::string b(base);
                if (name.rfind(b, 0) != 0) continue;
                need();
                if (index < 0 || index >= nsub || !cs.built[index]) throw ApiError(DDPCA_EINVAL, "subdomain index");
                const std::string ck = b + std::to_string(index);
                auto it = P.cache_csr.find(ck);
                if (it == P.cache_csr.end() && !cs.assembled && b[0] == 'g') {
                    // the first globTran_D_1 view assembles every built subdomain's at once, in
                    // parallel (Rc consStif[L] products: ~35 s per 1.2M-dof subdomain on one core);
                    // MCONTACT::globTran_D_1 only reads the established hierarchy
                    std::vector<int64_t> todo;
                    for (int64_t t = 0; t < nsub; ++t)
                        if (cs.built[t] && !P.cache_csr.count(b + std::to_string(t))) todo.push_back(t);
                    std::vector<Csr> out(todo.size());
                    std::vector<std::exception_ptr> err(todo.size());
#pragma omp parallel for schedule(dynamic, 1)
                    for (int64_t k = 0; k < (int64_t)todo.size(); ++k) {
                        try {
                            out[k] = P.mc.globTran_D_1(todo[k]);
                        } catch (...) {
                            err[k] = std::current_exception();
                        }
                    }
                    for (auto& e : err)
                        if (e) std::rethrow_exception(e);
                    for (size_t k = 0; k < todo.size(); ++k)
                        P.cache_csr.emplace(b + std::to_string(todo[k]), std::move(out[k]));
                    it = P.cache_csr.find(ck);
                }
                if (it == P.cache_csr.end()) {
                    Csr m = cs.assembled ? (b[0] == 'g' ? cs.globTran_D_full[index] : cs.accuProl_full[index])
                                         : (b[0] == 'g' ? P.mc.globTran_D_1(index) : P.mc.accuProl(index));
                    it = P.cache_csr.emplace(ck, std::move(m)).first;
                }
                put_csr(it->second, name.substr(b.size()));
                return;
            }
        }
        // ---- interface-side arrays: index = 2*ts + side
        static const char* kSideCsr[] = {"systMass", "systTran", "systTran_pena", "inteMass", "inteMass_pena",
                                          "inpoLagr", "inpoDisp", "inteInpo", "pemaInpo_r"};
        for (const char* base : kSideCsr) {
            const std::string b(base);
            if (name.rfind(b + ":", 0) != 0) continue;
            if (index < 0 || index >= 2 * nint) throw ApiError(DDPCA_EINVAL, "side index");
            Interface& itf = P.mc.searCont[index / 2];
            const int s = (int)(index % 2);
            const Csr* m = nullptr;
            if (b == "systMass") m = &itf.systMass[s];
            if (b == "systTran") m = &itf.systTran[s];
            if (b == "systTran_pena") m = &itf.systTran_pena[s];
            if (b == "inteMass") m = &itf.inteMass[s];
            if (b == "inteMass_pena") m = &itf.inteMass_pena[s];
            if (b == "inpoLagr") m = &itf.inpoLagr[s];
            if (b == "inpoDisp") m = &itf.inpoDisp[s];
            if (b == "inteInpo") m = &itf.inteInpo[s];
            if (b == "pemaInpo_r") m = &itf.pemaInpo_r[s];
            const std::string part = name.substr(b.size() + 1);
            if (part == "ptr") put(m->ptr, data, count, dtype);
            else if (part == "col") put(m->col, data, count, dtype);
            else if (part == "val") put(m->val, data, count, dtype);
            else if (part == "shape") { auto& v = P.cache_i64[key]; v = {m->nrow, m->ncol}; put(v, data, count, dtype); }
            else throw ApiError(DDPCA_EINVAL, "csr part");
            return;
        }
        if (name == "nodeCont") {
            put(P.mc.searCont.at(index / 2).nodeCont[index % 2], data, count, dtype);
            return;
        }
        if (name == "iface_param" || name == "iface_body" || name.rfind("ip_", 0) == 0 || name == "inpoNgap" ||
            name == "pemaDiag") {
            if (index < 0 || index >= nint) throw ApiError(DDPCA_EINVAL, "interface index");
            Interface& itf = P.mc.searCont[index];
            if (name == "inpoNgap") { put(itf.inpoNgap, data, count, dtype); return; }
            if (name == "pemaDiag") { put(itf.pemaDiag, data, count, dtype); return; }
            if (name == "iface_param") { auto& v = P.cache_f64[key]; v = {itf.fric, itf.penN, itf.penF}; put(v, data, count, dtype); return; }
            if (name == "iface_body") { auto& v = P.cache_i64[key]; v = {itf.body[0], itf.body[1]}; put(v, data, count, dtype); return; }
            if (name == "ip_node") {
                auto& v = P.cache_i64[key];
                v.clear();
                for (const auto& p : itf.ip)
                    for (int s = 0; s < 2; ++s)
                        for (int k = 0; k < 4; ++k) v.push_back(p.node[s][k]);
                put(v, data, count, dtype);
                return;
            }
            auto& v = P.cache_f64[key];
            v.clear();
            for (const auto& p : itf.ip) {
                if (name == "ip_shap") for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) v.push_back(p.shap[s][k]);
                else if (name == "ip_basis") for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) v.push_back(p.basis[a][b]);
                else if (name == "ip_gap") v.push_back(p.gap);
                else if (name == "ip_w") v.push_back(p.w);
                else throw ApiError(DDPCA_EINVAL, "unknown ip array " + name);
            }
            put(v, data, count, dtype);
            return;
        }
        // ---- subdomain arrays: index = subdomain
        if (index < 0 || index >= nsub) throw ApiError(DDPCA_EINVAL, "subdomain index");
        MULTIGRID& g = P.mc.multGrid[index];
        if (name == "coords") {
            auto& v = P.cache_f64[key];
            v.resize(3 * g.numNodes());
            for (int64_t i = 0; i < g.numNodes(); ++i)
                for (int a = 0; a < 3; ++a) v[3 * i + a] = g.nodeCoor[i][a];
            put(v, data, count, dtype);
        } else if (name == "maxiLeve") {
            auto& v = P.cache_i64[key]; v = {g.maxiLeve}; put(v, data, count, dtype);
        } else if (name == "leveCount") put(g.leveCount, data, count, dtype);
        else if (name == "freeCount") put(g.freeCount, data, count, dtype);
        else if (name == "consFlag") put(g.consFlag, data, count, dtype);
        else if (name == "freeIndex") put(g.freeIndex, data, count, dtype);
        else if (name == "consForc") put(g.consForc, data, count, dtype);
        else if (name == "dispForc") put(g.dispForc, data, count, dtype);
        else if (name == "exteForc") {
            auto& v = P.cache_f64[key];
            v.assign(3 * g.numNodes(), 0.0);
            for (const auto& kv : g.exteForc) v[kv.first] += kv.second;
            put(v, data, count, dtype);
        } else if (name == "consDofv") {
            auto& v = P.cache_i64[key];
            v.clear();
            for (const auto& kv : g.consDofv) v.push_back(kv.first);
            put(v, data, count, dtype);
        } else if (name == "consDofv_val") {
            auto& v = P.cache_f64[key];
            v.clear();
            for (const auto& kv : g.consDofv) v.push_back(kv.second);
            put(v, data, count, dtype);
        } else if (name == "nodeRota") {  // rotated nodes (MULTIGRID::nodeRota keys)
            auto& v = P.cache_i64[key];
            v.clear();
            for (const auto& kv : g.nodeRota) v.push_back(kv.first);
            put(v, data, count, dtype);
        } else if (name == "nodeRota_val") {  // their 3x3 matrices, row-major, 9 per node
            auto& v = P.cache_f64[key];
            v.clear();
            for (const auto& kv : g.nodeRota) v.insert(v.end(), kv.second.begin(), kv.second.end());
            put(v, data, count, dtype);
        } else if (name == "material") {
            auto& v = P.cache_f64[key];
            v = {g.mateElas, g.matePois};
            put(v, data, count, dtype);
        } else if (name.rfind("tree:", 0) == 0) {
            // the element tree as the generator left it (node ids; before establish's TRANSFER renumbers
            // a general tree): corner (8 per element), parent, level, refiPatt, child_ptr, child
            if (P.established && g.general) throw ApiError(DDPCA_ESTATE, "tree views before establish (a general tree is renumbered)");
            const std::string w = name.substr(5);
            auto& v = P.cache_i64[key];
            v.clear();
            if (w == "corner") {
                for (const auto& e : g.elemVect) v.insert(v.end(), e.cornNode.begin(), e.cornNode.end());
            } else if (w == "parent") {
                for (const auto& e : g.elemVect) v.push_back(e.parent);
            } else if (w == "level") {
                for (const auto& e : g.elemVect) v.push_back(e.level);
            } else if (w == "refiPatt") {
                for (const auto& e : g.elemVect) v.push_back(e.leaf() ? 7 : e.refiPatt);
            } else if (w == "child_ptr") {
                v.push_back(0);
                for (const auto& e : g.elemVect)
                    v.push_back(v.back() + (int64_t)(e.children.empty() && e.firstChild >= 0 ? 8 : e.children.size()));
            } else if (w == "child") {
                for (const auto& e : g.elemVect) {
                    if (e.children.empty() && e.firstChild >= 0)
                        for (int c = 0; c < 8; ++c) v.push_back(e.firstChild + c);
                    else v.insert(v.end(), e.children.begin(), e.children.end());
                }
            } else {
                throw ApiError(DDPCA_EINVAL, "unknown tree array " + w);
            }
            put(v, data, count, dtype);
        } else if (name.rfind("K:", 0) == 0 || name.rfind("P:", 0) == 0) {
            const bool isK = name[0] == 'K';
            if (level < 0 || level > g.maxiLeve - (isK ? 0 : 1)) throw ApiError(DDPCA_EINVAL, "level");
            // a rank-local build (establish_owned) leaves other ranks' subdomains without operators
            const bool built = (int64_t)g.freeCount.size() > level + (isK ? 0 : 1) &&
                               (isK ? (int64_t)g.levelStif.size() > level
                                    : (int64_t)std::max(g.prolOper.size(), g.scalProl.size()) > level);
            if (!built) throw ApiError(DDPCA_ESTATE, "operators of subdomain " + std::to_string(index) + " were not built here");
            const std::string ck = std::string(isK ? "K" : "P") + "#" + std::to_string(index) + "#" + std::to_string(level);
            auto it = P.cache_csr.find(ck);
            if (it == P.cache_csr.end()) it = P.cache_csr.emplace(ck, isK ? g.consStif(level) : g.realProl(level)).first;
            const Csr& m = it->second;
            const std::string part = name.substr(2);
            if (part == "ptr") put(m.ptr, data, count, dtype);
            else if (part == "col") put(m.col, data, count, dtype);
            else if (part == "val") put(m.val, data, count, dtype);
            else if (part == "shape") { auto& v = P.cache_i64[key]; v = {m.nrow, m.ncol}; put(v, data, count, dtype); }
            else throw ApiError(DDPCA_EINVAL, "csr part");
        } else if (name.rfind("H:", 0) == 0) {
            // the hanging level's rows of prolOper[maxiLeve] (3 (nodeAll - NL) x 3 NL; empty without one)
            const std::string ck = "H#" + std::to_string(index);
            auto it = P.cache_csr.find(ck);
            if (it == P.cache_csr.end()) {
                if (g.leveCount.empty()) throw ApiError(DDPCA_ESTATE, "subdomain " + std::to_string(index) + " was not built here");
                it = P.cache_csr.emplace(ck, g.hangRows()).first;
            }
            const Csr& m = it->second;
            const std::string part = name.substr(2);
            if (part == "ptr") put(m.ptr, data, count, dtype);
            else if (part == "col") put(m.col, data, count, dtype);
            else if (part == "val") put(m.val, data, count, dtype);
            else if (part == "shape") { auto& v = P.cache_i64[key]; v = {m.nrow, m.ncol}; put(v, data, count, dtype); }
            else throw ApiError(DDPCA_EINVAL, "csr part");
        } else if (name.rfind("B:", 0) == 0) {
            const Bsr3& m = g.levelStif.at(level);
            const std::string part = name.substr(2);
            if (part == "ptr") put(m.ptr, data, count, dtype);
            else if (part == "col") put(m.col, data, count, dtype);
            else if (part == "val") put(m.val, data, count, dtype);
            else throw ApiError(DDPCA_EINVAL, "bsr part");
        } else if (name.rfind("S:", 0) == 0) {
            const Stencil& m = g.scalProl.at(level);
            const std::string part = name.substr(2);
            if (part == "ptr") put(m.ptr, data, count, dtype);
            else if (part == "col") put(m.col, data, count, dtype);
            else if (part == "w") put(m.w, data, count, dtype);
            else throw ApiError(DDPCA_EINVAL, "stencil part");
        } else {
            throw ApiError(DDPCA_EINVAL, "unknown array " + name);
        }
    });
}

}  // extern "C"

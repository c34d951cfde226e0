// Sanitizer driver for the host C++ of libddpca_amd (SURVEY §5 "race detection / sanitizers").
//
// Built by tests/sanitize/Makefile from the host translation units only (capi_builder, capi_host,
// capi_multigrid, csearch, errors, lagrange, mcontact, multigrid, multiscale, sparse, writers) with
// -fsanitize=address,undefined; no device objects, no GPU.  It drives the setup code that produces
// every GPU operand through the C ABI the tests use:
//   * the problem generators (BEAM single / DD, the two-block contact frictionless and Coulomb,
//     the synthetic DEHW chain) -> MCONTACT::ESTABLISH (mortar operators, MCONTACT.h:181-896),
//     MULTIGRID's uniform pipeline (MULTIGRID.h:756-1255), both coarse spaces (MULTISCALE and
//     MULTISCALE_1, MCONTACT.h:898-1536, 1680-1870), the rank-local builds of 2 and 4 ranks;
//     every array and operator the C ABI exposes is read and folded into a checksum;
//   * a general octree through ddpca_multigrid_* (REFINE with all seven patterns and spliFlag
//     chains, GRLE_CHECK, CURVEDS planSurf, TRANSFER with the hanging level, PATCH, STIF_MATR,
//     CONSTRAINT with nodal rotations), then as a problem subdomain;
//   * CSEARCH's contact search and ADAPTIVE_REFINE's selection on two facing surfaces;
//   * the result-file writers;
//   * the refused-argument paths (bad indices, reversed pointers) of those entry points.
// The reference-comparison harnesses (oracle/ref_multigrid, ref_csearch, ref_refine,
// ref_lagrange_host) are linked to the same sanitized objects by the Makefile's `ref` target.
// Exit status 0 and no sanitizer report = clean.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ddpca_amd.h"

namespace {

int g_fail = 0;

void ok(int rc, const char* what) {
    if (rc < 0) {
        std::fprintf(stderr, "FAIL %s: %s\n", what, ddpca_last_error());
        ++g_fail;
    }
}

void refused(int rc, const char* what) {
    if (rc >= 0) {
        std::fprintf(stderr, "FAIL %s: accepted a bad argument\n", what);
        ++g_fail;
    }
}

double fold(const void* d, int64_t n, int dt) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double v = 0.0;
        switch (dt) {
            case 0: v = static_cast<const double*>(d)[i]; break;
            case 1: v = (double)static_cast<const int64_t*>(d)[i]; break;
            case 2: v = (double)static_cast<const int32_t*>(d)[i]; break;
            default: v = (double)static_cast<const uint8_t*>(d)[i]; break;
        }
        s += std::isfinite(v) ? std::fabs(v) * (1.0 + (double)(i % 7)) : 0.0;
    }
    return s;
}

// reads one view; returns its checksum (0 when the view is refused, e.g. no coarse space)
double view(ddpca_problem_t p, const std::string& name, int64_t idx, int64_t lev, bool must = true) {
    const void* d = nullptr;
    int64_t n = 0;
    int dt = 0;
    const int rc = ddpca_problem_view(p, name.c_str(), idx, lev, &d, &n, &dt);
    if (rc < 0) {
        if (must) ok(rc, name.c_str());
        return 0.0;
    }
    return fold(d, n, dt);
}

double view_csr(ddpca_problem_t p, const std::string& base, int64_t idx, int64_t lev, bool must = true) {
    double s = 0.0;
    for (const char* part : {":shape", ":ptr", ":col", ":val"}) s += view(p, base + part, idx, lev, must);
    return s;
}

int64_t view_i64(ddpca_problem_t p, const char* name, int64_t idx, int64_t k) {
    const void* d = nullptr;
    int64_t n = 0;
    int dt = 0;
    ok(ddpca_problem_view(p, name, idx, 0, &d, &n, &dt), name);
    return (d && k < n && dt == 1) ? static_cast<const int64_t*>(d)[k] : 0;
}

// every array and operator of an established problem
double read_all(ddpca_problem_t p, int64_t muscSett, bool latin, const std::vector<uint8_t>& owned) {
    const int64_t nsub = view_i64(p, "sizes", 0, 0), nint = view_i64(p, "sizes", 0, 1);
    double s = 0.0;
    for (int64_t tv = 0; tv < nsub; ++tv) {
        for (const char* a : {"coords", "maxiLeve", "leveCount", "freeCount", "consFlag", "freeIndex", "consForc",
                              "dispForc", "exteForc", "consDofv"})
            s += view(p, a, tv, 0);
        const int64_t L = view_i64(p, "maxiLeve", tv, 0);
        for (int64_t l = 0; l <= L; ++l) {
            if (!owned[tv]) {  // another rank's subdomain: no operators here, refused
                const void* d = nullptr;
                int64_t n = 0;
                int dt = 0;
                refused(ddpca_problem_view(p, "K:ptr", tv, l, &d, &n, &dt), "view K of a subdomain not owned");
                continue;
            }
            s += view_csr(p, "K", tv, l);
            if (l < L) s += view_csr(p, "P", tv, l);
        }
        if (muscSett && owned[tv]) {
            s += view_csr(p, "accuProl", tv, 0);
            if (!latin) s += view_csr(p, "globTran_D_1", tv, 0);
        }
    }
    for (int64_t ts = 0; ts < nint; ++ts) {
        for (const char* a : {"iface_param", "iface_body", "inpoNgap", "pemaDiag", "ip_node", "ip_shap", "ip_basis",
                              "ip_gap", "ip_w"})
            s += view(p, a, ts, 0);
        for (int64_t side = 2 * ts; side < 2 * ts + 2; ++side) {
            s += view(p, "nodeCont", side, 0);
            for (const char* b : {"systMass", "systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr",
                                  "inpoDisp", "inteInpo", "pemaInpo_r"})
                s += view_csr(p, b, side, 0);
            if (muscSett) {
                if (latin)
                    for (const char* b : {"globTran", "globTran_pena", "globTran_D"}) s += view_csr(p, b, side, 0, false);
                else
                    s += view_csr(p, "globTran_1", side, 0, false);
            }
        }
    }
    if (muscSett) {
        s += view(p, "baseReco", 0, 0) + view(p, "globForc_1", 0, 0) + view(p, "doleMcsc", 0, 0);
        s += view_csr(p, "globCoup_1", 0, 0);
    }
    // refused: out-of-range indices and unknown names
    const void* d = nullptr;
    int64_t n = 0;
    int dt = 0;
    refused(ddpca_problem_view(p, "consFlag", nsub, 0, &d, &n, &dt), "view subdomain nsub");
    refused(ddpca_problem_view(p, "consFlag", -1, 0, &d, &n, &dt), "view subdomain -1");
    refused(ddpca_problem_view(p, "ip_w", nint, 0, &d, &n, &dt), "view interface nint");
    refused(ddpca_problem_view(p, "systMass:ptr", 2 * nint, 0, &d, &n, &dt), "view side 2 nint");
    refused(ddpca_problem_view(p, "K:ptr", 0, 99, &d, &n, &dt), "view level 99");
    refused(ddpca_problem_view(p, "no_such_array", 0, 0, &d, &n, &dt), "view unknown name");
    return s;
}

struct Case {
    const char* kind;
    std::vector<double> params;
    int64_t musc;
    int ranks;  // 1: establish; > 1: establish_owned on every rank (contiguous blocks)
};

void run_case(const Case& c) {
    ddpca_problem_t probe = nullptr;
    ok(ddpca_problem_create(c.kind, c.params.data(), (int)c.params.size(), &probe), c.kind);
    if (!probe) return;
    const int64_t nsub = view_i64(probe, "sizes", 0, 0);
    ddpca_problem_destroy(probe);
    for (int r = 0; r < c.ranks; ++r) {
        ddpca_problem_t p = nullptr;
        ok(ddpca_problem_create(c.kind, c.params.data(), (int)c.params.size(), &p), c.kind);
        if (!p) return;
        std::vector<int64_t> dole(nsub, 1);
        if (c.musc) ok(ddpca_problem_set_coarse(p, c.musc, dole.data()), "set_coarse");
        std::vector<int32_t> owner(nsub);
        std::vector<uint8_t> owned(nsub, 1);
        for (int64_t tv = 0; tv < nsub; ++tv) {
            owner[tv] = (int32_t)(tv * c.ranks / nsub);
            owned[tv] = c.ranks == 1 || owner[tv] == r;
        }
        if (c.ranks == 1) ok(ddpca_problem_establish(p), "establish");
        else ok(ddpca_problem_establish_owned(p, owner.data(), r), "establish_owned");
        refused(ddpca_problem_set_coarse(p, 2, dole.data()), "set_coarse after establish");
        const double s = read_all(p, c.musc, c.musc == 1, owned);
        std::printf("{\"case\": \"%s\", \"params\": %zu, \"muscSett\": %ld, \"rank\": %d, \"ranks\": %d, \"checksum\": %.6e}\n",
                    c.kind, c.params.size(), (long)c.musc, r, c.ranks, s);
        ddpca_problem_destroy(p);
    }
}

// ---- a general octree: a 2 x 2 x 1 box refined with every pattern, curved top face
struct Tree {
    std::vector<double> xyz;
    std::vector<int64_t> corner, parent, level, patt, cptr{0}, child;
};

// the curved top face z = 1 + 0.01 (x^2 + y^2): box nodes and CURVEDS grid points coincide bitwise
double top(double x, double y) { return 1.0 + 0.01 * (x * x + y * y); }

Tree box(int nx, int ny, int nz) {
    Tree t;
    auto id = [&](int i, int j, int k) { return (int64_t)(i + (nx + 1) * (j + (ny + 1) * k)); };
    for (int k = 0; k <= nz; ++k)
        for (int j = 0; j <= ny; ++j)
            for (int i = 0; i <= nx; ++i) t.xyz.insert(t.xyz.end(), {(double)i, (double)j, k == nz ? top(i, j) : 0.5 * k});
    for (int k = 0; k < nz; ++k)
        for (int j = 0; j < ny; ++j)
            for (int i = 0; i < nx; ++i) {
                t.corner.insert(t.corner.end(), {id(i, j, k), id(i + 1, j, k), id(i + 1, j + 1, k), id(i, j + 1, k),
                                                 id(i, j, k + 1), id(i + 1, j, k + 1), id(i + 1, j + 1, k + 1),
                                                 id(i, j + 1, k + 1)});
                t.parent.push_back(-1);
                t.level.push_back(0);
                t.patt.push_back(-1);
                t.cptr.push_back(0);
            }
    return t;
}

template <typename T>
std::vector<T> tree_get(ddpca_multigrid_t g, const char* what) {
    const void* d = nullptr;
    int64_t n = 0;
    int dt = 0;
    ok(ddpca_multigrid_tree(g, what, &d, &n, &dt), what);
    const T* p = static_cast<const T*>(d);
    return p ? std::vector<T>(p, p + n) : std::vector<T>();
}

void run_octree() {
    const int nx = 4, ny = 4, nz = 2;
    Tree t = box(nx, ny, nz);
    const int64_t nnode = (int64_t)t.xyz.size() / 3, nelem = (int64_t)t.parent.size();
    ddpca_multigrid_t g = nullptr;
    ok(ddpca_multigrid_create(nnode, t.xyz.data(), nelem, t.corner.data(), t.parent.data(), t.level.data(),
                              t.patt.data(), t.cptr.data(), nullptr, &g),
       "multigrid_create");
    if (!g) return;
    // round 1: every element 8-way, spliFlag on some children (a hanging level in round 2)
    std::vector<int64_t> elem, patt, fe, fc;
    for (int64_t e = 0; e < nelem; ++e) {  // (all seven patterns: ref_multigrid_san "refine")
        elem.push_back(e);
        patt.push_back(0);
    }
    fe = {0, 0, 7};
    fc = {1, 6, 0};
    // a curved top face: CURVEDS point grid over z = 1 + 0.05 (x^2 + y^2), planSurf of the new nodes
    const int64_t ni = 8 * nx + 1, nj = 8 * ny + 1;
    std::vector<double> surf;
    for (int64_t j = 0; j < nj; ++j)
        for (int64_t i = 0; i < ni; ++i) {
            const double x = nx * (double)i / (ni - 1), y = ny * (double)j / (nj - 1);
            surf.insert(surf.end(), {x, y, top(x, y)});
        }
    ddpca_curveds_t cs = nullptr;
    ok(ddpca_curveds_create(ni, nj, surf.data(), nullptr, &cs), "curveds_create");
    const int64_t *pptr = nullptr, *pnode = nullptr;
    const double* pxyz = nullptr;
    int64_t nplan = 0;
    if (cs) {
        const double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, tr[3] = {0, 0, 0};
        ok(ddpca_curveds_rigid(cs, R, tr), "curveds_rigid");
        ok(ddpca_curveds_plan(cs, g, (int64_t)elem.size(), elem.data(), &pptr, &pnode, &pxyz, &nplan), "curveds_plan");
    }
    std::vector<int64_t> pp(pptr ? pptr : nullptr, pptr ? pptr + nplan + 1 : nullptr);
    std::vector<int64_t> pn(pnode ? pnode : nullptr, pnode ? pnode + (nplan ? pp.back() : 0) : nullptr);
    std::vector<double> px(pxyz ? pxyz : nullptr, pxyz ? pxyz + 3 * nplan : nullptr);
    // refused first (the tree must stay as it was): reversed plan_ptr, spliFlag child 9
    if (nplan >= 2) {
        std::vector<int64_t> bad(pp);
        std::swap(bad[0], bad[1]);
        bad[0] = 0;
        bad[1] = pp[2] + 1;
        refused(ddpca_multigrid_refine(g, (int64_t)elem.size(), elem.data(), patt.data(), nplan, bad.data(), pn.data(),
                                       px.data(), 0, nullptr, nullptr),
                "refine reversed plan_ptr");
    }
    {
        const int64_t bfe = 0, bfc = 9;
        refused(ddpca_multigrid_refine(g, (int64_t)elem.size(), elem.data(), patt.data(), 0, nullptr, nullptr, nullptr, 1,
                                       &bfe, &bfc),
                "refine spliFlag child 9");
    }
    if ((int64_t)tree_get<int64_t>(g, "parent").size() != nelem) {
        std::fprintf(stderr, "FAIL refused refine changed the tree\n");
        ++g_fail;
    }
    ok(ddpca_multigrid_refine(g, (int64_t)elem.size(), elem.data(), patt.data(), nplan, pp.empty() ? nullptr : pp.data(),
                              pn.empty() ? nullptr : pn.data(), px.empty() ? nullptr : px.data(), (int64_t)fe.size(),
                              fe.data(), fc.data()),
       "refine round 1");
    // round 2: the children spliFlag selected, pattern 0 (GRLE_CHECK balances their neighbours)
    auto next = tree_get<int64_t>(g, "nextSplit");
    std::vector<int64_t> p0(next.size(), 0);
    if (!next.empty())
        ok(ddpca_multigrid_refine(g, (int64_t)next.size(), next.data(), p0.data(), 0, nullptr, nullptr, nullptr, 0,
                                  nullptr, nullptr),
           "refine round 2");
    if (cs) ddpca_curveds_destroy(cs);
    const auto coor = tree_get<double>(g, "nodeCoor");
    const size_t nel = tree_get<int64_t>(g, "parent").size();
    const int64_t nn = (int64_t)coor.size() / 3;
    // boundary data: x = 0 clamped, a load on x = nx, rotations on every 7th node, bad dofs refused
    std::vector<int64_t> cd, fi, rn;
    std::vector<double> cv, fv, rv;
    for (int64_t i = 0; i < nn; ++i) {
        if (coor[3 * i] == 0.0)
            for (int a = 0; a < 3; ++a) cd.push_back(3 * i + a), cv.push_back(0.0);
        if (coor[3 * i] == (double)nx) fi.push_back(3 * i + 2), fv.push_back(-1.0);
        if (i % 7 == 3 && coor[3 * i] > 0.0) {
            const double c = std::cos(0.3), s = std::sin(0.3);
            rn.push_back(i);
            rv.insert(rv.end(), {c, -s, 0, s, c, 0, 0, 0, 1});
        }
    }
    ok(ddpca_multigrid_set(g, "consDofv", (int64_t)cd.size(), cd.data(), cv.data()), "set consDofv");
    ok(ddpca_multigrid_set(g, "exteForc", (int64_t)fi.size(), fi.data(), fv.data()), "set exteForc");
    ok(ddpca_multigrid_set(g, "nodeRota", (int64_t)rn.size(), rn.data(), rv.data()), "set nodeRota");
    const double mat[2] = {2.1e11, 0.3};
    ok(ddpca_multigrid_set(g, "material", 2, nullptr, mat), "set material");
    for (int64_t bad : {(int64_t)-1, (int64_t)-2, 3 * nn}) {
        const double v = 1.0;
        refused(ddpca_multigrid_set(g, "consDofv", 1, &bad, &v), "set consDofv bad dof");
        refused(ddpca_multigrid_set(g, "exteForc", 1, &bad, &v), "set exteForc bad dof");
    }
    ok(ddpca_multigrid_build(g, nullptr), "multigrid_build");
    double s = 0.0;
    for (const char* w : {"posiNode", "nodeCoor", "leveCount", "freeCount", "consFlag", "consForc", "dispForc"}) {
        const void* d = nullptr;
        int64_t n = 0;
        int dt = 0;
        ok(ddpca_multigrid_view(g, w, 0, &d, &n, &dt), w);
        s += d ? fold(d, n, dt) : 0.0;
    }
    // as subdomain 0 of a one-subdomain problem (the builder's general-tree path)
    ddpca_problem_t p = nullptr;
    ok(ddpca_problem_empty(1, 0, &p), "problem_empty");
    if (p) {
        ok(ddpca_problem_set_subdomain_multigrid(p, 0, g), "set_subdomain_multigrid");
        refused(ddpca_problem_set_subdomain_multigrid(p, 1, g), "set_subdomain_multigrid tv 1");
        ok(ddpca_problem_finalize(p), "finalize");
        std::vector<uint8_t> owned{1};
        s += read_all(p, 0, false, owned);
        ddpca_problem_destroy(p);
    }
    std::printf("{\"case\": \"octree\", \"nodes\": %ld, \"elements\": %zu, \"planSurf\": %ld, \"checksum\": %.6e}\n", (long)nn, nel,
                (long)nplan, s);
    ddpca_multigrid_destroy(g);
}

// ---- CSEARCH on two facing, non-matching, slightly curved surfaces
void run_csearch() {
    // master: 6 x 6 quads on z = 0; slave: 9 x 9 quads on z = 1e-3 + small bump, offset in x/y
    auto grid = [](int n, double off, double z0, double bump, std::vector<double>& xyz, std::vector<int64_t>& segm,
                   std::vector<double>& uv) {
        for (int j = 0; j <= n; ++j)
            for (int i = 0; i <= n; ++i) {
                const double x = off + (double)i / n, y = off + (double)j / n;
                xyz.insert(xyz.end(), {x, y, z0 + bump * std::sin(3.0 * x) * std::sin(2.0 * y)});
            }
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                const int64_t a = i + (n + 1) * j;
                segm.insert(segm.end(), {a, a + 1, a + n + 2, a + n + 1});
                uv.insert(uv.end(), {(double)i, (double)j, (double)i + 1, (double)j, (double)i + 1, (double)j + 1,
                                     (double)i, (double)j + 1});
            }
    };
    std::vector<double> mx, sx, mu, su;
    std::vector<int64_t> ms, ss;
    grid(6, 0.0, 0.0, 0.0, mx, ms, mu);
    grid(9, 0.05, 1.0e-3, 2.0e-4, sx, ss, su);
    const int64_t nm = (int64_t)ms.size() / 4, ns = (int64_t)ss.size() / 4;
    const int64_t buck[3] = {4, 4, 1};
    ddpca_ips_t ips = nullptr;
    ok(ddpca_contact_search(mx.data(), (int64_t)mx.size() / 3, sx.data(), (int64_t)sx.size() / 3, nm, ms.data(), mu.data(),
                            ns, ss.data(), su.data(), buck, 0.1, &ips),
       "contact_search");
    int64_t nip = 0;
    double s = 0.0;
    if (ips) {
        nip = ddpca_ips_count(ips);
        std::vector<int64_t> node(8 * nip);
        std::vector<double> shap(8 * nip), basis(9 * nip), gap(nip), w(nip);
        ok(ddpca_ips_get(ips, node.data(), shap.data(), basis.data(), gap.data(), w.data()), "ips_get");
        s = fold(node.data(), 8 * nip, 1) + fold(shap.data(), 8 * nip, 0) + fold(basis.data(), 9 * nip, 0) +
            fold(gap.data(), nip, 0) + fold(w.data(), nip, 0);
        ddpca_ips_destroy(ips);
    }
    // ADAPTIVE_REFINE's selection: the "elements" are the faces' nodes repeated as hexes
    std::vector<int64_t> me, se;
    for (int64_t f = 0; f < nm; ++f)
        for (int k = 0; k < 8; ++k) me.push_back(ms[4 * f + k % 4]);
    for (int64_t f = 0; f < ns; ++f)
        for (int k = 0; k < 8; ++k) se.push_back(ss[4 * f + k % 4]);
    std::vector<uint8_t> msp(nm), ssp(ns);
    const int sel = ddpca_refine_select(mx.data(), (int64_t)mx.size() / 3, sx.data(), (int64_t)sx.size() / 3, nm, ms.data(),
                                        mu.data(), ns, ss.data(), su.data(), buck, 0.05, nm, me.data(), ns, se.data(),
                                        msp.data(), ssp.data());
    ok(sel, "refine_select");
    std::printf("{\"case\": \"csearch\", \"ips\": %ld, \"selected\": %d, \"checksum\": %.6e}\n", (long)nip, sel, s);
}

void run_writers() {
    const char* dir = std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp";
    const std::string a = std::string(dir) + "/san_resuDisp.txt", b = std::string(dir) + "/san_resuCont.txt",
                      c = std::string(dir) + "/san_resuMoni.txt";
    std::vector<double> disp(3 * 50), gamma(3 * 20), basis(9 * 20), rows(7 * 12);
    std::vector<int32_t> stat(20);
    for (size_t i = 0; i < disp.size(); ++i) disp[i] = std::sin((double)i);
    for (size_t i = 0; i < gamma.size(); ++i) gamma[i] = std::cos((double)i);
    for (size_t i = 0; i < basis.size(); ++i) basis[i] = (double)(i % 9 == 0 || i % 9 == 4 || i % 9 == 8);
    for (size_t i = 0; i < stat.size(); ++i) stat[i] = (int32_t)(i % 3);
    for (size_t i = 0; i < rows.size(); ++i) rows[i] = 1.0 / (1.0 + (double)i);
    const int64_t rn[2] = {3, 17};
    std::vector<double> rot(18, 0.0);
    for (int k = 0; k < 2; ++k) rot[9 * k] = rot[9 * k + 4] = rot[9 * k + 8] = 1.0;
    ok(ddpca_write_resuDisp(a.c_str(), disp.data(), 50, 2, rn, rot.data()), "write_resuDisp");
    ok(ddpca_write_resuCont(b.c_str(), 0.0, 20, gamma.data(), stat.data(), basis.data()), "write_resuCont f0");
    ok(ddpca_write_resuCont(b.c_str(), 0.3, 20, gamma.data(), stat.data(), basis.data()), "write_resuCont f3");
    ok(ddpca_write_resuMoni(c.c_str(), rows.data(), 12, 7), "write_resuMoni");
    std::printf("{\"case\": \"writers\"}\n");
}

}  // namespace

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);  // the case lines before any sanitizer report
    const bool quick = argc > 1 && std::strcmp(argv[1], "quick") == 0;
    std::vector<Case> cases = {
        {"beam", {8, 2, 2, 1, 1, 1, 1}, 0, 1},        // beam_s1
        {"beam", {8, 2, 2, 2, 1, 1, 1}, 0, 1},        // beam_s2
        {"beam", {8, 2, 2, 1, 2, 1, 1}, 0, 1},        // beam_dd
        {"beam", {4, 2, 2, 2, 2, 1, 1}, 2, 1},        // beam_dd_m2
        {"beam", {4, 2, 2, 2, 2, 1, 1}, 2, 2},        // ... rank-local on 2 ranks
        {"twoblock", {0.0, 2}, 0, 1},                 // twoblock_f0
        {"twoblock", {0.3, 2}, 0, 1},                 // twoblock_f3
        {"twoblock", {0.0, 2}, 2, 1},                 // twoblock_f0_m2
        {"twoblock", {0.3, 2}, 1, 1},                 // twoblock_f3_m1
        {"twoblock", {0.3, 2}, 1, 2},                 // ... rank-local on 2 ranks
        {"dehw", {2, 2, 2, 1, 2, 0.3}, 2, 1},         // the synthetic chain, 4 subdomains
        {"dehw", {2, 2, 2, 1, 2, 0.3}, 2, 4},         // ... one subdomain per rank
        {"dehw", {2, 2, 2, 1, 2, 0.3}, 1, 2},         // LATIN coarse space, 2 ranks
        {"dehw", {4, 3, 2, 2, 2, 0.2, 2, 1}, 2, 1},   // the headline workload's shape at gl 2
    };
    if (quick) cases.resize(3);
    for (const auto& c : cases) run_case(c);
    // refused generator arguments
    {
        ddpca_problem_t p = nullptr;
        const double bad[7] = {7, 2, 2, 1, 2, 1, 1};
        refused(ddpca_problem_create("beam", bad, 7, &p), "beam 7 elements on 2 subdomains");
        refused(ddpca_problem_create("beam", bad, 3, &p), "beam 3 params");
        refused(ddpca_problem_create("no_such_kind", bad, 7, &p), "unknown kind");
    }
    run_octree();
    run_csearch();
    run_writers();
    std::printf("{\"ok\": %s, \"failures\": %d}\n", g_fail ? "false" : "true", g_fail);
    return g_fail ? 1 : 0;
}

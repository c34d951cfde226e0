// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// ADAPTIVE_REFINE's selection against the reference: the reference builds its CYLINDER example
// (CYLINDER_1.h: curved cylinder surfaces, locally refined contact bands) and runs its own
// CSEARCH::ADAPTIVE_REFINE (CSEARCH.h:839-956) on the first curved contact pair, at the finest
// leaf level and the given distCrit; the leaf elements of that level that the reference then has
// refined (they gained children) are compared with the elements libddpca_amd's
// ddpca_refine_select flags on the same faces, coordinates and buckets.  CPU only.  One JSON line.
//   ref_refine distCrit [locaLeve]
#include <unistd.h>

#include <cstdio>

#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"

int main(int argc, char** argv) {
    const double distCrit = argc > 1 ? std::atof(argv[1]) : 1.0e-5;
    const long locaLeve = argc > 2 ? std::atol(argv[2]) : 4;
    const int saved = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;
    CYLINDER_1 c;
    c.copyNumb = 1;
    c.locaLeve = locaLeve;
    c.globInho = 2;
    c.bandWidt = 2.0e-4;
    c.SOLVE(0);  // MESH, the contact searches, ESTABLISH
    const long ts = 0;
    MULTIGRID* g[2] = {&c.multGrid[c.contBody[ts][0]], &c.multGrid[c.contBody[ts][1]]};
    CURVEDS* surf[2] = {&c.cyliSurf[c.contBody[ts][0]], &c.cyliSurf[c.contBody[ts][1]]};
    // candidates: leaf elements of the finest leaf level of the pair, recorded before the refinement
    long lev = 0;
    for (int s = 0; s < 2; ++s)
        for (const auto& e : g[s]->elemVect)
            if (e.children.empty()) lev = std::max(lev, e.level);
    std::vector<long> cand[2];
    std::vector<int64_t> corner[2];
    for (int s = 0; s < 2; ++s)
        for (long i = 0; i < (long)g[s]->elemVect.size(); ++i) {
            const auto& e = g[s]->elemVect[i];
            if (!e.children.empty() || e.level != lev) continue;
            cand[s].push_back(i);
            for (int k = 0; k < 8; ++k) corner[s].push_back(e.cornNode[k]);
        }
    std::vector<double> xyz[2];
    for (int s = 0; s < 2; ++s) {
        long nmax = 0;
        for (const auto& nc : g[s]->nodeCoor) nmax = std::max(nmax, nc.first + 1);
        xyz[s].assign(3 * nmax, 0.0);
        for (const auto& nc : g[s]->nodeCoor)
            for (int a = 0; a < 3; ++a) xyz[s][3 * nc.first + a] = nc.second[a];
    }
    CSEARCH cs = c.searCont[ts];
    cs.mastSegm.clear();
    cs.slavSegm.clear();
    cs.intePoin.clear();
    bool isnoRefi = false;
    const std::vector<long> buck = {c.buckNumb[ts][0], c.buckNumb[ts][1]};
    cs.ADAPTIVE_REFINE(g[0], g[1], isnoRefi, surf[0], surf[1], lev, distCrit, buck, [](COOR p, double& xi, double& et) {
        xi += p[0];  // the example's 2-D bucket coordinates: x and z (CYLINDER_1.h:600-627)
        et += p[2];
    });
    std::fflush(stdout);
    dup2(saved, 1);
    // the same selection through the C ABI, on the faces the reference iterated
    const VECTOR2L* segs[2] = {&cs.mastSegm, &cs.slavSegm};
    std::vector<int64_t> seg[2];
    std::vector<double> c2[2];
    for (int s = 0; s < 2; ++s)
        for (const auto& f : *segs[s]) {
            double x = 0.0, z = 0.0;
            for (int k = 0; k < 4; ++k) {
                seg[s].push_back(f[k]);
                x += xyz[s][3 * f[k]];
                z += xyz[s][3 * f[k] + 2];
            }
            c2[s].push_back(x / 4.0);
            c2[s].push_back(z / 4.0);
        }
    const int64_t bk[2] = {buck[0], buck[1]};
    std::vector<uint8_t> flag[2] = {std::vector<uint8_t>(cand[0].size()), std::vector<uint8_t>(cand[1].size())};
    const int any = ddpca_refine_select(xyz[0].data(), (int64_t)xyz[0].size() / 3, xyz[1].data(), (int64_t)xyz[1].size() / 3,
                                        (int64_t)cs.mastSegm.size(), seg[0].data(), c2[0].data(), (int64_t)cs.slavSegm.size(),
                                        seg[1].data(), c2[1].data(), bk, distCrit, (int64_t)cand[0].size(), corner[0].data(),
                                        (int64_t)cand[1].size(), corner[1].data(), flag[0].data(), flag[1].data());
    ddpca_bind::check(std::min(any, 0));
    bool equal = (any == 1) == isnoRefi;
    long nref[2] = {0, 0}, nflag[2] = {0, 0};
    for (int s = 0; s < 2; ++s)
        for (size_t i = 0; i < cand[s].size(); ++i) {
            const bool refined = !g[s]->elemVect[cand[s][i]].children.empty();
            nref[s] += refined;
            nflag[s] += flag[s][i];
            equal = equal && refined == (flag[s][i] != 0);
        }
    std::fprintf(stderr,
                 "{\"equal\": %s, \"isnoRefi\": %s, \"level\": %ld, \"candidates\": [%zu, %zu], \"refined_ref\": [%ld, %ld], "
                 "\"flagged\": [%ld, %ld], \"faces\": [%zu, %zu]}\n",
                 equal ? "true" : "false", isnoRefi ? "true" : "false", lev, cand[0].size(), cand[1].size(), nref[0], nref[1],
                 nflag[0], nflag[1], cs.mastSegm.size(), cs.slavSegm.size());
    return equal ? 0 : 1;
}

// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Contact search against the reference: the reference's own CYLINDER example (CYLINDER_1.h,
// curved cylinder surfaces, locally refined contact bands, non-matching master / slave faces)
// builds its meshes and runs its CSEARCH (BUCKET_SORT + CONTACT_SEARCH) on every interface; the
// same faces, node coordinates, 2-D bucket coordinates (the example's face-centre x / z) and
// bucket counts then go through libddpca_amd's ddpca_contact_search, and the integration points
// are compared one by one (count, node ids exactly; shape values, basis, gap and weight to
// rounding).  One JSON line on stderr.  CPU only (no GPU call).
//   ref_csearch copyNumb locaLeve globInho bandWidt
#include <unistd.h>

#include <cstdio>

#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"

int main(int argc, char** argv) {
    const long copyNumb = argc > 1 ? std::atol(argv[1]) : 1;
    const long locaLeve = argc > 2 ? std::atol(argv[2]) : 4;
    const long globInho = argc > 3 ? std::atol(argv[3]) : 2;
    const double bandWidt = argc > 4 ? std::atof(argv[4]) : 2.0e-4;
    const int saved = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    CYLINDER_1 c;  // creates ./Cylinder/ for the reference's result files
    c.copyNumb = copyNumb;
    c.locaLeve = locaLeve;
    c.globInho = globInho;
    c.bandWidt = bandWidt;
    c.SOLVE(0);  // MESH, the contact searches, ESTABLISH (APPS is a no-op for the LATIN space)
    std::fflush(stdout);
    dup2(saved, 1);
    std::string out = "[";
    bool ok = true;
    const long nsearch = 3;  // the curved-surface searches (the rest are copies / glued links)
    for (long ts = 0; ts < nsearch; ++ts) {
        const CSEARCH& S = c.searCont[ts];
        const MULTIGRID* g[2] = {S.mastGrid, S.slavGrid};
        std::vector<double> xyz[2];
        for (int s = 0; s < 2; ++s) {
            long nmax = 0;
            for (const auto& nc : g[s]->nodeCoor) nmax = std::max(nmax, nc.first + 1);
            xyz[s].assign(3 * nmax, 0.0);
            for (const auto& nc : g[s]->nodeCoor)
                for (int a = 0; a < 3; ++a) xyz[s][3 * nc.first + a] = nc.second[a];
        }
        const VECTOR2L* segs[2] = {&S.mastSegm, &S.slavSegm};
        std::vector<int64_t> seg[2];
        std::vector<double> c2[2];
        for (int s = 0; s < 2; ++s)
            for (const auto& f : *segs[s]) {
                double x = 0.0, z = 0.0;  // the face centre's x and z: the example's bucket coordinates
                for (int k = 0; k < 4; ++k) {
                    seg[s].push_back(f[k]);
                    x += xyz[s][3 * f[k]];
                    z += xyz[s][3 * f[k] + 2];
                }
                c2[s].push_back(x / 4.0);
                c2[s].push_back(z / 4.0);
            }
        const int64_t buck[2] = {c.buckNumb[ts][0], c.buckNumb[ts][1]};
        ddpca_ips_t ips = nullptr;
        ddpca_bind::check(ddpca_contact_search(xyz[0].data(), (int64_t)xyz[0].size() / 3, xyz[1].data(),
                                               (int64_t)xyz[1].size() / 3, (int64_t)S.mastSegm.size(), seg[0].data(),
                                               c2[0].data(), (int64_t)S.slavSegm.size(), seg[1].data(), c2[1].data(),
                                               buck, 1.0e12, &ips));
        const int64_t n = ddpca_ips_count(ips);
        std::vector<int64_t> node(8 * n);
        std::vector<double> shap(8 * n), basis(9 * n), gap(n), w(n);
        ddpca_bind::check(ddpca_ips_get(ips, node.data(), shap.data(), basis.data(), gap.data(), w.data()));
        ddpca_ips_destroy(ips);
        const int64_t nref = (int64_t)S.intePoin.size();
        bool nodes_equal = n == nref;
        double dshap = 0.0, dbasis = 0.0, dgap = 0.0, dw = 0.0, wmax = 0.0, gmax = 0.0;
        for (int64_t q = 0; q < std::min(n, nref); ++q) {
            const INTEGRAL_POINT& p = S.intePoin[q];
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    nodes_equal &= node[8 * q + 4 * s + k] == p.node[s][k];
                    dshap = std::max(dshap, std::abs(shap[8 * q + 4 * s + k] - p.shapFunc[s][k]));
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) dbasis = std::max(dbasis, std::abs(basis[9 * q + 3 * a + b] - p.basiVect[a](b)));
            dgap = std::max(dgap, std::abs(gap[q] - p.initNgap));
            dw = std::max(dw, std::abs(w[q] - p.quadWeig));
            wmax = std::max(wmax, std::abs(p.quadWeig));
            gmax = std::max(gmax, std::abs(p.initNgap));
        }
        const double wrel = wmax > 0 ? dw / wmax : dw;
        const bool ok_ts = nodes_equal && dshap <= 1e-9 && dbasis <= 1e-9 && wrel <= 1e-9 && dgap <= 1e-12;
        ok = ok && ok_ts;
        char buf[400];
        std::snprintf(buf, sizeof(buf),
                      "%s{\"ts\": %ld, \"faces\": [%zu, %zu], \"ips\": %ld, \"ips_ref\": %ld, \"nodes_equal\": %s, "
                      "\"shap\": %.3g, \"basis\": %.3g, \"gap\": %.3g, \"gap_max\": %.3g, \"w_rel\": %.3g}",
                      ts ? ", " : "", ts, S.mastSegm.size(), S.slavSegm.size(), (long)n, (long)nref,
                      nodes_equal ? "true" : "false", dshap, dbasis, dgap, gmax, wrel);
        out += buf;
    }
    out += "]";
    std::fprintf(stderr, "{\"ok\": %s, \"interfaces\": %s}\n", ok ? "true" : "false", out.c_str());
    return ok ? 0 : 1;
}
